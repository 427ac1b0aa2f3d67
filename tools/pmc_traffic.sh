#!/bin/bash
# HBM traffic of the bench's kernels: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/traffic
B="python bench.py --steps 4 --warmup 1 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/traffic/fetch -o run -- $B > gpurun_out/traffic/fetch.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/traffic/write -o run -- $B > gpurun_out/traffic/write.log 2>&1
