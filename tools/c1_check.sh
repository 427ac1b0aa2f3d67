#!/bin/bash
# dev: conv tests, then the conv1_fused kernel time in a short profiled bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c1b && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c1b/t.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c1b/p -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/c1b/b.log 2>&1
