#!/bin/bash
# dev: per-layer A/B (rocprofv3 kernel traces) of conv3 variants in one GPU call
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lab
P="--kernel-trace --output-format csv -o run"
B="python bench.py --steps 6 --warmup 3 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 $P -d gpurun_out/lab/base -- $B > gpurun_out/lab/base.log 2>&1
OPK_LIB_PATH=openpose_amd/variants/libopk_vaddr.so timeout -k 10 300 rocprofv3 $P -d gpurun_out/lab/vaddr -- $B > gpurun_out/lab/vaddr.log 2>&1
OPK_CONV3_PERSIST=0 timeout -k 10 300 rocprofv3 $P -d gpurun_out/lab/nopersist -- $B > gpurun_out/lab/nopersist.log 2>&1
