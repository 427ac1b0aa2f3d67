#!/bin/bash
# GPU: the given test files (default: all -m gpu tests), one pytest process, own time limit
#   gpu_tests.sh OUTDIR [pytest args...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; shift
mkdir -p $out
timeout -k 10 400 python -u -m pytest ${@:-tests} -m gpu -x -v -rA --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
