#!/bin/bash
# round 6, last: the sharded-bench GPU tests and a short bench after the runtime's queue addition
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6y}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-extra-configs --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
