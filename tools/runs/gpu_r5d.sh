#!/bin/bash
# round 5: split precision at a large batch (frame runs), its cost, and the default bench with the
# parity block in both precisions
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-r5d} && mkdir -p $O || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_net.py::test_split_precision_large_batch_frame_runs" \
  "tests/test_gpu_net.py::test_body25_split_precision_vs_oracle" > $O/pytest_split.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/precision_bench.py 130 > $O/precision_bench.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 || exit 1
