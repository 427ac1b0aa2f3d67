#!/bin/bash
# round 5: split precision -- its GPU tests, the fp16 net / layer tests, the two precisions timed
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-r5c} && mkdir -p $O || exit 1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_net.py \
  "tests/test_gpu_pipeline.py::test_end_to_end_unscaled_heads" \
  "tests/test_gpu_pipeline.py::test_end_to_end_unscaled_heads_split_precision" > $O/pytest_split.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/precision_bench.py 130 > $O/precision_bench.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_layers.py > $O/pytest_layers.log 2>&1 || exit 1
