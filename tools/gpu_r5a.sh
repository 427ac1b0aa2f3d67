#!/bin/bash
# round 5, first GPU call: the new ordering / RCCL / parity tests, then the whole GPU suite and
# the default bench (parity block + CPU baseline)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT_TAG:-r5a}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_preprocess.py::test_gpu_pose_direct_forward_between_submit_and_collect" \
  "tests/test_gpu_sharded.py::test_rccl_gather_one_rank" \
  "tests/test_gpu_pipeline.py::test_end_to_end_unscaled_heads" > $OUT/pytest_new.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || exit 1
