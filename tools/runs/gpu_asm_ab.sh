#!/bin/bash
# A/B of a host-side change (this tree vs openpose_amd/variants/libopk_asmold.so, built from the
# previous commit): connector / pipeline GPU tests, the sharded-records tests, then config 5 and
# config 2 benches interleaved on one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-asm_ab} && mkdir -p $O || exit 1
V=$PWD/openpose_amd/variants/libopk_asmold.so
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "connector or pipeline or inject or sharded or pose or semantics" > $O/pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline > $O/b135_new_$r.log 2>&1 || exit 1
  OPK_LIB_PATH=$V timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline > $O/b135_old_$r.log 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/b25_new.log 2>&1 || exit 1
OPK_LIB_PATH=$V timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/b25_old.log 2>&1 || exit 1
