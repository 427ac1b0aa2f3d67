#!/bin/bash
# round 6: split conv_head with separate A / B slot rings (x_hi w_lo, x_hi w_hi, x_lo w_hi: the second
# reuses the staged A tile, the third the staged weights) -- head / split tests, split bench against
# the previous head (openpose_amd/ab/libopk_hold.so) x2, traces
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6u}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "head or split_every or split_launch or body25_split or large_batch" > $O/pytest_gpu.log 2>&1 || exit 1
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra-configs --precision split"
for r in 1 2; do
  for v in new hold; do
    unset OPK_LIB_PATH
    [ $v = hold ] && export OPK_LIB_PATH=$GRAFT_REPO_ROOT/openpose_amd/ab/libopk_hold.so
    timeout -k 10 200 $B > $O/split_${v}_$r.log 2>&1 || exit 1
  done
done
for v in new hold; do
  unset OPK_LIB_PATH
  [ $v = hold ] && export OPK_LIB_PATH=$GRAFT_REPO_ROOT/openpose_amd/ab/libopk_hold.so
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$v -o run -- \
    python bench.py --precision split --steps 3 --warmup 1 --no-cpu-baseline --no-extra-configs > $O/prof_$v.log 2>&1 || exit 1
done
