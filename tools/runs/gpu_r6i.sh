#!/bin/bash
# round 6: split-precision conv_head (Mconv6 + Mconv7 fused in split precision) -- tests, split
# bench A/B (HEAD_FUSE_SPLIT=0: the unfused split pair; HEAD_PERSIST=0: per-tile head grid),
# fp16 bench (unchanged kernels), split kernel trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "head or split or layers or body25" > $O/pytest_gpu.log 2>&1 || exit 1
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra-configs"
for r in 1 2; do
  timeout -k 10 200 $B --precision split > $O/split_def_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --precision split --dev HEAD_FUSE_SPLIT=0 > $O/split_unfused_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --precision split --dev HEAD_PERSIST=0 > $O/split_pertile_$r.log 2>&1 || exit 1
done
timeout -k 10 200 $B > $O/fp16.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split -o run -- \
  python bench.py --precision split --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/prof_split.log 2>&1 || exit 1
