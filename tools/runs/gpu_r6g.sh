#!/bin/bash
# round 6: conv1_2 + pool1 on conv3w8's 64-channel pooled epilogue (split precision) -- tests, split
# bench A/B (POOL_FUSE=0; the 1x1 head tiles CONV1_TILE=1 / 0), kernel trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6g}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
  -k "split or pool or tile_variants or layers or conv1" > $O/pytest_gpu.log 2>&1 || exit 1
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra-configs --precision split"
for r in 1 2; do
  timeout -k 10 200 $B > $O/split_def_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --dev POOL_FUSE=0 > $O/split_nopool_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --dev CONV1_TILE=1 > $O/split_t1_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --dev CONV1_TILE=0 > $O/split_t0_$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split -o run -- \
  python bench.py --precision split --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/prof_split.log 2>&1 || exit 1
