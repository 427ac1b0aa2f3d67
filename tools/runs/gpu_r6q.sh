#!/bin/bash
# round 6: the fp16 stage layers on conv3w8 (CONV3W8=2: 128-output layers, 3: also 96) against the
# 16-wave conv3w default -- fp16 bench interleaved x2, kernel trace of each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6q}
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra-configs"
for r in 1 2; do
  for v in 1 2 3; do
    timeout -k 10 200 $B --dev CONV3W8=$v > $O/fp16_w8_${v}_$r.log 2>&1 || exit 1
  done
done
for v in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$v -o run -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra-configs --dev CONV3W8=$v > $O/prof_$v.log 2>&1 || exit 1
done
