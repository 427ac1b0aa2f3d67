#!/bin/bash
# round 6: strip width A/B (CONV3_STRIP caps it) in split precision -- kernel traces of the split
# bench at the default (82-column strips at full resolution) and capped widths
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6j}
mkdir -p $O
for sw in 0 56 40 28; do
  D=""; [ $sw != 0 ] && D="--dev CONV3_STRIP=$sw"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$sw -o run -- \
    python bench.py --precision split --steps 3 --warmup 1 --no-cpu-baseline --no-extra-configs $D > $O/split_$sw.log 2>&1 || exit 1
done
