#!/bin/bash
# dev: conv3w8 (8 waves of 64 x BN) against conv3w (16 waves of 64 x 64) on the short-K stage
# layers at the bench batch: probe launches (event-timed) and bench A/B (CONV3W8=3: conv3w8 for
# every single-n-block 3x3 layer)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && OUT=gpurun_out/${1:-w8} && mkdir -p $OUT && {
for r in 1 2; do
  for c in "128 128" "96 96" "256 128"; do
    for v in 0 1; do timeout -k 5 60 tools/conv3w_probe_ns 130 46 82 $c 50 1 0 $v || exit 1; done
  done
done ; } > $OUT/probe.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $OUT/bench_base_$i.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev CONV3W8=3 > $OUT/bench_w8_$i.log 2>&1 || exit 1
done
