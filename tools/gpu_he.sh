#!/bin/bash
# dev: halo-early DMA schedule A/B -- probe launches (conv3w v0/v2, conv3w8 v1/v3, bit-checked
# against conv3w), net outputs bit for bit, bench interleaved (base / HE on conv3w / on both)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && OUT=gpurun_out/${1:-he} && mkdir -p $OUT && {
for r in 1 2; do
  for c in "128 128" "96 96" "256 128" "384 128"; do
    for v in 0 2 1 3; do timeout -k 5 60 tools/conv3w_probe_ns 130 46 82 $c 50 1 0 $v || exit 1; done
  done
done ; } > $OUT/probe.log 2>&1 &&
timeout -k 10 200 python tools/ab_outputs.py $OUT/out_base.npy 130 > $OUT/outputs.log 2>&1 &&
OPK_AB_DEV=CONV3W_HE=1,CONV3W8_HE=1 timeout -k 10 200 python tools/ab_outputs.py $OUT/out_he.npy 130 >> $OUT/outputs.log 2>&1 &&
python tools/ab_outputs.py --compare $OUT/out_base.npy $OUT/out_he.npy >> $OUT/outputs.log 2>&1 &&
rm -f $OUT/*.npy &&
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $OUT/bench_base_$i.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev CONV3W_HE=1 > $OUT/bench_he_$i.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev CONV3W_HE=1 --dev CONV3W8_HE=1 > $OUT/bench_he8_$i.log 2>&1 || exit 1
done
