#!/bin/bash
# dev: one-strip epilogue positions (in-tree build vs variants/libopk_old.so) and the halo-early
# DMA schedule (CONV3W_HE / CONV3W8_HE): probe launches, net outputs bit for bit, bench interleaved
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && OUT=gpurun_out/${1:-he} && mkdir -p $OUT && OLD=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_old.so && {
for r in 1 2; do
  for c in "128 128" "96 96" "256 128" "384 128"; do
    for v in 0 2 1 3; do timeout -k 5 60 tools/conv3w_probe_ns 130 46 82 $c 50 1 0 $v || exit 1; done
  done
done ; } > $OUT/probe.log 2>&1 &&
OPK_LIB_PATH=$OLD timeout -k 10 200 python tools/ab_outputs.py $OUT/out_old.npy 130 > $OUT/outputs.log 2>&1 &&
timeout -k 10 200 python tools/ab_outputs.py $OUT/out_new.npy 130 >> $OUT/outputs.log 2>&1 &&
OPK_AB_DEV=CONV3W_HE=1,CONV3W8_HE=1 timeout -k 10 200 python tools/ab_outputs.py $OUT/out_he.npy 130 >> $OUT/outputs.log 2>&1 &&
python tools/ab_outputs.py --compare $OUT/out_old.npy $OUT/out_new.npy >> $OUT/outputs.log 2>&1 &&
python tools/ab_outputs.py --compare $OUT/out_new.npy $OUT/out_he.npy >> $OUT/outputs.log 2>&1 &&
rm -f $OUT/*.npy &&
for i in 1 2; do
  OPK_LIB_PATH=$OLD timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $OUT/bench_old_$i.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $OUT/bench_new_$i.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev CONV3W_HE=1 > $OUT/bench_he_$i.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev CONV3W_HE=1 --dev CONV3W8_HE=1 > $OUT/bench_he8_$i.log 2>&1 || exit 1
done
