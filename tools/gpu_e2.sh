#!/bin/bash
# dev: E2 tile transition A/B -- probe timeline + event-timed launches, net outputs bit for bit,
# bench interleaved (base / E2 on conv3w / E2 on conv3w and conv3w8)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && OUT=gpurun_out/${1:-e2} && mkdir -p $OUT &&
bash tools/probe_r4.sh r4 && cp gpurun_out/probe/r4.log $OUT/probe.log &&
timeout -k 10 200 python tools/ab_outputs.py $OUT/out_base.npy 130 > $OUT/outputs.log 2>&1 &&
OPK_AB_DEV=CONV3W_E2=1,CONV3W8_E2=1 timeout -k 10 200 python tools/ab_outputs.py $OUT/out_e2.npy 130 >> $OUT/outputs.log 2>&1 &&
python tools/ab_outputs.py --compare $OUT/out_base.npy $OUT/out_e2.npy >> $OUT/outputs.log 2>&1 &&
rm -f $OUT/*.npy &&
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $OUT/bench_base_$i.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev CONV3W_E2=1 > $OUT/bench_e2_$i.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev CONV3W_E2=1 --dev CONV3W8_E2=1 > $OUT/bench_e28_$i.log 2>&1 || exit 1
done
