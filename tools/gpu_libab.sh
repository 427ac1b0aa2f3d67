#!/bin/bash
# dev: in-tree build vs variants/libopk_old.so -- net outputs bit for bit, bench interleaved, and
# the kernel statistics of both
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && OUT=gpurun_out/${1:-libab} && mkdir -p $OUT && OLD=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_old.so &&
OPK_LIB_PATH=$OLD timeout -k 10 200 python tools/ab_outputs.py $OUT/out_old.npy 130 > $OUT/outputs.log 2>&1 &&
timeout -k 10 200 python tools/ab_outputs.py $OUT/out_new.npy 130 >> $OUT/outputs.log 2>&1 &&
python tools/ab_outputs.py --compare $OUT/out_old.npy $OUT/out_new.npy >> $OUT/outputs.log 2>&1 &&
rm -f $OUT/*.npy &&
for i in 1 2; do
  OPK_LIB_PATH=$OLD timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $OUT/bench_old_$i.log 2>&1 &&
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $OUT/bench_new_$i.log 2>&1 || exit 1
done &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_new -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_new.log 2>&1 &&
OPK_LIB_PATH=$OLD timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_old -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_old.log 2>&1
