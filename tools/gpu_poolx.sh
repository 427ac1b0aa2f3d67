#!/bin/bash
# dev: pool epilogue exchange through LDS (in-tree) vs the global round trip (variants/libopk_old.so):
# per-layer parity + fault variant, net outputs bit for bit, bench interleaved, kernel statistics
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && OUT=gpurun_out/${1:-poolx} && mkdir -p $OUT && OLD=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_old.so &&
PYT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread" &&
timeout -k 10 400 $PYT -m gpu tests/test_gpu_layers.py > $OUT/pytest_layers.log 2>&1 &&
{ OPK_LIB_PATH=openpose_amd/variants/libopk_faultpool.so timeout -k 10 300 $PYT -m gpu tests/test_gpu_layers.py > $OUT/pytest_fault_variant.log 2>&1; rc=$?; echo "exit $rc (1 = test failed as expected)" >> $OUT/pytest_fault_variant.log; [ $rc -lt 2 ]; } &&
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
