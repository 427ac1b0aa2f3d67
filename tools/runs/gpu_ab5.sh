#!/bin/bash
# dev (round 5): the in-tree build ("new") against variant builds openpose_amd/variants/libopk_<v>.so
# in one GPU call -- net outputs bit for bit, per-layer + net GPU tests on the new build, the bench
# interleaved (2 reps), and rocprofv3 kernel statistics of every build
#   OUT=<dir under gpurun_out> bash tools/runs/gpu_ab5.sh <variant> [<variant> ...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-ab5} && mkdir -p $O || exit 1
V=$GRAFT_REPO_ROOT/openpose_amd/variants
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_net.py > $O/pytest_layers.log 2>&1 || exit 1
timeout -k 10 200 python tools/ab_outputs.py $O/out_new.npy 130 > $O/outputs.log 2>&1 || exit 1
for v in "$@"; do
  OPK_LIB_PATH=$V/libopk_$v.so timeout -k 10 200 python tools/ab_outputs.py $O/out_$v.npy 130 >> $O/outputs.log 2>&1 &&
  python tools/ab_outputs.py --compare $O/out_new.npy $O/out_$v.npy >> $O/outputs.log 2>&1 || exit 1
done
rm -f $O/*.npy
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/bench_new_$i.log 2>&1 || exit 1
  for v in "$@"; do
    OPK_LIB_PATH=$V/libopk_$v.so timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/bench_${v}_$i.log 2>&1 || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_new.log 2>&1 || exit 1
for v in "$@"; do
  OPK_LIB_PATH=$V/libopk_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_$v.log 2>&1 || exit 1
done
