#!/bin/bash
# dev: the alternating net-output buffers (NET_OUT_ALT) -- pipeline GPU tests, then the bench with
# and without them interleaved (configs 2 and 4), and a kernel trace of each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && OUT=gpurun_out/${1:-outalt} && mkdir -p $OUT &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pipeline.py tests/test_gpu_sharded.py tests/test_pose_shim.py > $OUT/pytest.log 2>&1 &&
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python -u bench.py --steps 30 --no-cpu-baseline --dev NET_OUT_ALT=$v > $OUT/bench_alt${v}_$i.log 2>&1 || exit 1
  done
done &&
for v in 0 1; do
  timeout -k 10 200 python -u bench.py --config multiscale --steps 15 --no-cpu-baseline --dev NET_OUT_ALT=$v > $OUT/ms_alt${v}.log 2>&1 || exit 1
done &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_alt1 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_alt1.log 2>&1
