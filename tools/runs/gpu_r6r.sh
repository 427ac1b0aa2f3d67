#!/bin/bash
# round 6: the NMS walk's whole-footprint cold exit (NMS_COLD_EXIT) -- the post-processing tests,
# config 5 / config 2 benches A/B interleaved x2, kernel trace of config 5 both ways
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6r}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_postprocess.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
B5="python -u bench.py --config body135 --steps 30 --warmup 3 --no-cpu-baseline --no-extra-configs"
B2="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra-configs"
for r in 1 2; do
  for e in 1 0; do
    timeout -k 10 200 $B5 --dev NMS_COLD_EXIT=$e > $O/b135_exit${e}_$r.log 2>&1 || exit 1
  done
done
for e in 1 0; do
  timeout -k 10 200 $B2 --dev NMS_COLD_EXIT=$e > $O/b25_exit${e}.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b135_$e -o run -- \
    python bench.py --config body135 --steps 10 --warmup 2 --no-cpu-baseline --no-extra-configs --dev NMS_COLD_EXIT=$e > $O/prof_b135_$e.log 2>&1 || exit 1
done
