#!/bin/bash
# dev: PAF line integrals with one sample per lane (PAF_SPL=1, default) vs one line per lane:
# bit-exactness tests, then config 5 / config 2 bench A/B and per-kernel statistics
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && OUT=gpurun_out/${1:-paf} && mkdir -p $OUT &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_postprocess.py tests/test_gpu_pipeline.py tests/test_connector_gpu.py > $OUT/pytest_paf.log 2>&1 &&
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python -u bench.py --config body135 --steps 20 --no-cpu-baseline --dev PAF_SPL=$v > $OUT/b135_spl${v}_$i.log 2>&1 &&
    timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev PAF_SPL=$v > $OUT/b25_spl${v}_$i.log 2>&1 || exit 1
  done
done &&
for v in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_b135_$v -o run -- python bench.py --config body135 --steps 10 --warmup 2 --no-cpu-baseline --dev PAF_SPL=$v > $OUT/prof_b135_$v.log 2>&1 || exit 1
done
