#!/bin/bash
# A/B of the NMS walk's cold-window skip (NMS_COLD=1, the default, vs 0): NMS / pipeline GPU tests,
# then config 5 and config 2 benches interleaved on one box, kernel statistics of both on config 5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-nms_cold} && mkdir -p $O || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "nms or pipeline or multiscale or upsampling or inject or extract" > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline > $O/b135_cold_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline --dev NMS_COLD=0 > $O/b135_full_$r.log 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/b25_cold_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev NMS_COLD=0 > $O/b25_full_$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cold -o run -- python bench.py --config body135 --steps 10 --no-cpu-baseline > $O/prof_cold.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_full -o run -- python bench.py --config body135 --steps 10 --no-cpu-baseline --dev NMS_COLD=0 > $O/prof_full.log 2>&1 || exit 1
