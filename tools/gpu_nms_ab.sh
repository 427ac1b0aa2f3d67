#!/bin/bash
# dev (round 5): NMS walk, one vs two maps per wave (NMS_MAPS) -- the NMS / pipeline GPU tests,
# configs 5 and 2 interleaved, kernel statistics of config 5 under both
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-nms_ab} && mkdir -p $O || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_postprocess.py tests/test_semantics.py > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do
  for m in 1 2; do
    timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline --dev NMS_MAPS=$m > $O/b135_m${m}_$i.log 2>&1 || exit 1
    timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev NMS_MAPS=$m > $O/b25_m${m}_$i.log 2>&1 || exit 1
  done
done
for m in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b135_m$m -o run -- python bench.py --config body135 --steps 10 --no-cpu-baseline --dev NMS_MAPS=$m > $O/prof_b135_m$m.log 2>&1 || exit 1
done
