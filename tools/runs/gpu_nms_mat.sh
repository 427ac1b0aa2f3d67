#!/bin/bash
# config 4: multi-source NMS on materialised part maps (NMS_MAT=3) vs the lazy 4-source walk
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-nms_mat} && mkdir -p $O || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "multiscale or nms" > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config multiscale --steps 10 --no-cpu-baseline > $O/b4_lazy_$r.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --config multiscale --steps 10 --no-cpu-baseline --dev NMS_MAT=3 > $O/b4_mat_$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --config multiscale --steps 5 --warmup 2 --no-cpu-baseline --dev NMS_MAT=3 > $O/prof.log 2>&1 || exit 1
