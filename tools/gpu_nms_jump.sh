#!/bin/bash
# A/B of the NMS walk's window jump (this tree vs openpose_amd/variants/libopk_nmsprev.so, the
# previous walk): NMS tests, config 5 / config 2 benches interleaved, config-5 kernel statistics
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-nms_jump} && mkdir -p $O || exit 1
V=$PWD/openpose_amd/variants/libopk_nmsprev.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "nms or pipeline or multiscale or upsampling or inject or extract or connector or paf or semantics or pose" > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline > $O/b135_new_$r.log 2>&1 || exit 1
  OPK_LIB_PATH=$V timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline > $O/b135_prev_$r.log 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/b25_new.log 2>&1 || exit 1
OPK_LIB_PATH=$V timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/b25_prev.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o run -- python bench.py --config body135 --steps 10 --no-cpu-baseline > $O/prof_new.log 2>&1 || exit 1
OPK_LIB_PATH=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_prev -o run -- python bench.py --config body135 --steps 10 --no-cpu-baseline > $O/prof_prev.log 2>&1 || exit 1
