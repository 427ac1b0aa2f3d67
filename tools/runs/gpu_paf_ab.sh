#!/bin/bash
# A/B of the PAF line-integral kernel (interleaved x/y planes in LDS vs separate planes, the
# variant build openpose_amd/variants/libopk_pafold.so): GPU tests of the post-processing, then
# BODY_135 (config 5) and config 2 benches interleaved, one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-paf_ab} && mkdir -p $O || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "paf or pipeline or connector or inject or body135 or semantics" > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline > $O/b135_new_$r.log 2>&1 || exit 1
  OPK_LIB_PATH=$PWD/openpose_amd/variants/libopk_pafold.so timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline > $O/b135_old_$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o run -- python bench.py --config body135 --steps 10 --no-cpu-baseline > $O/prof_new.log 2>&1 || exit 1
