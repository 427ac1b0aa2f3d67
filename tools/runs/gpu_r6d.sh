#!/bin/bash
# round 6: A/B of the NMS cold-window jump + PAF early exit (the product build) against a variant
# build without both (-DOPK_NMS_JUMP=0 -DOPK_PAF_EXIT=0, openpose_amd/ab/libopk_nojump.so):
# config 5 and config 2 benches interleaved, config-5 kernel statistics of both
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6d}
mkdir -p $O
V=$GRAFT_REPO_ROOT/openpose_amd/ab/libopk_nojump.so
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config body135 --steps 50 --no-cpu-baseline > $O/b135_new_$r.log 2>&1 || exit 1
  OPK_LIB_PATH=$V timeout -k 10 200 python -u bench.py --config body135 --steps 50 --no-cpu-baseline > $O/b135_old_$r.log 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --no-extra-configs > $O/b25_new_$r.log 2>&1 || exit 1
  OPK_LIB_PATH=$V timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --no-extra-configs > $O/b25_old_$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o run -- python bench.py --config body135 --steps 20 --no-cpu-baseline > $O/prof_new.log 2>&1 || exit 1
OPK_LIB_PATH=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_old -o run -- python bench.py --config body135 --steps 20 --no-cpu-baseline > $O/prof_old.log 2>&1 || exit 1
PMC_COMMIT=$(cat .pmc_commit 2>/dev/null) bash tools/pmc_round.sh r6d/pmc_split --precision split > $O/pmc_split.log 2>&1 || exit 1
