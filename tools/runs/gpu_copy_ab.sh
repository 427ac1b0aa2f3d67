#!/bin/bash
# A/B of the collect's copy sizes (and the 3-pass connection sort) against a variant build of the
# previous commit: GPU tests of the pipeline, then config 2 and config 5 benches interleaved,
# and the kernel trace of config 2 with the new copies
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-copy_ab} && mkdir -p $O || exit 1
V=$PWD/openpose_amd/variants/libopk_prevcopy.so
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "connector or pipeline or inject or sharded or pose or semantics or collect" > $O/pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/b25_new_$r.log 2>&1 || exit 1
  OPK_LIB_PATH=$V timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/b25_old_$r.log 2>&1 || exit 1
done
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline > $O/b135_new_$r.log 2>&1 || exit 1
  OPK_LIB_PATH=$V timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline > $O/b135_old_$r.log 2>&1 || exit 1
done
# the HIP runtime's blit-copy controls (environment, read at HIP init), config 2
GPU_BLIT_ENGINE_TYPE=2 timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/b25_blit2.log 2>&1 || exit 1
DEBUG_CLR_LIMIT_BLIT_WG=16 timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/b25_blitwg16.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
