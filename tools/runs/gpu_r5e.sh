#!/bin/bash
# round-5 evidence at HEAD: every GPU test, smoke, the default / multi-scale / BODY_135 benches,
# rocprofv3 kernel stats of the default bench, then the PMC passes (default bench and BODY_135)
#   OUT_TAG=<dir under gpurun_out>  PMC_COMMIT=<commit of the tree>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${OUT_TAG:-r5e}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
OUT_TAG=$T STEPS=smoke,bench,multi,prof bash tools/runs/gpu_round.sh || exit 1
timeout -k 10 300 python -u bench.py --config body135 --steps 10 > $OUT/bench_body135.log 2>&1 || exit 1
bash tools/pmc_round.sh $T/pmc || exit 1
bash tools/pmc_round.sh $T/pmc_body135 --config body135 --batch 64 || exit 1
