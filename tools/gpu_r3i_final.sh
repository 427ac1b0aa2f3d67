#!/bin/bash
# round-3 HEAD evidence in one call: GPU suite, smoke, default bench (with the CPU baseline),
# multi-scale and BODY_135 benches, kernel statistics of the default bench, PMC summaries
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r3i}
mkdir -p $OUT
OUT_TAG=${1:-r3i} STEPS=tests,smoke,bench,multi,prof bash tools/gpu_round.sh || exit 1
timeout -k 10 300 python -u bench.py --config body135 > $OUT/bench_body135.log 2>&1 || exit 1
bash tools/pmc_round.sh ${1:-r3i}/pmc || exit 1
bash tools/pmc_round.sh ${1:-r3i}/pmc_body135 --config body135 --batch 64 || exit 1
