#!/bin/bash
# GPU round evidence: parity tests, smoke, default bench, multi-scale and BODY_135 benches,
# rocprofv3 kernel stats of the default bench
#   OUT_TAG=<dir under gpurun_out>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT_TAG:-r2}
OUT_TAG=${OUT_TAG:-r2} STEPS=tests,smoke,bench,multi,prof bash tools/gpu_round.sh || exit 1
timeout -k 10 300 python -u bench.py --config body135 --steps 10 > $OUT/bench_body135.log 2>&1
