#!/bin/bash
# GPU round evidence in one call: parity tests, smoke, default bench, multi-scale bench, rocprofv3
# kernel stats, then the HBM traffic PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs)
#   OUT_TAG=<dir under gpurun_out>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT_TAG=${OUT_TAG:-r2} STEPS=tests,smoke,bench,multi,prof bash tools/gpu_round.sh || exit 1
bash tools/pmc_traffic.sh
