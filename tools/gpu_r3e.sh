#!/bin/bash
# round-3 evidence at HEAD: PMC passes (default bench, body135), kernel trace + layer report, bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/pmc_round.sh pmc_head_r3e || exit 1
bash tools/pmc_round.sh pmc_body135 --config body135 || exit 1
mkdir -p gpurun_out/r3e
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3e/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3e/prof.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r3e/bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config body135 > gpurun_out/r3e/bench_body135.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config multiscale --steps 10 > gpurun_out/r3e/bench_multiscale.log 2>&1 || exit 1
