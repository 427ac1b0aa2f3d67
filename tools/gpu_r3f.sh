#!/bin/bash
# round-3 evidence at HEAD: GPU tests, smoke, benches (default with CPU baseline, multi-scale,
# BODY_135), kernel trace, PMC passes
#   gpu_r3f.sh TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
t=${1:-r3f}
out=gpurun_out/$t
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -rA --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $out/bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config multiscale --steps 10 > $out/bench_multiscale.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config body135 > $out/bench_body135.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1 || exit 1
bash tools/pmc_round.sh pmc_head_$t || exit 1
