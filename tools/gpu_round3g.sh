#!/bin/bash
# GPU evidence at HEAD in one call: parity tests, smoke, default bench (tile-aligned batch),
# multi-scale + BODY_135 benches, rocprofv3 kernel trace/stats + layer report, PMC passes
#   gpu_round3g.sh OUTDIR [BATCH]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r3g}; B=${2:-130}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config multiscale --steps 20 --no-cpu-baseline > $OUT/bench_multiscale.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config body135 --steps 20 --no-cpu-baseline > $OUT/bench_body135.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
python tools/layer_report.py $OUT/prof/run_kernel_trace.csv $B > $OUT/layers.txt 2>&1
python tools/layer_report.py $OUT/prof/run_kernel_trace.csv $B --layers > $OUT/layers_detail.txt 2>&1
bash tools/pmc_round.sh ${1:-r3g}/pmc --batch $B
