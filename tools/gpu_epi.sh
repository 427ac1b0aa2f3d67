#!/bin/bash
# dev: epilogue max-activation + single-strip halo rows A/B -- net tests, benches, kernel trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-epi}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/pytest_net.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $out/bench_max.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --dev EPI_MAX=0 > $out/bench_sel.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --dev CONV3W8=2 > $out/bench_w8all.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $out/bench_max2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_w8 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dev CONV3W8=2 > $out/prof_w8.log 2>&1 || exit 1
