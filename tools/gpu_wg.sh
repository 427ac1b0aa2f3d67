#!/bin/bash
# dev: Winograd conv A/B -- net tests, then bench with and without CONV3WG, then a kernel trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-wg}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/pytest_net.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $out/bench_wg.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --dev CONV3WG=0 > $out/bench_direct.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $out/bench_wg2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1 || exit 1
