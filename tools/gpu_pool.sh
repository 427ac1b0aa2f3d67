#!/bin/bash
# dev: pool-fusion check -- net tests, bench with and without POOL_FUSE, kernel trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-pool}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/pytest_net.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $out/bench_fused.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --dev POOL_FUSE=0 > $out/bench_sep.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $out/bench_fused2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/two_stream.py --streams 1 2 1 2 --grid-cus 128 --batch 64 > $out/two_stream_half_grid.log 2>&1 || exit 1
