#!/bin/bash
# dev: conv3t (tall waves, register-shifted halo fragments) -- net tests incl. the bit-identical
# variant test, interleaved bench A/B against the default kernels, a kernel trace of each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-tall}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/pytest_net.log 2>&1 || exit 1
for rep in 1 2; do
  for v in base CONV3T=1 CONV3T=2; do
    args=""; [ "$v" != base ] && args="--dev $v"
    timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $out/bench_${v}_$rep.log 2>&1 || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_base -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof_base.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_tall -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dev CONV3T=2 > $out/prof_tall.log 2>&1 || exit 1
