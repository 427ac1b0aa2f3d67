#!/bin/bash
# dev: conv3w8 single-strip variant (scalar-descriptor halo DMA issued a unit earlier) A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-s1}
mkdir -p $out
true || timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/pytest_net.log 2>&1 || exit 1
for v in "" "S1W8=0" "HALO_EARLY=0" "CONV3W8=2" "CONV3W8=2 S1W8=0" "CONV3W8=2 HALO_EARLY=0" "S1W8=0" "HALO_EARLY=0" ""; do
  tag=$(echo "${v:-default}" | tr ' =' '_-')_$((++k))
  args=""; for kv in $v; do args="$args --dev $kv"; done
  timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $out/bench_$tag.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1 || exit 1
