#!/bin/bash
# dev: warp on its own stream -- GPU tests, smoke, bench A/B (config 2 and 4)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-warp}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
for rep in 1 2; do
  for v in "" "WARP_STREAM=0"; do
    tag=${v:-default}; tag=${tag//=/-}_$rep
    args=""; for kv in $v; do args="$args --dev $kv"; done
    timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $out/bench_$tag.log 2>&1 || exit 1
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --config multiscale --steps 10 $args > $out/ms_$tag.log 2>&1 || exit 1
  done
done
