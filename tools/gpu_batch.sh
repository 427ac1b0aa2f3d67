#!/bin/bash
# dev: bench frames/s at several batch sizes (tile quantisation of the 46x82 layers), interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-batch}; shift
mkdir -p $out
for rep in 1 2; do
  for b in "$@"; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --batch $b > $out/bench_b${b}_$rep.log 2>&1 || exit 1
  done
done
