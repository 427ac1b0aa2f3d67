#!/bin/bash
# frames per step at 4 / 6 / 8 persistent tiles per CU (130 / 195 / 260 frames), interleaved on one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-batch_ab} && mkdir -p $O || exit 1
for r in 1 2; do
  for b in 130 260 195; do
    timeout -k 10 300 python -u bench.py --batch $b --steps 20 --no-cpu-baseline > $O/b${b}_$r.log 2>&1 || exit 1
  done
done
