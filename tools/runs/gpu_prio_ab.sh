#!/bin/bash
# A/B: the pipeline's side streams (post-processing, result copies) at the lowest priority
# (--dev SIDE_PRIO=1) vs the default, config 2 and config 5 interleaved on one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-prio_ab} && mkdir -p $O || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > $O/b25_def_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --dev SIDE_PRIO=1 > $O/b25_low_$r.log 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline > $O/b135_def_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline --dev SIDE_PRIO=1 > $O/b135_low_$r.log 2>&1 || exit 1
done
