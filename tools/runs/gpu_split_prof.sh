#!/bin/bash
# split precision end to end (bench.py --precision split) and its per-kernel statistics
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-split_prof} && mkdir -p $O || exit 1
timeout -k 10 300 python -u bench.py --precision split --steps 10 --no-cpu-baseline > $O/bench_split.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --precision split --steps 5 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
