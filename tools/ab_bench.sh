#!/bin/bash
# dev: whole-bench A/B (frames/s) of env variants in one GPU call, after the GPU test suite
#   ab_bench.sh OUTDIR "name:KEY=VAL,KEY=VAL" ...     (name "base" = no switch; keys: opk_dev_set)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; shift
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
for spec in "$@"; do
  name=${spec%%:*}; sw=${spec#*:}; [ "$name" = "$spec" ] && sw=""
  devs=""; for kv in ${sw//,/ }; do devs="$devs --dev $kv"; done
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $devs > $out/$name.log 2>&1 || exit 1
done
