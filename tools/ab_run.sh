#!/bin/bash
# dev: per-layer A/B (rocprofv3 kernel traces) of conv3 variants in one GPU call
#   ab_run.sh "name:KEY=VAL,KEY=VAL" ...     (name "base" = no switch; keys: opk_dev_set)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lab
P="--kernel-trace --output-format csv -o run"
for spec in "$@"; do
  name=${spec%%:*}; sw=${spec#*:}; [ "$name" = "$spec" ] && sw=""
  devs=""; for kv in ${sw//,/ }; do devs="$devs --dev $kv"; done
  timeout -k 10 300 rocprofv3 $P -d gpurun_out/lab/$name -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline $devs > gpurun_out/lab/$name.log 2>&1 || exit 1
done
