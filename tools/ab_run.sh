#!/bin/bash
# dev: per-layer A/B (rocprofv3 kernel traces) of conv3 variants in one GPU call
#   ab_run.sh "name:ENV=VAL ..." ...     (name "base" = no env)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lab
P="--kernel-trace --output-format csv -o run"
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}; [ "$name" = "$spec" ] && envs=""
  env $envs true || exit 1
  (export $envs; timeout -k 10 300 rocprofv3 $P -d gpurun_out/lab/$name -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline > gpurun_out/lab/$name.log 2>&1) || exit 1
done
