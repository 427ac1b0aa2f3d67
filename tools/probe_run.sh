#!/bin/bash
# dev: conv3 phase probe with ablation builds (tools/conv3_probe_aN, -DOPK3_ABLATE=N)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
{
for cfg in "64 46 82 128 128" "64 92 164 256 256"; do
  for a in 0 2 6 7; do
    echo "== nonpersist ablate $a cfg $cfg"
    OPK_CONV3_PERSIST=0 timeout -k 5 60 tools/conv3_probe_a$a $cfg 20 || exit 1
  done
done
} > gpurun_out/probe/probe2.log 2>&1
