#!/bin/bash
# dev: conv3 phase probe with ablation builds (tools/conv3_probe_aN, -DOPK3_ABLATE=N)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
{
for cfg in "64 46 82 128 128" "64 46 82 128 96"; do
  echo "== persistent cfg $cfg"; timeout -k 5 60 tools/conv3_probe_a0 $cfg 20 || exit 1
  for a in 0 1 2 3 4 5; do
    echo "== nonpersist ablate $a cfg $cfg"
    OPK_CONV3_PERSIST=0 timeout -k 5 60 tools/conv3_probe_a$a $cfg 20 || exit 1
  done
done
for cfg in "64 92 164 256 256" "64 46 82 512 512"; do
  for a in 0 1 2 3 4 5; do
    echo "== ablate $a cfg $cfg"
    timeout -k 5 60 tools/conv3_probe_a$a $cfg 20 || exit 1
  done
done
} > gpurun_out/probe/probe.log 2>&1
