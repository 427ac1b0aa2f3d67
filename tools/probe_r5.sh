#!/bin/bash
# dev (round 5): conv3w stage-layer probe at the bench batch, event-timed NOSTAMPS builds --
# shipped vs halo-same (L2-warm halo for chunks 1..3) vs start-desync of workgroup groups
#   build here:  bash tools/probe_r5.sh build      run on the box:  bash tools/probe_r5.sh run TAG
set -e
B="hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -DNOSTAMPS"
if [ "$1" = build ]; then
  $B -o tools/conv3w_probe_ns tools/conv3w_probe.hip &
  $B -DOPKW_HALO_SAME=1 -o tools/conv3w_probe_ns_same tools/conv3w_probe.hip &
  $B -DOPKW_DESYNC=4500 -DOPKW_DESYNC_N=2 -o tools/conv3w_probe_ns_ds2 tools/conv3w_probe.hip &
  $B -DOPKW_DESYNC=3000 -DOPKW_DESYNC_N=3 -o tools/conv3w_probe_ns_ds3 tools/conv3w_probe.hip &
  $B -DOPKW_DESYNC=1500 -DOPKW_DESYNC_N=3 -o tools/conv3w_probe_ns_ds3s tools/conv3w_probe.hip &
  wait; exit 0
fi
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe
{
for r in 1 2 3; do
  for v in ns ns_same ns_ds2 ns_ds3 ns_ds3s; do
    for cin in 128 384; do
      echo "== $v cin $cin rep $r" && timeout -k 5 60 tools/conv3w_probe_$v 130 46 82 $cin 128 30 1
    done
  done
done ; } > gpurun_out/probe/${2:-r5}.log 2>&1
