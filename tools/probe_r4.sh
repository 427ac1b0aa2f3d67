#!/bin/bash
# dev: conv3w skeleton at the bench batch (130 frames): phase stamps (wave 0 of every block) and
# event-timed launches, cin 128 / 384 / 96; E2 (OPK_CONV3W_E2=1) against the default
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe && {
for f in 32 65 130 260; do
  timeout -k 5 60 tools/conv3w_probe_bin $f 46 82 128 128 20 1 || exit 1
done
timeout -k 5 60 tools/conv3w_probe_bin 130 46 82 384 128 20 1 &&
timeout -k 5 60 tools/conv3w_probe_bin 130 46 82 96 96 20 1 &&
timeout -k 5 60 tools/conv3w_probe_bin 130 46 82 128 128 20 1 1 &&
for r in 1 2; do
  echo "== rep $r: base / E2 (no stamps)" &&
  timeout -k 5 60 tools/conv3w_probe_ns 130 46 82 128 128 50 1 &&
  timeout -k 5 60 tools/conv3w_probe_ns 130 46 82 128 128 50 1 0 2 &&
  timeout -k 5 60 tools/conv3w_probe_ns 130 46 82 96 96 50 1 &&
  timeout -k 5 60 tools/conv3w_probe_ns 130 46 82 96 96 50 1 0 2 &&
  timeout -k 5 60 tools/conv3w_probe_ns 130 46 82 256 128 50 1 &&
  timeout -k 5 60 tools/conv3w_probe_ns 130 46 82 256 128 50 1 0 2 || exit 1
done
timeout -k 5 60 tools/conv3w_probe_bin 130 46 82 128 128 20 1 0 2 ; } > gpurun_out/probe/${1:-r4}.log 2>&1
