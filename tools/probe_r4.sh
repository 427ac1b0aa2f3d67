#!/bin/bash
# dev: conv3w skeleton at the bench batch (130 frames): phase stamps (wave 0 of every block) and
# event-timed launches, cin 128 / 384 / 96
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe && {
for f in 32 65 130 260; do
  timeout -k 5 60 tools/conv3w_probe_bin $f 46 82 128 128 20 1 || exit 1
done
timeout -k 5 60 tools/conv3w_probe_bin 130 46 82 384 128 20 1 &&
timeout -k 5 60 tools/conv3w_probe_bin 130 46 82 96 96 20 1 &&
timeout -k 5 60 tools/conv3w_probe_bin 130 46 82 128 128 20 1 1 &&
timeout -k 5 60 tools/conv3w_probe_ns 130 46 82 128 128 20 1 0 1 ; } > gpurun_out/probe/${1:-r4}.log 2>&1
