#!/bin/bash
# dev: conv3w per-launch vs per-tile cost -- the stage-layer shape at 16..256 frames (NOSTAMPS build)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe && {
for cin in 128 384; do for f in 16 32 64 128 256; do
  timeout -k 5 60 tools/conv3w_probe_ns $f 46 82 $cin 128 20 1 || exit 1
done; done; } > gpurun_out/probe/frames.log 2>&1
