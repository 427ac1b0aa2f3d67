#!/bin/bash
# dev: conv3w8 DMA ablations (0 as built, 4 no DMA, 7 no halo DMA, 8 no weight DMA after the prologue)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe && {
for rep in 1 2; do
for cin in 384 128; do
for v in 0 4 7 8; do
  echo "== ablate $v cin $cin rep $rep"
  timeout -k 5 60 tools/conv3w_probe_w8a$v 64 46 82 $cin 128 30 1 0 1 || exit 1
done; done; done; } > gpurun_out/probe/w8dma.log 2>&1
