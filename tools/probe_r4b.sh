#!/bin/bash
# dev: conv3w at the bench batch -- per-unit stamps of a steady-state tile (cin 128 / 96 / 384),
# then ablation and DMA cache-policy builds against the shipped kernel, interleaved
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe && {
timeout -k 5 60 tools/conv3w_probe_bin 130 46 82 128 128 20 1 &&
timeout -k 5 60 tools/conv3w_probe_bin 130 46 82 96 96 20 1 &&
timeout -k 5 60 tools/conv3w_probe_bin 130 46 82 384 128 20 1 &&
for r in 1 2; do
  for c in "128 128" "96 96"; do
    for v in ns a1 a3 a4 ant bnt; do
      echo -n "$v: " && timeout -k 5 60 tools/conv3w_probe_$v 130 46 82 $c 50 1 || exit 1
    done
  done
done ; } > gpurun_out/probe/${1:-r4b}.log 2>&1
