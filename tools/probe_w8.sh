#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe_w8 && {
for rep in 1 2; do
for v in 0 6; do
  echo "== ablate $v rep $rep"
  timeout -k 5 60 tools/conv3w_probe_w8a$v 64 46 82 384 128 30 1 0 1 || exit 1
  timeout -k 5 60 tools/conv3w_probe_w8a$v 64 46 82 384 128 30 1 1 1 || exit 1
done; done; } > gpurun_out/probe_w8/w8.log 2>&1
