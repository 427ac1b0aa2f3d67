#!/bin/bash
# dev: conv3w phase probe (tools/conv3w_probe.hip) on the BODY_25 stage-layer shapes
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe && {
timeout -k 5 60 tools/conv3w_probe_bin 64 46 82 128 128 20 1 &&
timeout -k 5 60 tools/conv3w_probe_bin 64 46 82 384 128 20 1 &&
timeout -k 5 60 tools/conv3w_probe_bin 64 46 82 96 96 20 1 ; } > gpurun_out/probe/${1:-w}.log 2>&1
