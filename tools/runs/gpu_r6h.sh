#!/bin/bash
# round 6: two forwards in flight on two streams (tools/probe_streams.py), both precisions
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6h}
mkdir -p $O
PYTHONPATH=. timeout -k 10 240 python -u tools/probe_streams.py > $O/streams_fp16.log 2>&1 || exit 1
PYTHONPATH=. timeout -k 10 300 python -u tools/probe_streams.py --precision split --iters 3 > $O/streams_split.log 2>&1 || exit 1
