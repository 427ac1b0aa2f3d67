#!/bin/bash
# round 6: frame warp with R destination rows per workgroup (WARP_ROWS A/B) + its bit-exact tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6m}
mkdir -p $O
PYTHONPATH=. timeout -k 10 240 python -u tools/probe_warp.py > $O/warp.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_preprocess.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
