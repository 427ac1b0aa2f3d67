#!/bin/bash
# round 6, first call: split precision on the fused kernels (conv3w8 split, conv_image split),
# the pending NMS jump / PAF exit, the frame-run and net-lifetime fixes -- the whole GPU suite,
# the default bench (with its new split / config-4 / config-5 legs) and the split kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6a}
mkdir -p $O
timeout -k 10 840 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
  ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split -o run -- \
  python bench.py --precision split --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/prof_split.log 2>&1 || exit 1
