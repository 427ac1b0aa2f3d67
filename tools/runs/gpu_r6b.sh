#!/bin/bash
# round 6: the two fixed tests + the split per-layer bound, then the default bench (with its split /
# config-4 / config-5 legs) and the split kernel stats; conv_head partials XOR layout A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
  -k "split or head or layers or tile_variants" > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split -o run -- \
  python bench.py --precision split --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/prof_split.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fp16 -o run -- \
  python bench.py --steps 10 --no-cpu-baseline --no-extra-configs > $O/prof_fp16.log 2>&1 || exit 1
