#!/bin/bash
# round 6: conv_image -- bias / slopes in LDS (4 waves per SIMD in split instead of 3) and whole-pixel
# stores through a per-wave LDS image (CONV_IMAGE_STAGE) -- tests, split bench A/B, kernel trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6o}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "conv_image or split or conv1 or tile_variants or cvmat" > $O/pytest_gpu.log 2>&1 || exit 1
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra-configs"
for r in 1 2; do
  timeout -k 10 200 $B --precision split > $O/split_def_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --precision split --dev CONV_IMAGE_STAGE=0 > $O/split_direct_$r.log 2>&1 || exit 1
done
for st in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$st -o run -- \
    python bench.py --precision split --steps 3 --warmup 1 --no-cpu-baseline --no-extra-configs --dev CONV_IMAGE_STAGE=$st > $O/prof_$st.log 2>&1 || exit 1
done
