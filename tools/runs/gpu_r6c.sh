#!/bin/bash
# round 6: split weights packed once (w_hi, w_lo), n-blocks by XCD (W8_NBX) -- tests, then split
# bench A/B (default / W8_NBX=0 / CONV3_SMALL=0 for the 64-channel full-resolution layer) and the
# fp16 bench with and without W8_NBX, interleaved; kernel trace of the default split bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6c}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
  -k "split or tile_variants or layers" > $O/pytest_gpu.log 2>&1 || exit 1
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra-configs"
for r in 1 2; do
  timeout -k 10 200 $B --precision split > $O/split_def_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --precision split --dev W8_NBX=0 > $O/split_nonbx_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --precision split --dev CONV3_SMALL=0 > $O/split_big64_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --steps 20 > $O/fp16_def_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --steps 20 --dev W8_NBX=1 > $O/fp16_nbx_$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split -o run -- \
  python bench.py --precision split --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/prof_split.log 2>&1 || exit 1
