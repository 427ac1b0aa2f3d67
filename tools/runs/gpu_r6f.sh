#!/bin/bash
# round 6: split precision chunk-major (hi halo staged once for two products), conv_image 16-byte
# stores, split pool2 / pool3 in conv3w8's epilogue -- tests, split bench A/B (CONV_IMAGE_WIDE=0,
# POOL_FUSE=0), kernel trace, PMC of the split bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6f}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit 1
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra-configs"
for r in 1 2; do
  timeout -k 10 200 $B --precision split > $O/split_def_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --precision split --dev CONV_IMAGE_WIDE=0 > $O/split_imgnarrow_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --precision split --dev POOL_FUSE=0 > $O/split_nopool_$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split -o run -- \
  python bench.py --precision split --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/prof_split.log 2>&1 || exit 1
PMC_COMMIT=$(cat .pmc_commit 2>/dev/null) bash tools/pmc_round.sh r6f/pmc_split --precision split > $O/pmc_split.log 2>&1 || exit 1
