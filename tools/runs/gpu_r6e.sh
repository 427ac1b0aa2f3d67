#!/bin/bash
# round 6: conv3w8 BN = 64 (conv1_2 in split precision), NMS jump off / PAF exit on -- tests, split
# bench A/B (CONV3W8_64=0), config-5 A/B against the build without the PAF exit, split kernel trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6e}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
  -k "split or tile_variants or layers or conv1 or nms or paf or connector" > $O/pytest_gpu.log 2>&1 || exit 1
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra-configs"
V=$GRAFT_REPO_ROOT/openpose_amd/ab/libopk_noexit.so
for r in 1 2; do
  timeout -k 10 200 $B --precision split > $O/split_def_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B --precision split --dev CONV3W8_64=0 > $O/split_no64_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --config body135 --steps 50 --no-cpu-baseline > $O/b135_exit_$r.log 2>&1 || exit 1
  OPK_LIB_PATH=$V timeout -k 10 200 python -u bench.py --config body135 --steps 50 --no-cpu-baseline > $O/b135_noexit_$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split -o run -- \
  python bench.py --precision split --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/prof_split.log 2>&1 || exit 1
