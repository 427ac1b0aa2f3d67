#!/bin/bash
# round 6: the NMS walk at 7 / 8 waves per SIMD (register-allocator hint, builds
# openpose_amd/ab/libopk_n7/n8.so) against the default 6 -- config 5 interleaved x2 + kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6s}
mkdir -p $O
B5="python -u bench.py --config body135 --steps 30 --warmup 3 --no-cpu-baseline --no-extra-configs"
for r in 1 2; do
  for v in def n7 n8; do
    unset OPK_LIB_PATH
    [ $v != def ] && export OPK_LIB_PATH=$GRAFT_REPO_ROOT/openpose_amd/ab/libopk_$v.so
    timeout -k 10 200 $B5 > $O/b135_${v}_$r.log 2>&1 || exit 1
  done
done
for v in def n7 n8; do
  unset OPK_LIB_PATH
  [ $v != def ] && export OPK_LIB_PATH=$GRAFT_REPO_ROOT/openpose_amd/ab/libopk_$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- \
    python bench.py --config body135 --steps 10 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/prof_$v.log 2>&1 || exit 1
done
