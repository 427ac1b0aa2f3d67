#!/bin/bash
# round 6: conv_image occupancy -- offsets table in LDS (default build: 4 waves per SIMD in split)
# against builds asking the register allocator for 5 / 6 waves (openpose_amd/ab/libopk_w5/w6.so);
# kernel traces of the split bench, interleaved x2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6p}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "conv_image or split_launch or split_every" > $O/pytest_gpu.log 2>&1 || exit 1
for r in 1 2; do
  for v in def w5 w6; do
    unset OPK_LIB_PATH
    [ $v != def ] && export OPK_LIB_PATH=$GRAFT_REPO_ROOT/openpose_amd/ab/libopk_$v.so
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_${v}_$r -o run -- \
      python bench.py --precision split --steps 3 --warmup 1 --no-cpu-baseline --no-extra-configs > $O/prof_${v}_$r.log 2>&1 || exit 1
  done
done
