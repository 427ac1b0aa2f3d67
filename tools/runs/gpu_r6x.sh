#!/bin/bash
# round 6: conv3w8 with unit u+2's DMA issued right after the mid-unit barrier (OPK8_DMA_EARLY=1,
# openpose_amd/ab/libopk_de.so) against after tap 2 -- split kernel traces x2 (interleaved)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6x}
mkdir -p $O
for r in 1 2; do
  for v in def de; do
    unset OPK_LIB_PATH
    [ $v != def ] && export OPK_LIB_PATH=$GRAFT_REPO_ROOT/openpose_amd/ab/libopk_$v.so
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_${v}_$r -o run -- \
      python bench.py --precision split --steps 3 --warmup 1 --no-cpu-baseline --no-extra-configs > $O/prof_${v}_$r.log 2>&1 || exit 1
  done
done
