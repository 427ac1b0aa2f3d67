#!/bin/bash
# round 6: ablation probe of the split conv3w8 (timing only, wrong results): no halo DMA after the
# prologue (OPK8_ABLATE=7) / no weight DMA (=8) against the product build -- kernel traces
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6w}
mkdir -p $O
for v in def a7 a8; do
  unset OPK_LIB_PATH
  [ $v != def ] && export OPK_LIB_PATH=$GRAFT_REPO_ROOT/openpose_amd/ab/libopk_$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$v -o run -- \
    python bench.py --precision split --steps 3 --warmup 1 --no-cpu-baseline --no-extra-configs > $O/prof_$v.log 2>&1 || exit 1
done
