#!/bin/bash
# dev: conv1_fused ablation / A-B builds (openpose_amd/variants/libopk_<name>.so) under a short
# profiled bench each, one GPU call:   c1_ablate.sh OUTDIR name ...   ("base" = the product build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; shift
mkdir -p $out
for v in "$@"; do
  lib=""; [ "$v" != "base" ] && lib=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_$v.so
  OPK_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline > $out/$v.log 2>&1 || exit 1
done
