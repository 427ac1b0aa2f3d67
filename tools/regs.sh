#!/bin/bash
# dev: per-kernel VGPR / AGPR / scratch / spills of one .hip source (extra hipcc flags after it)
#   bash tools/regs.sh openpose_amd/csrc/kernels/conv_head.hip -DOPKH_PIPE=0
src=$1; shift
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -Iinclude -x hip --offload-arch=gfx950 \
  -munsafe-fp-atomics "$@" -c "$src" -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk -F': ' '/^Function Name/{n=$2} /^VGPRs:/{v=$2} /^AGPRs/{a=$2} /^ScratchSize/{s=$2} /^SGPRs Spill/{ss=$2} /^VGPRs Spill/{print n, "vgpr", v, "agpr", a, "scratch", s, "sspill", ss, "vspill", $2}' |
  sed 's/_ZN3opk12_GLOBAL__N_1//'
rm -f /tmp/regs_$$.o
