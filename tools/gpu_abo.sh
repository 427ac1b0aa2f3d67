#!/bin/bash
# dev: bit-for-bit BODY_25 net output of the in-tree build against variants/libopk_old.so (each
# twice: the forward is deterministic), then the bench A/B (tools/gpu_ab.sh)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-headab}; mkdir -p $out
OLD=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_old.so
for k in 1 2; do
  OPK_LIB_PATH=$OLD timeout -k 10 120 python tools/ab_outputs.py $out/old$k.npy 16 > $out/out_old$k.log 2>&1 || exit 1
  timeout -k 10 120 python tools/ab_outputs.py $out/new$k.npy 16 > $out/out_new$k.log 2>&1 || exit 1
done
for p in "old1 old2" "new1 new2" "old1 new1"; do set -- $p; python tools/ab_outputs.py --compare $out/$1.npy $out/$2.npy >> $out/compare.log 2>&1; done
rm -f $out/*.npy
[ -n "$2" ] && bash tools/gpu_ab.sh ${1:-headab} "LIB=old" ""
exit 0
