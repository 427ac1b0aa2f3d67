#!/bin/bash
# dev: old (variants/libopk_old.so) vs in-tree net outputs under several dev-switch sets
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-bisect}; shift; mkdir -p $out
OLD=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_${OLDLIB:-old}.so
NEW=${NEWLIB:+$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_$NEWLIB.so}
for sw in "$@"; do
  tag=$(echo "$sw" | tr ',=' '__')
  OPK_AB_DEV=$sw OPK_LIB_PATH=$OLD timeout -k 10 120 python tools/ab_outputs.py $out/o.npy 16 > $out/o_$tag.log 2>&1 || exit 1
  OPK_AB_DEV=$sw OPK_LIB_PATH=$NEW timeout -k 10 120 python tools/ab_outputs.py $out/n.npy 16 > $out/n_$tag.log 2>&1 || exit 1
  echo "[$sw] $(python tools/ab_outputs.py --compare $out/o.npy $out/n.npy)" >> $out/compare.log
done
rm -f $out/*.npy
