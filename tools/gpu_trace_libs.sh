#!/bin/bash
# dev: per-layer kernel traces of the bench for several builds (variants/libopk_<name>.so; "base"
# = the in-tree build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-libs}; shift; mkdir -p $out
for v in "$@"; do
  lib=""; [ "$v" != base ] && lib=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_$v.so
  OPK_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr_$v -o run -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline > $out/tr_$v.log 2>&1 || exit 1
  python tools/layer_report.py $out/tr_$v/run_kernel_trace.csv 130 > $out/layers_$v.txt || exit 1
done
