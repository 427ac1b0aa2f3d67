#!/bin/bash
# dev: conv3t ablation builds (openpose_amd/variants/libopk_t*.so), per-layer kernel traces
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-tall_abl}; shift
mkdir -p $out
for v in "$@"; do
  name=${v%%:*}; sw=${v#*:}; lib=""; args=""
  for kv in ${sw//,/ }; do case $kv in LIB=*) lib=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_${kv#LIB=}.so ;; *) args="$args --dev $kv" ;; esac; done
  OPK_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr_$name -o run -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline $args > $out/tr_$name.log 2>&1 || exit 1
  python tools/layer_report.py $out/tr_$name/run_kernel_trace.csv 64 > $out/layers_$name.txt || exit 1
done
