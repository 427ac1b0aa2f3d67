#!/bin/bash
# dev: net tests, then interleaved bench A/B of dev-switch sets, then a kernel trace of the default
#   gpu_ab.sh OUTDIR "SWITCHES_A" "SWITCHES_B" ...   ("" = defaults; KEY=VAL separated by spaces;
#   LIB=name loads the variant build openpose_amd/variants/libopk_name.so through OPK_LIB_PATH)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; shift
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/pytest_net.log 2>&1 || exit 1
k=0
for rep in 1 2; do
for v in "$@"; do
  k=$((k+1)); tag=$(echo "${v:-default}" | tr ' =' '_-')_$k
  args=""; lib=""
  for kv in $v; do case $kv in LIB=*) lib=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_${kv#LIB=}.so ;; *) args="$args --dev $kv" ;; esac; done
  OPK_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $out/bench_$tag.log 2>&1 || exit 1
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1 || exit 1
