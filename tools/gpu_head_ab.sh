#!/bin/bash
# dev: one GPU call for a conv kernel change -- net output bit for bit against a variant build
# (variants/libopk_<ref>.so), the net tests, an interleaved bench A/B over variant builds and the
# product build, and a kernel trace of the product build (tools/layer_report.py, trace_gaps.py)
#   gpu_head_ab.sh OUTDIR REF VARIANT...      ("base" = the in-tree product build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; ref=$2; shift 2
mkdir -p $out
V=$GRAFT_REPO_ROOT/openpose_amd/variants
OPK_LIB_PATH=$V/libopk_$ref.so timeout -k 10 120 python tools/ab_outputs.py $out/ref.npy 16 > $out/out_ref.log 2>&1 || exit 1
timeout -k 10 120 python tools/ab_outputs.py $out/new.npy 16 > $out/out_new.log 2>&1 || exit 1
python tools/ab_outputs.py --compare $out/ref.npy $out/new.npy > $out/compare.log 2>&1
rm -f $out/*.npy
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_net.log 2>&1 || exit 1
for rep in 1 2; do
  for v in "$@"; do
    lib=""; [ "$v" != "base" ] && lib=$V/libopk_$v.so
    OPK_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 60 > $out/bench_${v}_$rep.log 2>&1 || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1 || exit 1
