#!/bin/bash
# dev: the whole GPU suite + smoke, then interleaved bench A/B of a variant build against the
# defaults on configs 2, 4 and 5, and kernel traces of the defaults (configs 2 and 5)
#   gpu_post_abv.sh OUTDIR VARIANT  (variants/libopk_VARIANT.so as the A side)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; sw=$2
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
V=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_$sw.so
for rep in 1 2; do
  for cfg in body135 body25 multiscale; do
    OPK_LIB_PATH=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline --config $cfg --steps 40 > $out/${cfg}_ab_$rep.log 2>&1 || exit 1
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --config $cfg --steps 40 > $out/${cfg}_base_$rep.log 2>&1 || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof135 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --config body135 > $out/prof135.log 2>&1 || exit 1
