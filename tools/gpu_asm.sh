#!/bin/bash
# dev: host assembly rework (worker pool, scratch, packed sort, one overflow copy, lean gather
# unpack) -- GPU tests, then config 5 / config 2 bench A/B against the previous library
# (LIB=oldasm: openpose_amd/variants/libopk_oldasm.so)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-asm}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
for rep in 1 2; do
  for v in "" "LIB=oldasm"; do
    tag=${v:-new}; tag=${tag//=/-}_$rep
    lib=""; case $v in LIB=*) lib=$GRAFT_REPO_ROOT/openpose_amd/variants/libopk_${v#LIB=}.so ;; esac
    OPK_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --config body135 > $out/b135_$tag.log 2>&1 || exit 1
    OPK_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline > $out/bench_$tag.log 2>&1 || exit 1
  done
done
# per-dispatch kernel trace (start / end stamps) of a short bench: gaps between the CNN's kernels
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o kt -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 2 > $out/trace.log 2>&1 || exit 1
