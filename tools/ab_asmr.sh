#!/bin/bash
# dev: tile-variant bit-identity test, then per-layer kernel traces of conv variants in one call
#   ab_asmr.sh OUTDIR "name:ENV=VAL" ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; shift
mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_gpu_net.py -k "tile_variants" -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
bash tools/ab_run.sh "$@" > /dev/null || exit 1
for spec in "$@"; do
  v=${spec%%:*}
  python tools/layer_report.py gpurun_out/lab/$v/run_kernel_trace.csv 64 > $out/$v.txt
done
