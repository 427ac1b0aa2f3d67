#!/bin/bash
# dev: conv tests, then per variant a whole bench (frames/s) and a rocprofv3 kernel trace with
# its per-layer report, in one GPU call.
#   ab_all.sh OUTDIR "name:KEY=VAL,KEY=VAL" ...     (name "base" = no switch; keys: opk_dev_set)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; shift
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -x -q --timeout 120 --timeout-method thread > $out/pytest_net.log 2>&1 || exit 1
for spec in "$@"; do
  name=${spec%%:*}; sw=${spec#*:}; [ "$name" = "$spec" ] && sw=""
  devs=""; for kv in ${sw//,/ }; do devs="$devs --dev $kv"; done
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $devs > $out/$name.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr_$name -o run -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline $devs > $out/tr_$name.log 2>&1 || exit 1
  python tools/layer_report.py $out/tr_$name/run_kernel_trace.csv 64 > $out/layers_$name.txt || exit 1
done
