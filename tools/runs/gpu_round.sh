#!/bin/bash
# GPU round: parity tests, smoke, default bench, multi-scale bench, rocprofv3 kernel stats (CSV)
#   OUT_TAG=<dir under gpurun_out>  STEPS=<what to run: tests,smoke,bench,multi,prof>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT_TAG:-r2}
STEPS=${STEPS:-tests,smoke,bench,multi,prof}
mkdir -p $OUT
run() { case ",$STEPS," in *",$1,"*) return 0;; *) return 1;; esac; }
if run tests; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
fi
if run smoke; then
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
fi
if run bench; then
  timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || exit 1
fi
if run multi; then
  timeout -k 10 300 python -u bench.py --config multiscale --steps 10 > $OUT/bench_multiscale.log 2>&1 || exit 1
fi
if run prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_prof.log 2>&1 || exit 1
fi
