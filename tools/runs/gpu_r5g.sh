#!/bin/bash
# end-of-round refresh at HEAD (kernels as at r5f): every GPU test, smoke, default and BODY_135 benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT_TAG:-r5g}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config body135 --steps 30 > $OUT/bench_body135.log 2>&1 || exit 1
