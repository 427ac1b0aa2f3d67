#!/bin/bash
# round 6, frozen kernels: the whole GPU suite, smoke(), the default bench (the driver's command,
# configs legs and CPU baseline included), kernel statistics of the fp16 and split benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6k}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fp16 -o run -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/prof_fp16.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split -o run -- \
  python bench.py --precision split --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/prof_split.log 2>&1 || exit 1
