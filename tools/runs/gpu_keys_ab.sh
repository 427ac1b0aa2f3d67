#!/bin/bash
# the GPU-path connection keys sorted on the device (PAF_KEYS=1, the default) vs on the host
# (PAF_KEYS=0): post-processing / connector / sharded GPU tests, config 5 benches interleaved,
# kernel statistics of config 5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-keys_ab} && mkdir -p $O || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "connector or pipeline or inject or sharded or pose or semantics" > $O/pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline > $O/b135_keys_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --config body135 --steps 30 --no-cpu-baseline --dev PAF_KEYS=0 > $O/b135_host_$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --config body135 --steps 10 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
