#!/bin/bash
# round 6, last: smoke + the conv_image / split-launch tests at HEAD, then the PMC passes bench.py reads
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6v}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "conv_image or split_launch or split_every" > $O/pytest_gpu.log 2>&1 || exit 1
export PMC_COMMIT=$(cat .pmc_commit 2>/dev/null)
bash tools/pmc_round.sh ${OUT_TAG:-r6v}/pmc > $O/pmc.log 2>&1 || exit 1
bash tools/pmc_round.sh ${OUT_TAG:-r6v}/pmc_split --precision split > $O/pmc_split.log 2>&1 || exit 1
bash tools/pmc_round.sh ${OUT_TAG:-r6v}/pmc_body135 --config body135 --batch 64 > $O/pmc_body135.log 2>&1 || exit 1
