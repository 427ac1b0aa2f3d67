#!/bin/bash
# round 6, frozen kernels: PMC passes (tools/pmc_round.sh) of the fp16 bench, the split bench and
# config 5 (BODY_135) -- the files bench.py reads (profiles/round6/pmc*)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6l}
mkdir -p $O
export PMC_COMMIT=$(cat .pmc_commit 2>/dev/null)
bash tools/pmc_round.sh ${OUT_TAG:-r6l}/pmc > $O/pmc.log 2>&1 || exit 1
bash tools/pmc_round.sh ${OUT_TAG:-r6l}/pmc_split --precision split > $O/pmc_split.log 2>&1 || exit 1
bash tools/pmc_round.sh ${OUT_TAG:-r6l}/pmc_body135 --config body135 --batch 64 > $O/pmc_body135.log 2>&1 || exit 1
