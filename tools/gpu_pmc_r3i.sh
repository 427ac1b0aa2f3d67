#!/bin/bash
# PMC summaries at HEAD for the bench's post-processing roofline (bench.py POST_PMC*): config 2 at
# its default batch and config 5 at 64 frames (tools/pmc_round.sh, one counter set per pass)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/pmc_round.sh ${1:-pmc_r3i} || exit 1
bash tools/pmc_round.sh ${2:-pmc_body135_r3i} --config body135 --batch 64 || exit 1
