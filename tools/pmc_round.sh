#!/bin/bash
# PMC passes over a short bench.py run (one rocprofv3 pass per counter set, each under its own
# time limit), then tools/pmc_report.py turns them into per-kernel-group summaries:
#   pmc_round.sh OUTDIR [bench args...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$1; shift
mkdir -p $out
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra-configs $*"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- $B > $out/p$i.log 2>&1 || exit 1
done
# frames per step of the profiled run (bench.py's default unless --batch is passed)
batch=$(python -c "import sys; a=sys.argv[1:]; print(a[a.index('--batch')+1] if '--batch' in a else '')" "$@")
[ -z "$batch" ] && batch=$(python -c "import torch, bench; print(bench.tile_aligned_batch(torch.cuda.get_device_properties(0).multi_processor_count))")
python tools/pmc_report.py $out/p1 $out/p2 $out/p3 $out/p4 --json $out/report.json --batch $batch > $out/report.txt 2>&1 &&
python tools/pmc_summary.py $out/p3/run_counter_collection.csv $out/p4/run_counter_collection.csv $batch $out/pmc_traffic.json > $out/pmc_traffic.log 2>&1
# provenance: the commit (PMC_COMMIT, passed in by the caller: the box has no .git) and the digests
# of the kernel sources these counters were collected with, whole and per group (bench.py reports
# them and whether they still describe the running tree)
python - "$out" <<'PY'
import json, os, sys
for name in ("report.json", "pmc_traffic.json"):
    p = os.path.join(sys.argv[1], name)
    if os.path.exists(p):
        d = json.load(open(p))
        d["commit"] = os.environ.get("PMC_COMMIT")
        json.dump(d, open(p, "w"), indent=1)
PY
for name in report.json pmc_traffic.json; do
  [ -f $out/$name ] && python tools/pmc_stamp.py $out/$name
done
true
