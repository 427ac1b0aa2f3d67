"""dev: per-kernel mean of rocprofv3 --pmc counters (tools/pmc_conv.sh output dirs)."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        name = r["Kernel_Name"]
        if "conv" not in name and "pool" not in name and "nms" not in name and "cvmat" not in name:
            continue
        short = name.replace("void opk::(anonymous namespace)::", "").replace("opk::(anonymous namespace)::", "").split("(")[0]
        agg[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print("==", k, "dispatches", len(next(iter(cs.values()))))
    wc = m.get("SQ_WAVE_CYCLES")
    for c in sorted(m):
        extra = ""
        if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")):
            extra = "  (%.1f%% of wave cycles)" % (100 * m[c] / wc)
        print("   %-32s %16.0f%s" % (c, m[c], extra))
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CU_CYCLES" in m:
        pass
