"""Per-kernel PMC summary of tools/pmc_round.sh passes (rocprofv3 --pmc, one pass per counter set).

    python tools/pmc_report.py <pass dir>... [--json out.json] [--batch FRAMES]

Per kernel (mean per launch): duration, effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration),
MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x the cycles the launch ran), wave time parked
(SQ_WAIT_ANY / SQ_WAVE_CYCLES), VALU wave-instructions and their issue rate against the chip's
VALU issue peak, LDS bank conflicts per LDS cycle, and HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, the
gfx950 correction of MI355X_MICROARCH.md §HBM).  Also the time-weighted MFMA busy of the CNN's conv
kernels and the per-step counts of the post-processing kernels (bench.py's post_roofline).
Durations come from the profiled passes (counters collected, so clocks read a few % low).
"""
import collections
import csv
import json
import os
import sys

SIMDS = 1024                 # 256 CUs x 4 SIMDs
VALU_PEAK = SIMDS * 0.5 * 2.4e9   # wave64 VALU instructions/s: one per 2 cycles per SIMD-32 at 2.4 GHz
POST = ("add_inplace", "nms_detect", "nms_finalize", "paf_compact")


def short(name):
    name = name.replace("void ", "").replace("opk::(anonymous namespace)::", "")
    return name[:name.find("(")] if "(" in name else name


def load(dirs):
    """{kernel: {counter: [values per launch]}} and {kernel: [durations ns]}"""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for d in dirs:
        path = os.path.join(d, "run_counter_collection.csv")
        seen = set()
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (r["Dispatch_Id"], k)
            if d == dirs[0] and key not in seen:
                seen.add(key)
                durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals, durs


def summarise(vals, durs):
    out = {}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = durs.get(k)
        if not d:
            continue
        dur = sum(d) / len(d) * 1e-9
        e = {"launches": len(d), "mean_us": dur * 1e6}
        gui = m.get("GRBM_GUI_ACTIVE")
        if gui:
            cyc = gui / 8.0
            e["clock_ghz"] = cyc / dur / 1e9
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                e["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc)
            if "SQ_INSTS_MFMA" in m:
                e["mfma_busy_16cyc"] = 16.0 * m["SQ_INSTS_MFMA"] / (SIMDS * cyc)
        if m.get("SQ_WAVE_CYCLES"):
            e["parked"] = m.get("SQ_WAIT_ANY", 0.0) / m["SQ_WAVE_CYCLES"]
            e["issue_stalled"] = m.get("SQ_WAIT_INST_ANY", 0.0) / m["SQ_WAVE_CYCLES"]
        if "SQ_INSTS_VALU" in m:
            e["valu_insts"] = m["SQ_INSTS_VALU"]
            e["valu_frac"] = m["SQ_INSTS_VALU"] / dur / VALU_PEAK
        for c in ("SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_MFMA", "SQ_WAVES"):
            if c in m:
                e[c.lower()] = m[c]
        if m.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"]
        if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
            e["hbm_bytes"] = 1024.0 * (2.0 * m.get("FETCH_SIZE", 0.0) + m.get("WRITE_SIZE", 0.0))
            e["hbm_frac"] = e["hbm_bytes"] / dur / 8e12
        out[k] = e
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    js = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 64
    for x in (js, str(batch)):
        if x in args:
            args.remove(x)
    vals, durs = load(args)
    ks = summarise(vals, durs)
    conv = {k: e for k, e in ks.items() if ("conv" in k and "kernel" in k) or "maxpool" in k}
    tot = sum(e["mean_us"] * e["launches"] for e in conv.values())
    busy = sum(e.get("mfma_busy", 0.0) * e["mean_us"] * e["launches"] for e in conv.values())
    post = {}
    for tag in POST:
        for k, e in ks.items():
            if k.startswith(tag):
                post[k] = e
    step = {"valu_insts": sum(e.get("valu_insts", 0.0) for e in post.values()),
            "hbm_bytes": sum(e.get("hbm_bytes", 0.0) for e in post.values()),
            "kernel_us": sum(e["mean_us"] for e in post.values())}
    res = {"batch": batch, "valu_peak_insts_per_s": VALU_PEAK,
           "cnn": {"conv_kernel_us_profiled": tot,
                   "time_weighted_mfma_busy": busy / tot if tot else None},
           "post_step": step, "post_kernels": post, "kernels": ks}
    for k, e in sorted(ks.items(), key=lambda kv: -kv[1]["mean_us"] * kv[1]["launches"]):
        print("%-44s n=%4d %9.1f us" % (k[:44], e["launches"], e["mean_us"]) +
              "".join("  %s=%.3g" % (f, e[f]) for f in ("clock_ghz", "mfma_busy", "parked",
                                                        "valu_frac", "hbm_frac",
                                                        "lds_bank_conflict_frac") if f in e))
    print("CNN conv kernels: time-weighted MFMA busy %.3f over %.0f us"
          % (res["cnn"]["time_weighted_mfma_busy"] or 0, tot))
    print("post-processing per step: %.3g VALU wave-insts, %.3g HBM bytes, %.1f us of kernels"
          % (step["valu_insts"], step["hbm_bytes"], step["kernel_us"]))
    if js:
        json.dump(res, open(js, "w"), indent=1)


if __name__ == "__main__":
    main()
