"""dev: per-launch durations of one net forward from a rocprofv3 kernel trace (the LAST forward in
the trace whose first launch matches --first), with the layer order of BODY_25 for labels.

    python tools/trace_forward.py gpurun_out/r6b/prof_split/run_kernel_trace.csv [--first conv_image]
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", default="conv_image")
    ap.add_argument("--last", default=None, help="kernel name that ends a forward (default: the "
                    "next --first)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.first in r["Kernel_Name"]]
    i0 = starts[-2] if len(starts) > 1 else starts[-1]
    i1 = starts[-1] if len(starts) > 1 else len(rows)
    tot = 0.0
    from oracle import body25
    convs = [l for l in body25.layers() if l["type"] == "Convolution"]
    for r in rows[i0:i1]:
        n = r["Kernel_Name"].replace("void opk::(anonymous namespace)::", "")
        n = n.replace("opk::(anonymous namespace)::", "").split("(")[0]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        print("%9.1f us  %-60s grid %s" % (d, n[:60], r["Grid_Size_X"]))
    print("total %.2f ms over %d launches" % (tot / 1e3, i1 - i0))


if __name__ == "__main__":
    main()
