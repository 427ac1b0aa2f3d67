"""dev: idle time between consecutive kernels of one CNN forward in a rocprofv3 kernel trace.

    python tools/trace_gaps.py <kernel_trace.csv>

A forward starts at a conv1_fused (or conv_image) launch and runs to the next; the gap of a launch
is its start minus the previous launch's end on the same queue.  Prints per-forward busy / span and
the largest gaps (launch-boundary cost that a graph or a cross-layer schedule could remove)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "conv1_fused" in r["Kernel_Name"] or "conv_image" in r["Kernel_Name"]]
fw = []
for a, b in zip(starts, starts[1:]):
    seg = rows[a:b]
    # the forward ends at its last conv kernel (post-processing follows on the same stream)
    last = max(i for i, r in enumerate(seg) if "conv" in r["Kernel_Name"])
    seg = seg[:last + 1]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    gaps = defaultdict(list)
    for p, r in zip(seg, seg[1:]):
        g = int(r["Start_Timestamp"]) - int(p["End_Timestamp"])
        gaps[r["Kernel_Name"].split("(")[0][-60:]].append(g)
    fw.append((t1 - t0, busy, len(seg), gaps))
for span, busy, n, _ in fw:
    print(f"launches {n:4d}  span {span / 1e3:9.1f} us  kernels {busy / 1e3:9.1f} us  idle {(span - busy) / 1e3:7.1f} us")
if fw:
    g = fw[len(fw) // 2][3]
    print("gaps before (median forward), us: name  n  mean  max")
    for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:60s} {len(v):3d} {sum(v) / len(v) / 1e3:7.2f} {max(v) / 1e3:7.2f}")
