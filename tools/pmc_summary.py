"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into HBM bytes per CNN
forward (the unit bench.py's roofline uses), with the gfx950 correction of MI355X_MICROARCH.md §HBM:
FETCH_SIZE counts 64-B units per 128-B request on wide streaming reads -> x2; WRITE_SIZE exact.

    python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
        <frames_per_step> <out.json>

A CNN forward = every conv*/maxpool kernel; forwards are counted by the first conv's launches
(conv1_fused_kernel, or conv_image_kernel when the front end is not fused).  Post-processing kernels are reported per launch.
"""
import collections
import csv
import json
import sys


def per_kernel(path):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        agg[name][0] += 1
        agg[name][1] += float(r["Counter_Value"]) * 1024.0   # counters are KB
    return agg


def short(name):
    name = name.replace("void ", "").replace("opk::(anonymous namespace)::", "")
    return name[:name.rfind("(")] if name.endswith(")") else name


def main():
    fetch, write, frames, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    f, w = per_kernel(fetch), per_kernel(write)
    cnn = [k for k in f if ("conv" in k and "kernel" in k) or "maxpool" in k]
    forwards = sum(f[k][0] for k in f if "conv1_fused_kernel" in k or "conv_image_kernel" in k)
    # a pass with no CNN (the BODY_135 injection config: post-processing only) has no forward to
    # divide by: its CNN fields are None and only the post kernels are summarised
    fetch_b = 2.0 * sum(f[k][1] for k in cnn) / forwards if forwards else None
    write_b = sum(w[k][1] for k in cnn if k in w) / forwards if forwards else None
    by_kernel = {}
    for k in (cnn if forwards else []):
        by_kernel[short(k)] = {
            "launches_per_forward": f[k][0] / forwards,
            "fetch_bytes_per_forward": 2.0 * f[k][1] / forwards,
            "write_bytes_per_forward": (w[k][1] if k in w else 0.0) / forwards}
    post = {}
    for tag in ("cvmat_to_input", "nms_detect", "nms_finalize", "paf_compact", "resize_merge"):
        ks = [k for k in f if tag in k]
        n = sum(f[k][0] for k in ks)
        if n:
            post[tag] = {"fetch_bytes_per_launch": 2.0 * sum(f[k][1] for k in ks) / n,
                         "write_bytes_per_launch": sum(w[k][1] for k in ks if k in w) / n}
    res = {"unit": "bytes per CNN forward of %d frames" % frames, "batch": frames,
           "forwards_profiled": forwards,
           "cnn_forward_fetch_bytes": fetch_b, "cnn_forward_write_bytes": write_b,
           "cnn_forward_hbm_bytes": fetch_b + write_b if forwards else None,
           "by_kernel": by_kernel, "post": post,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "by_kernel"}, indent=1))


if __name__ == "__main__":
    main()
