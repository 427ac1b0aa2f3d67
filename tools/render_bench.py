"""Time the GPU renderers (render.hip) on a 1920x1080 float BGR frame, HIP events on the context's
stream, and price each against HBM: algorithmic bytes = the frame read + written once (24 B/pixel)
plus, for heat-map renders, the heat planes read once.

    python tools/render_bench.py [--iters N] [--out FILE]

Prints one JSON object per case (and writes them to --out)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from openpose_amd.api import Context  # noqa: E402
from tests.test_render import people_on  # noqa: E402

HBM_PEAK = 8000.0   # GB/s, MI355X_MICROARCH.md


def timed(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters   # us per call


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--out", default=None)
    ap.add_argument("--cpu", action="store_true", help="also time the oracle (CPU, 1 thread)")
    args = ap.parse_args()
    ctx = Context(0)
    w, h = 1920, 1080
    hw, hh = 656, 368            # the x8 net-resolution heat maps of a 16:9 frame at -1x368
    scale = h / hh
    rng = np.random.default_rng(0)
    frame = torch.from_numpy(rng.uniform(0, 255, (h, w, 3)).astype(np.float32)).cuda()
    heat = torch.from_numpy(rng.uniform(-0.2, 1.0, (78, hh, hw)).astype(np.float32)).cuda()
    frame_bytes = 24.0 * w * h
    rows = []
    cases = []
    for n in (1, 20, 127):
        kp = torch.from_numpy(people_on(w, h, n, 25, seed=n, spread=0.08)).cuda()
        cases.append(("pose_keypoints_%dp" % n, frame_bytes,
                      lambda kp=kp: ctx.render_pose_keypoints(frame, kp, 0, threshold=0.05)))
    plane = 4.0 * hw * hh
    cases += [
        ("heat_map_bicubic", frame_bytes + plane, lambda: ctx.render_heat_map(frame, heat, scale, 3)),
        ("heat_maps_25_nearest", frame_bytes + 25 * plane,
         lambda: ctx.render_heat_maps(frame, heat, scale)),
        ("paf_bilinear", frame_bytes + 2 * plane, lambda: ctx.render_pafs(frame, heat, scale, part=26)),
        ("pafs_26_nearest", frame_bytes + 52 * plane, lambda: ctx.render_pafs(frame, heat, scale)),
    ]
    for name, nbytes, fn in cases:
        us = timed(fn, args.iters)
        gbs = nbytes / (us * 1e-6) / 1e9
        row = {"case": name, "frame": "%dx%d" % (w, h), "us_per_call": round(us, 2),
               "fps": round(1e6 / us, 1), "algorithmic_bytes": int(nbytes),
               "achieved_GBps": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK, 3)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.cpu:
        import oracle
        f = frame.cpu().numpy()
        kp = people_on(w, h, 20, 25, seed=20, spread=0.08)
        t0 = time.perf_counter()
        oracle.render_keypoints(f, kp, "BODY_25", threshold=0.05)
        dt = time.perf_counter() - t0
        row = {"case": "cpu_oracle_pose_keypoints_20p", "seconds": round(dt, 3), "cores": 1}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as fo:
            json.dump(rows, fo, indent=1)


if __name__ == "__main__":
    main()
