"""CPU timing of the people assembly (connectBodyPartsGpu host half) on a synthetic BODY_135 or
BODY_25 frame: oracle peaks + dense pair scores, then the library's opk_assemble_people_semantics
(CONNECT_GPU) timed single-threaded.  Host-only: runs here, no GPU.

    python tools/time_assembly.py [--model body135|body25] [--people 20] [--reps 50]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import oracle  # noqa: E402  (checker only: makes the inputs, never timed)
from openpose_amd import synth  # noqa: E402
from openpose_amd.api import assemble_people, pose_model_info  # noqa: E402
from openpose_amd.pose_tables import BODY_25, BODY_135, CONNECT_GPU  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="body135")
    ap.add_argument("--people", type=int, default=20)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--seed", type=int, default=7000)
    args = ap.parse_args()
    model = {"body135": BODY_135, "body25": BODY_25}[args.model]
    t = pose_model_info(model)
    tab = next(v for v in oracle.pose_tables() if v["id"] == model)
    C = t["parts"] + int(t["bkg"]) + len(t["map_idx"])
    H, W = 368, 656
    f = synth.overlay(args.people, H // 8, W // 8, seed=args.seed, table=t).astype(np.float32)
    f += np.random.default_rng(0).normal(0, 0.01, (C, H // 8, W // 8)).astype(np.float32)
    heat = oracle.resize_merge([f], H, W)
    peaks = oracle.nms(heat, 0.05, 128, channels=t["parts"], cuda=True)
    ps = oracle.pair_scores_table(heat, peaks, tab)
    counts = peaks[:, 0, 0].astype(int)
    print(f"peaks/part mean {counts.mean():.1f} max {counts.max()}, nonzero scores "
          f"{int((ps > 0).sum())}")
    kp, ks = assemble_people(ps, peaks, pose_model=model, semantics=CONNECT_GPU)
    ref = oracle.connect_gpu_semantics(ps, peaks, tab)
    same = kp.shape == ref[0].shape and np.array_equal(kp, ref[0]) and np.array_equal(ks, ref[1])
    print(f"people {kp.shape[0]} (oracle {ref[0].shape[0]}), identical {same}")
    t0 = time.perf_counter()
    for _ in range(args.reps):
        assemble_people(ps, peaks, pose_model=model, semantics=CONNECT_GPU)
    dt = (time.perf_counter() - t0) / args.reps
    print(f"assembly {dt * 1e3:.3f} ms/frame (single thread, includes the ctypes call)")


if __name__ == "__main__":
    main()
