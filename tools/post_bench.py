"""Post-processing microbenchmark (dev tool, GPU): PoseExtractor.forward_net_output on a batch of
synthetic BODY_25 net outputs (people overlay + noise), i.e. lazy resize -> NMS -> PAF -> assembly.

    python tools/post_bench.py [--frames 16] [--iters 20] [--people 5]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpose_amd import synth  # noqa: E402
from openpose_amd.api import Context, PoseExtractor  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--people", type=int, default=5)
    a = ap.parse_args()
    ctx = Context(0)
    pose = PoseExtractor(ctx, None)
    rng = np.random.default_rng(0)
    f = np.stack([synth.overlay(a.people, 46, 82, seed=k) + rng.normal(0, 0.01, (78, 46, 82))
                  for k in range(a.frames)]).astype(np.float32)
    x = torch.from_numpy(f).cuda()
    for _ in range(3):
        pose.forward_net_output(x, (656, 368), (1280, 720))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        pose.forward_net_output(x, (656, 368), (1280, 720))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    print("frames=%d: %.3f ms per batch (%.1f us/frame), people found frame0=%d" %
          (a.frames, dt * 1e3, dt * 1e6 / a.frames, pose.num_people(0)))


if __name__ == "__main__":
    main()
