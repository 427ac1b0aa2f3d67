"""Dev experiment: the bench workload split over S concurrent pipelines (one context, net and pose
extractor per torch stream, B/S frames each) against one pipeline of B frames.  Measures whether a
second stream fills the per-launch prologue / epilogue tails of the persistent conv kernels.

    python tools/two_stream.py [--streams S] [--batch B] [--steps K]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from openpose_amd import synth  # noqa: E402
from openpose_amd.api import Context, Net, PoseExtractor, dev_switches  # noqa: E402


def run(streams, batch, steps, warmup=3):
    pipes = []
    sub = batch // streams
    gen = torch.Generator(device="cuda").manual_seed(7)
    for s in range(streams):
        st = torch.cuda.Stream() if streams > 1 else torch.cuda.current_stream()
        ctx = Context(0, stream=st)
        net = Net(ctx, "builtin:BODY_25")
        net.set_params(synth.he_weights(net.convs(), seed=0, out_scale=0.02))
        pose = PoseExtractor(ctx, net)
        pose.set_input((-1, 368))
        frames = [torch.randint(0, 256, (sub, 720, 1280, 3), generator=gen, device="cuda",
                                dtype=torch.uint8) for _ in range(2)]
        pipes.append((ctx, net, pose, frames))

    def step(i):
        for (_, _, pose, frames) in pipes:
            pose.submit_frames(frames[i % 2])
        for (_, _, pose, _) in pipes:
            if pose.pending() > 1:
                pose.collect()

    def drain():
        for (_, _, pose, _) in pipes:
            while pose.pending() > 0:
                pose.collect()

    for i in range(warmup):
        step(i)
    drain()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    drain()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"streams": streams, "batch": batch, "steps": steps,
            "ms_per_step": round(dt / steps * 1e3, 3), "fps": round(batch * steps / dt, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--streams", type=int, nargs="+", default=[1, 2, 1, 2])
    ap.add_argument("--grid-cus", type=int, default=0, help="GRID_CUS for runs with > 1 stream")
    args = ap.parse_args()
    for s in args.streams:
        if s > 1 and args.grid_cus:
            with dev_switches(GRID_CUS=args.grid_cus):
                r = run(s, args.batch, args.steps)
            r["grid_cus"] = args.grid_cus
        else:
            r = run(s, args.batch, args.steps)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
