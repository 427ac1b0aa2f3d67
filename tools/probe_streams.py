"""Probe: do two forwards in flight on two streams fill each other's launch prologues and tails?

Two nets (same synthetic weights, two contexts on two torch streams) run the 130-frame bench
forward (a) one after the other on one stream, (b) side by side, one per stream, and (c) one
130-frame batch as two halves side by side.  Frames per second of each, event-free (host clock
around a synchronised loop).  Usage: probe_streams.py [--precision split] [--iters K]
"""
import argparse
import time

import torch

from openpose_amd import synth
from openpose_amd.api import PRECISION_SPLIT, Context, Net


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp16")
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--batch", type=int, default=130)
    a = ap.parse_args()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    c1, c2 = Context(0, s1), Context(0, s2)
    nets = []
    for c in (c1, c2):
        n = Net(c, "builtin:BODY_25")
        n.set_params(synth.he_weights(n.convs(), seed=0, out_scale=0.02))
        if a.precision == "split":
            n.set_precision(PRECISION_SPLIT)
        nets.append(n)
    B = a.batch
    x = torch.randn(B, 3, 368, 656, device="cuda")
    h1, h2 = B // 2, B - B // 2

    def run(mode):
        if mode == "serial":       # two full batches, one stream
            nets[0].forward(x)
            nets[0].forward(x)
        elif mode == "pair":       # two full batches, two streams
            nets[0].forward(x)
            nets[1].forward(x)
        elif mode == "halves":     # one batch as two halves, two streams (two batches per iter)
            for _ in range(2):
                nets[0].forward(x[:h1])
                nets[1].forward(x[h1:])

    res = {}
    for mode in ("serial", "pair", "halves", "serial", "pair", "halves"):
        run(mode)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            run(mode)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        fps = 2 * B * a.iters / dt
        res.setdefault(mode, []).append(fps)
        print(f"{a.precision} {mode:7s} {fps:8.1f} frames/s  ({1e3 * dt / (2 * a.iters):.2f} ms per batch)",
              flush=True)
    print({k: round(max(v), 1) for k, v in res.items()})


if __name__ == "__main__":
    main()
