"""Microbenchmark of the conv kernels on BODY_25 layer shapes (dev tool, GPU).

Builds a chain graph image -> c0 (3->C) -> L identical convs (C->C, k x k) -> net_output and times
the forward with HIP events; reports TFLOP/s of the identical convs (c0 subtracted via a
chain with L=1).  python tools/conv_bench.py [--frames 16] [--iters 10]
"""
import argparse
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpose_amd import synth  # noqa: E402
from openpose_amd.api import Context, Net  # noqa: E402
from tests import prototxt  # noqa: E402


def chain(c, k, n):
    L = [dict(name="c0", type="Convolution", bottom=["image"], top=["c0"], num_output=c,
              kernel_size=3, pad=1),
         dict(name="r0", type="PReLU", bottom=["c0"], top=["c0"])]
    prev = "c0"
    for i in range(1, n + 1):
        nm = "c%d" % i
        L.append(dict(name=nm, type="Convolution", bottom=[prev], top=[nm], num_output=c,
                      kernel_size=k, pad=1 if k == 3 else 0))
        L.append(dict(name="r%d" % i, type="PReLU", bottom=[nm], top=[nm]))
        prev = nm
    L.append(dict(name="net_output", type="Concat", bottom=[prev], top=["net_output"]))
    return L


def time_chain(ctx, c, k, n, frames, h, w, iters):
    text = prototxt.emit(chain(c, k, n))
    with tempfile.NamedTemporaryFile("w", suffix=".prototxt", delete=False) as f:
        f.write(text)
    net = Net(ctx, f.name)
    os.unlink(f.name)
    net.set_params(synth.he_weights(prototxt.parse(text), seed=0))
    x = torch.rand((frames, 3, h, w), device="cuda") - 0.5
    for _ in range(3):
        net.forward(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        net.forward(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    net.close()
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cases", default="128:3:46:82,96:3:46:82,256:3:92:164,512:3:46:82,"
                                       "512:1:46:82,64:3:368:656,128:3:184:328")
    a = ap.parse_args()
    ctx = Context(0)
    for case in a.cases.split(","):
        c, k, h, w = map(int, case.split(":"))
        n = 8
        t1 = time_chain(ctx, c, k, 1, a.frames, h, w, a.iters)
        tn = time_chain(ctx, c, k, n + 1, a.frames, h, w, a.iters)
        per = (tn - t1) / n
        flops = 2.0 * a.frames * h * w * c * c * k * k
        print("C=%4d k=%d %4dx%-4d frames=%d: %8.1f us/layer  %7.1f TFLOP/s" %
              (c, k, h, w, a.frames, per * 1e3, flops / (per * 1e-3) / 1e12), flush=True)


if __name__ == "__main__":
    main()
