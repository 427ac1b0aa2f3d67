"""dev: numerics of a Winograd F(2,3)-along-x formulation of the BODY_25 3x3 convs in fp16 (CPU).

    python tools/wino_numerics.py [N H W]

Evaluates the net three ways with torch on the CPU, all against the fp32 forward:
  direct  -- fp16 activations and weights, fp32 accumulation (what the MFMA kernels compute);
  wino    -- the same, but every 3x3 conv (except conv1_1) as F(2,3) along x: input transforms
             t0 = d0-d2, t1 = d1+d2, t2 = d2-d1, t3 = d1-d3 rounded to fp16, weight transforms
             U0 = g0, U1 = (g0+g1+g2)/2, U2 = (g0-g1+g2)/2, U3 = g2 (fp32, rounded to fp16),
             fp32 products summed over (ci, ky), out(2j) = M0+M1+M2, out(2j+1) = M1-M2-M3.
Prints the relative L2 error of net_output of each (the GPU test bar is 5e-3).
"""
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from oracle import body25  # noqa: E402
from openpose_amd import synth  # noqa: E402


def h16(t):
    return t.half().float()


def wino_conv(x, w, b):
    """x [N,C,H,W] (fp16 values), w [co,ci,3,3] fp32 -> fp32 [N,co,H,W]"""
    n, c, h, wd = x.shape
    assert wd % 2 == 0
    xp = F.pad(x, (1, 1, 1, 1))
    d = [xp[..., k:k + wd:2] for k in range(4)]   # d_k[.., y, j] = xp[.., y, 2j+k]
    t = [h16(d[0] - d[2]), h16(d[1] + d[2]), h16(d[2] - d[1]), h16(d[1] - d[3])]
    g0, g1, g2 = w[..., 0:1], w[..., 1:2], w[..., 2:3]
    U = [h16(g0), h16((g0 + g1 + g2) * 0.5), h16((g0 - g1 + g2) * 0.5), h16(g2)]
    M = [F.conv2d(t[i], U[i]) for i in range(4)]  # [N,co,H,W/2] (valid in y: H+2 -> H)
    out = torch.empty((n, w.shape[0], h, wd))
    out[..., 0::2] = M[0] + M[1] + M[2]
    out[..., 1::2] = M[1] - M[2] - M[3]
    return out + b.view(1, -1, 1, 1)


def forward(graph, params, x, mode):
    blobs = {"image": torch.from_numpy(x)}
    producer = {}
    for l in graph:
        t = l["type"]
        if t == "Convolution":
            producer[l["top"][0]] = l["name"]
            w, b = (torch.from_numpy(np.asarray(a)) for a in params[l["name"]][:2])
            inp = blobs[l["bottom"][0]]
            if mode == "fp32":
                y = F.conv2d(inp, w, b, padding=l["pad"])
            elif mode == "wino" and l["kernel_size"] == 3 and l["name"] != "conv1_1":
                y = wino_conv(h16(inp), w, b)
            else:
                y = F.conv2d(h16(inp), h16(w), b, padding=l["pad"])
            blobs[l["top"][0]] = y
        elif t == "ReLU":
            blobs[l["top"][0]] = torch.relu(blobs[l["bottom"][0]])
        elif t == "PReLU":
            s = torch.from_numpy(np.asarray(params[producer[l["bottom"][0]]][2]))
            blobs[l["top"][0]] = F.prelu(blobs[l["bottom"][0]], s)
        elif t == "Pooling":
            blobs[l["top"][0]] = F.max_pool2d(blobs[l["bottom"][0]], 2, 2, ceil_mode=True)
        elif t == "Concat":
            blobs[l["top"][0]] = torch.cat([blobs[b] for b in l["bottom"]], 1)
    return blobs["net_output"]


def main():
    n, h, w = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (2, 64, 96)
    torch.set_num_threads(8)
    graph = body25.layers()
    for seed in (3, 13):
        params = synth.he_weights(graph, seed=seed)
        x = np.random.default_rng(seed + 1).uniform(-0.5, 0.5, (n, 3, h, w)).astype(np.float32)
        with torch.no_grad():
            ref = forward(graph, params, x, "fp32")
            for mode in ("direct", "wino"):
                got = forward(graph, params, x, mode)
                err = float((got - ref).norm() / ref.norm())
                ch = ((got - ref).flatten(2).norm(dim=2) / ref.flatten(2).norm(dim=2)).max()
                print("seed %d %dx%dx%d %-6s rel-L2 %.3e  worst channel %.3e" % (seed, n, h, w, mode, err, ch))


if __name__ == "__main__":
    main()
