"""fp16-storage emulation of the Caffe pose CNNs -- TEST INFRASTRUCTURE ONLY (see oracle.h).

What it restates: the arithmetic contract of the product's conv kernels (NetHip,
openpose_amd/csrc/kernels/conv*.hip) for the layers of models/pose/body_25/pose_deploy.prototxt as
Caffe runs them (ConvolutionLayer + bias, ReLU / PReLU in place, MAX pooling, Concat; netCaffe.cpp:
212-261 drives them): every activation a conv reads is the fp16 value stored in HBM, weights are
fp16, the products and sums are fp32 (fp16 x fp16 products are exact in fp32), bias and PReLU
slopes are fp32, and the result is rounded to fp16 (round to nearest even) where the kernel stores
it -- except the net_output blob, written in fp32.  A 2x2 max pool of fp16 values is exact.

Only the summation ORDER is left open (the MFMA's internal order is the hardware's), so a kernel's
output is compared with this emulation through a per-element bound instead of bit equality:

    |gpu - ref| <= 2 ulp16(ref) + C * S,   S = sum_k |w_k x_k| + |b|   (same conv with |w|, |x|)

ulp16(v) is the fp16 spacing at |v| (2^-24 below 2^-14).  The first term is the output rounding
(1 ulp) plus one more ulp for the case where the fp32 sums of two orders straddle a rounding
boundary; the second bounds the fp32 summation-order difference, which the ulp term cannot cover
where the sum cancels (|ref| << S).  C is stated where the bound is used (tests/test_gpu_layers.py)
and is set from measurement with headroom.  A fused kernel that keeps an fp16 intermediate on chip
(conv1_1 -> conv1_2, Mconv6 -> Mconv7) is emulated the same way, the intermediate rounded to fp16.
"""
import numpy as np

from . import conv2d, maxpool


def f16(a):
    """Round to fp16 (RNE, with subnormals) and back: the value an fp16 buffer holds."""
    return np.asarray(a, np.float32).astype(np.float16).astype(np.float32)


def ulp16(v):
    """Spacing of fp16 at |v| (2^-24 in the subnormal range)."""
    a = np.maximum(np.abs(np.asarray(v, np.float32)), np.float32(2.0 ** -14))
    return np.exp2(np.floor(np.log2(a)) - 10).astype(np.float32)


def _act(t, act, slope):
    if act == 1:
        return np.maximum(t, np.float32(0))
    if act == 2:
        s = np.asarray(slope, np.float32).reshape(1, -1, 1, 1)
        return np.where(t > 0, t, t * s).astype(np.float32)
    return t


def conv(x16, params, layer, nthreads=None, need_s=True):
    """One conv as the kernels compute it: x16 holds fp16 values (fp32 array), weights rounded to
    fp16; returns (activation output before the store's rounding, S or None)."""
    w, b, slope = params[layer["name"]]
    w16 = f16(w)
    b = np.asarray(b, np.float32)
    pad = layer["pad"]
    t = conv2d(x16, w16, b, pad, nthreads)
    s = conv2d(np.abs(x16), np.abs(w16), np.abs(b), pad, nthreads) if need_s else None
    return _act(t, layer.get("act", 0), slope), s


def annotate(graph):
    """conv layers of a graph with their fused activation ("act": 0 / 1 ReLU / 2 PReLU), by name,
    and the consumers of every top (for which stores are fp16 and which net_output only)."""
    convs, consumers = {}, {}
    for i, l in enumerate(graph):
        for b in l["bottom"]:
            consumers.setdefault(b, []).append(l)
        if l["type"] == "Convolution":
            c = dict(l)
            c["act"] = 0
            nxt = graph[i + 1] if i + 1 < len(graph) else None
            if nxt is not None and nxt["type"] in ("ReLU", "PReLU") and nxt["bottom"] == [l["top"][0]]:
                c["act"] = 1 if nxt["type"] == "ReLU" else 2
            convs[l["name"]] = c
    return convs, consumers


def unit_from_launch(graph, layer_field):
    """Kernel unit of a launch-log layer field (NetHip::forward_steps): "A" (one conv), "A+pool"
    (conv + its 2x2 pool in the epilogue), "A+B" (a fused 1x1 head pair), "A+B+pool" (the fused
    first layers).  Returns dict(convs=[...], pool=pool layer or None, input=blob, output=blob)."""
    convs, consumers = annotate(graph)
    parts = layer_field.split("+")
    pool = parts[-1] == "pool"
    names = parts[:-1] if pool else parts
    cl = [convs[n] for n in names]
    out = cl[-1]["top"][0]
    pl = None
    if pool:
        pl = [c for c in consumers[out] if c["type"] == "Pooling"]
        assert len(pl) == 1, layer_field
        pl = pl[0]
        out = pl["top"][0]
    return dict(convs=cl, pool=pl, input=cl[0]["bottom"][0], output=out,
                fp32_output=all(c["type"] == "Concat" and c["top"][0] == "net_output"
                                for c in consumers.get(out, [])) and not pool)


def unit(u, x, params, c_acc, nthreads=None):
    """Emulated output of a kernel unit for input blob values x (fp32 array of fp16 values, or the
    fp32 image for a first conv: rounded here as the kernels convert it).  Returns (ref, tol): the
    stored value (fp16-rounded unless the output is net_output only) and the per-element bound."""
    y = f16(x)
    for i, c in enumerate(u["convs"]):
        t, s = conv(y, params, c, nthreads)
        last = i == len(u["convs"]) - 1
        if not last:
            y = f16(t)
            continue
        if u["fp32_output"]:
            ref = t
            tol = np.float32(c_acc) * s + np.abs(t) * np.float32(2.0 ** -22)
        else:
            ref = f16(t)
            tol = 2 * ulp16(ref) + np.float32(c_acc) * s
    if u["pool"] is not None:
        ref = maxpool(ref, u["pool"]["kernel_size"], u["pool"]["stride"])
        tol = maxpool(tol, u["pool"]["kernel_size"], u["pool"]["stride"])
    return ref, tol


def forward(x, params, graph, nthreads=None):
    """Whole-net emulation (every stored activation fp16, net_output fp32): x [n, 3, h, w]."""
    convs, _ = annotate(graph)
    blobs = {"image": np.ascontiguousarray(x, np.float32)}
    for l in graph:
        t = l["type"]
        if t == "Convolution":
            v, _ = conv(f16(blobs[l["bottom"][0]]), params, convs[l["name"]], nthreads, False)
            blobs[l["top"][0]] = v          # rounded by its readers (f16 is idempotent)
        elif t == "Pooling":
            blobs[l["top"][0]] = maxpool(f16(blobs[l["bottom"][0]]), l["kernel_size"], l["stride"])
        elif t == "Concat":
            if l["top"][0] == "net_output":
                blobs["net_output"] = np.concatenate([blobs[b] for b in l["bottom"]], axis=1)
            else:
                blobs[l["top"][0]] = np.concatenate([f16(blobs[b]) for b in l["bottom"]], axis=1)
    return blobs["net_output"]
