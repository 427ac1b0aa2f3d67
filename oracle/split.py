"""Split-precision bound for one conv launch -- TEST INFRASTRUCTURE ONLY (see oracle.h).

What it restates: the arithmetic contract of the product's split-precision conv kernels
(ConvArgs::split, openpose_amd/csrc/kernels/conv.h; NetHip precision OPK_PRECISION_SPLIT) for the
layers of models/pose/body_25/pose_deploy.prototxt as Caffe runs them (ConvolutionLayer + bias,
ReLU / PReLU in place; netCaffe.cpp:212-261): every activation is held as an fp16 pair
(hi, lo) whose sum the next conv reads; the weights of a layer are scaled by 2^e and held as
w_hi + w_lo; the kernel sums x_hi w_hi + x_lo w_hi + x_hi w_lo in fp32 (each product exact),
scales by 2^-e, adds the bias, applies the activation and stores hi = fp16(v), lo = fp16(v - hi).

So against the exact (float64) convolution of the input the kernel actually read (the GPU's own
hi + lo blob, exact in fp32) with the fp32 weights, a launch's output may differ by

    |gpu - ref| <= C * S + 2^-21 |ref| + 2^-24,   S = sum_k |w_k x_k| + |b|

C * S covers the fp32 accumulation (one rounding per 32-term MFMA step, at most 3 * K / 32 of
them; C is stated where the bound is used), the dropped x_lo w_lo term (<= 2^-24 S) and the
weight pair's residue (<= 2^-23 S); 2^-21 |ref| + 2^-24 the stored pair's residue (lo rounded to
fp16, subnormal near zero).  A missing or misplaced pass leaves errors of ~2^-11 S, a wrong lane or
tap O(S): neither fits.
"""
import numpy as np


def _conv64(x, w, b, pad):
    import torch
    import torch.nn.functional as F
    xt = torch.from_numpy(np.ascontiguousarray(x, np.float64))
    wt = torch.from_numpy(np.ascontiguousarray(w, np.float64))
    bt = torch.from_numpy(np.ascontiguousarray(b, np.float64))
    return F.conv2d(xt, wt, bt, padding=pad).numpy()


def _act64(t, act, slope):
    if act == 1:
        return np.maximum(t, 0.0)
    if act == 2:
        s = np.asarray(slope, np.float32).astype(np.float64).reshape(1, -1, 1, 1)
        return np.where(t > 0, t, t * s)
    return t


def _maxpool64(x, k, st):
    """Caffe MAX pooling (ceil sizing, pad 0) in float64."""
    n, c, h, w = x.shape
    oh, ow = -(-(h - k) // st) + 1, -(-(w - k) // st) + 1
    out = np.full((n, c, oh, ow), -np.inf)
    for dy in range(k):
        for dx in range(k):
            v = x[:, :, dy::st, dx::st][:, :, :oh, :ow]
            out[:, :, :v.shape[2], :v.shape[3]] = np.maximum(out[:, :, :v.shape[2], :v.shape[3]], v)
    return out


def unit(u, x, params, c_acc):
    """Reference and per-element bound of a launch unit (oracle/fp16.py unit_from_launch: one conv,
    one conv + its 2x2 max pool in the epilogue, or a fused 1x1 head pair Mconv6 + Mconv7) for the
    input blob values x (fp32: the GPU's hi + lo, or the fp32 image, which the first conv splits
    itself).  A pooled unit: the max of the reference and of the bound over each window (the
    kernel's pair maximum is within the bound of the exact maximum).  A head pair: Mconv6's value
    never leaves the chip but is split into the same (hi, lo) pair a stored blob holds, so its
    bound (times the activation's Lipschitz constant) propagates through |w7|."""
    assert len(u["convs"]) in (1, 2), "split precision runs single convs and head pairs"
    x = np.asarray(x, np.float32)
    err = None   # bound on the error of the current input (None: exact)
    for i, c in enumerate(u["convs"]):
        w, b, slope = params[c["name"]]
        last = i == len(u["convs"]) - 1
        t = _act64(_conv64(x, w, b, c["pad"]), c.get("act", 0), slope)
        s = _conv64(np.abs(x), np.abs(w), np.abs(b), c["pad"])
        if err is not None:   # the input's own error through |w|
            s = s + _conv64(err, np.abs(w), np.zeros_like(b), c["pad"])
            prop = _conv64(err, np.abs(w), np.zeros_like(b), c["pad"])
        else:
            prop = 0.0
        if last and u["fp32_output"]:   # net_output: the fp32 activation, no pair
            tol = c_acc * s + prop + np.abs(t) * 2.0 ** -22 + 2.0 ** -30
        else:
            tol = c_acc * s + prop + np.abs(t) * 2.0 ** -21 + 2.0 ** -24
        if not last:
            lip = 1.0
            if c.get("act", 0) == 2:
                lip = max(1.0, float(np.max(np.abs(np.asarray(slope, np.float64)))))
            err = tol * lip
            x = t
    if u["pool"] is not None:
        k, st = u["pool"]["kernel_size"], u["pool"]["stride"]
        t, tol = _maxpool64(t, k, st), _maxpool64(tol, k, st)
    return t, tol
