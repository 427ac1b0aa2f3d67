"""CPU: the split-precision bound (oracle/split.py) that test_split_every_launch_within_bound uses.

An independent CPU emulation of the split contract (ConvArgs::split / HeadArgs::split) -- weights
scaled by 2^e and split into w_hi + w_lo, the input as an exact (hi, lo) fp16 pair, the three
products x_hi w_hi + x_lo w_hi + x_hi w_lo summed in fp32, scaled back, bias, activation, the result
stored as a (hi, lo) pair -- must sit inside the bound, and dropping any one product must not: the
bound is what tells a complete split kernel from one that misses a pass.  Covered for a 3x3 conv,
a 3x3 conv + 2x2 pool and a fused 1x1 head pair (Mconv6 + Mconv7, the intermediate split on chip).
"""
import numpy as np
import pytest
import torch

from oracle import split as sp

C_SPLIT = 2.0 ** -19   # tests/test_gpu_layers.py


def _f16(a):
    return np.asarray(a, np.float32).astype(np.float16).astype(np.float32)


def _pair_input(rng, shape):
    """fp32 values that are exactly hi + lo of two fp16 numbers (what a stored blob holds)."""
    x = rng.uniform(-1.0, 1.0, shape).astype(np.float32)
    hi = _f16(x)
    lo = _f16(x - hi)
    return (hi.astype(np.float64) + lo).astype(np.float32), hi, lo


def _conv32(x, w, pad):
    return torch.nn.functional.conv2d(torch.from_numpy(x), torch.from_numpy(w), padding=pad).numpy()


def _split_conv(hi, lo, w, b, slope, act, pad, drop=None):
    """One split conv as the kernels compute it; drop: 0 / 1 / 2 leaves out x_hi w_hi / x_lo w_hi /
    x_hi w_lo.  Returns the fp32 activation v (before the pair split)."""
    mx = float(np.abs(w).max())
    e = 15 - int(np.frexp(mx)[1])
    ws = np.ldexp(w.astype(np.float32), e)
    w_hi = _f16(ws)
    w_lo = _f16(ws - w_hi)
    acc = np.zeros(1, np.float32)
    terms = [(hi, w_hi), (lo, w_hi), (hi, w_lo)]
    for k, (xa, wa) in enumerate(terms):
        if k != drop:
            acc = acc + _conv32(xa, wa, pad)
    t = np.ldexp(acc, -e).astype(np.float32) + b.reshape(1, -1, 1, 1).astype(np.float32)
    if act == 1:
        t = np.maximum(t, 0)
    elif act == 2:
        s = slope.reshape(1, -1, 1, 1).astype(np.float32)
        t = np.where(t > 0, t, t * s)
    return t.astype(np.float32)


def _store_pair(v):
    hi = _f16(v)
    lo = _f16(v - hi)
    return hi, lo


def _params(rng, cout, cin, k, act):
    w = (rng.standard_normal((cout, cin, k, k)) * np.sqrt(2.0 / (cin * k * k))).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, cout).astype(np.float32)
    s = rng.uniform(0.0, 1.0, cout).astype(np.float32) if act == 2 else None
    return w, b, s


def _frac_beyond(got, ref, tol):
    return float((np.abs(got.astype(np.float64) - ref) > tol).mean())


@pytest.mark.parametrize("pool", [False, True])
def test_split_bound_3x3(pool):
    rng = np.random.default_rng(3)
    x, hi, lo = _pair_input(rng, (1, 32, 12, 14))
    w, b, s = _params(rng, 48, 32, 3, 2)
    params = {"c": (w, b, s)}
    u = dict(convs=[dict(name="c", pad=1, act=2)], pool=None, fp32_output=False)
    if pool:
        u["pool"] = dict(kernel_size=2, stride=2)
    ref, tol = sp.unit(u, x, params, C_SPLIT)
    for drop in (None, 0, 1, 2):
        v = _split_conv(hi, lo, w, b, s, 2, 1, drop)
        ph, pl = _store_pair(v)
        got = ph.astype(np.float64) + pl
        if pool:   # the pair with the larger hi + lo per window
            got = torch.nn.functional.max_pool2d(torch.from_numpy(got), 2, 2, ceil_mode=True).numpy()
        frac = _frac_beyond(got, ref, tol)
        if drop is None:
            assert frac == 0.0, frac
        else:
            assert frac > 0.2, (drop, frac)


def test_split_bound_head_pair():
    """Mconv6 (1x1, PReLU) -> Mconv7 (1x1): the intermediate split into the stored pair on chip,
    Mconv7 as v_hi w7_hi + v_lo w7_hi + v_hi w7_lo; a missing Mconv7 w_lo pass is caught."""
    rng = np.random.default_rng(5)
    x, hi, lo = _pair_input(rng, (1, 64, 10, 12))
    w6, b6, s6 = _params(rng, 96, 64, 1, 2)
    w7, b7, _ = _params(rng, 20, 96, 1, 0)
    params = {"m6": (w6, b6, s6), "m7": (w7, b7, None)}
    u = dict(convs=[dict(name="m6", pad=0, act=2), dict(name="m7", pad=0, act=0)], pool=None,
             fp32_output=False)
    ref, tol = sp.unit(u, x, params, C_SPLIT)
    v6 = _split_conv(hi, lo, w6, b6, s6, 2, 0)
    h6, l6 = _store_pair(v6)
    for drop in (None, 2):
        v7 = _split_conv(h6, l6, w7, b7, None, 0, 0, drop)
        ph, pl = _store_pair(v7)
        frac = _frac_beyond(ph.astype(np.float64) + pl, ref, tol)
        if drop is None:
            assert frac == 0.0, frac
        else:
            assert frac > 0.2, frac
    # the fp32 net-output form of the same unit (no pair at the end)
    u["fp32_output"] = True
    ref32, tol32 = sp.unit(u, x, params, C_SPLIT)
    v7 = _split_conv(h6, l6, w7, b7, None, 0, 0)
    assert _frac_beyond(v7, ref32, tol32) == 0.0
