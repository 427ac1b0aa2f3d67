"""CPU: the fp16-storage emulation (oracle/fp16.py) that the per-layer GPU test relies on.

* every unit's bound holds against an independent float64 evaluation of the same fp16 contract
  (torch CPU conv2d in float64 on the fp16 values, rounded at the same points) -- the emulation
  and its bound do not depend on the C oracle's summation order;
* the bound is tight enough to catch a wrong value: perturbing one output element by a few % of
  its magnitude, or using the partner column's value in a 2x2 pool, is detected;
* the launch-log layer fields of the BODY_25 forward map onto the right units.
"""
import numpy as np
import pytest
import torch

from oracle import body25
from oracle import fp16 as emu
from openpose_amd import synth


def _f64_unit(u, x, params):
    """The same contract in float64 (torch conv2d), fp16 rounding at the stores."""
    y = torch.from_numpy(emu.f16(x).astype(np.float64))
    for i, c in enumerate(u["convs"]):
        w, b, s = params[c["name"]]
        w16 = torch.from_numpy(emu.f16(w).astype(np.float64))
        t = torch.nn.functional.conv2d(y, w16, torch.from_numpy(b.astype(np.float64)),
                                       padding=c["pad"])
        if c["act"] == 1:
            t = torch.clamp(t, min=0)
        elif c["act"] == 2:
            t = torch.where(t > 0, t, t * torch.from_numpy(s.astype(np.float64)).view(1, -1, 1, 1))
        if i < len(u["convs"]) - 1 or not u["fp32_output"]:
            t = torch.from_numpy(t.numpy().astype(np.float32).astype(np.float16).astype(np.float64))
        y = t
    if u["pool"] is not None:
        y = torch.nn.functional.max_pool2d(y, 2, 2, ceil_mode=True)
    return y.numpy()


def _params(graph, seed):
    p = synth.he_weights(graph, seed=seed)
    rng = np.random.default_rng(seed)
    return {k: (w, rng.normal(0, 0.05, b.shape).astype(np.float32),
                None if s is None else rng.uniform(0.05, 0.5, s.shape).astype(np.float32))
            for k, (w, b, s) in p.items()}


UNITS = ["conv1_1+conv1_2+pool", "conv2_1", "conv2_2+pool", "conv4_2", "Mconv1_stage0_L2_0",
         "Mconv6_stage0_L2+Mconv7_stage0_L2", "Mconv6_stage1_L1+Mconv7_stage1_L1"]


@pytest.mark.parametrize("layer", UNITS)
def test_unit_bound_holds_against_float64(layer):
    graph = body25.layers()
    params = _params(graph, 5)
    u = emu.unit_from_launch(graph, layer)
    cin = {l["name"]: l["cin"] for l in graph if l["type"] == "Convolution"}[u["convs"][0]["name"]]
    rng = np.random.default_rng(6)
    h, w = (24, 40) if u["input"] == "image" else (12, 20)
    x = rng.uniform(-0.5, 0.5, (1, cin, h, w)).astype(np.float32)
    if u["input"] != "image":   # activations after a ReLU / PReLU: mostly positive, fp16 values
        x = emu.f16(np.abs(x) * 2)
    chained = len(u["convs"]) > 1
    ref, tol = emu.unit(u, x, params, 2.0 ** -14 if chained else 2.0 ** -16, nthreads=2)
    exact = _f64_unit(u, x, params)
    d = np.abs(exact - ref)
    assert (d <= tol).all(), (layer, float((d - tol).max()))
    # one conv: within 2 ulp16 where the sum does not cancel (a chained kernel's intermediate
    # rounding may flip and move the second conv's sum by more)
    big = np.abs(ref) > 0.05
    if not u["fp32_output"] and not chained:
        assert (d[big] <= 2 * emu.ulp16(ref[big])).all()


def test_bound_detects_wrong_values():
    graph = body25.layers()
    params = _params(graph, 7)
    u = emu.unit_from_launch(graph, "conv2_2+pool")
    x = emu.f16(np.random.default_rng(8).uniform(0, 1, (1, 128, 16, 24)).astype(np.float32))
    ref, tol = emu.unit(u, x, params, 2.0 ** -16, nthreads=2)
    # one element off by 2 % of its value
    i = np.unravel_index(np.argmax(np.abs(ref)), ref.shape)
    bad = ref.copy()
    bad[i] *= np.float32(1.02)
    assert np.abs(bad - ref)[i] > tol[i]
    # the pool taking a neighbour column's pair instead of its own (a wrong DPP partner)
    u_np = dict(u, pool=None)
    pre, _ = emu.unit(u_np, x, params, 2.0 ** -16, nthreads=2)
    rows = np.maximum(emu.f16(pre[:, :, 0::2, :]), emu.f16(pre[:, :, 1::2, :]))
    wrong = np.maximum(rows[..., 0::2], np.roll(rows, -2, axis=-1)[..., 0::2])   # column 2k+2, not 2k+1
    frac_caught = float((np.abs(wrong - ref) > tol).mean())
    assert frac_caught > 0.2


def test_layer_fields_of_the_body25_forward():
    graph = body25.layers()
    u = emu.unit_from_launch(graph, "conv1_1+conv1_2+pool")
    assert u["input"] == "image" and u["output"] == "pool1_stage1" and len(u["convs"]) == 2
    u = emu.unit_from_launch(graph, "conv3_4+pool")
    assert u["input"] == "conv3_3" and u["output"] == "pool3_stage1"
    u = emu.unit_from_launch(graph, "Mconv6_stage3_L2+Mconv7_stage3_L2")
    assert u["input"] == "Mconv5_stage3_L2_concat" and u["output"] == "Mconv7_stage3_L2"
    assert not u["fp32_output"]          # also read by the L1 stages' concats (fp16 slices)
    u = emu.unit_from_launch(graph, "Mconv6_stage1_L1+Mconv7_stage1_L1")
    assert u["fp32_output"]              # net_output only
    u = emu.unit_from_launch(graph, "Mconv2_stage1_L1_1")
    assert u["input"] == "Mconv2_stage1_L1_0" and [c["act"] for c in u["convs"]] == [2]


def test_whole_net_emulation_close_to_fp32():
    """fp16 storage changes the BODY_25 output by about the fp16 rounding (rel-L2 ~1e-3), not more."""
    graph = body25.layers()
    params = _params(graph, 9)
    x = np.random.default_rng(10).uniform(-0.5, 0.5, (1, 3, 64, 96)).astype(np.float32)
    a = emu.forward(x, params, graph, nthreads=4)
    b = body25.forward(x, params, graph=graph, nthreads=4)
    err = float(np.linalg.norm(a - b) / np.linalg.norm(b))
    assert 1e-5 < err < 5e-3, err
