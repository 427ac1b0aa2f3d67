"""GPU parity of the BODY_25 CNN (NetHip, MFMA fp16 / fp32 accumulate) vs the fp32 Caffe-semantics
oracle (oracle/caffe_cpu.c) on identical inputs and seeded weights.

Tolerance (floating point, north_star: outputs within a stated float tolerance): fp16 operands give
~2^-11 relative rounding per operand; the bar below is relative L2 error of the net output.
"""
import os
import tempfile

import numpy as np
import pytest
import torch

import oracle
from oracle import body25
from openpose_amd import synth
from openpose_amd.api import Net
from tests import prototxt

pytestmark = pytest.mark.gpu

SMALL_TOL = 4e-3      # relative L2, graphs of <= 6 layers
BODY25_TOL = 2e-2     # relative L2, the full 114-conv network


def rel_l2(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-30))


def conv(name, bottom, cout, k, act=None):
    out = [dict(name=name, type="Convolution", bottom=[bottom], top=[name], num_output=cout,
                kernel_size=k, pad=1 if k == 3 else 0)]
    if act:
        out.append(dict(name=act + "_" + name, type="ReLU" if act == "relu" else "PReLU",
                        bottom=[name], top=[name]))
    return out


def run_graph(ctx, layers, x, seed=0):
    text = prototxt.emit(layers)
    graph = prototxt.parse(text)
    params = synth.he_weights(graph, seed=seed)
    with tempfile.NamedTemporaryFile("w", suffix=".prototxt", delete=False) as f:
        f.write(text)
        path = f.name
    try:
        net = Net(ctx, path)
        net.set_params(params)
        net.forward(torch.from_numpy(x).cuda())
        got = net.output_numpy()
        net.close()
    finally:
        os.unlink(path)
    ref = body25.forward(x, params, graph=graph)
    return got, ref


def test_conv_relu_prelu_1x1(ctx):
    L = conv("c1", "image", 64, 3, "relu") + conv("c2", "c1", 96, 3, "prelu") + conv("c3", "c2", 52, 1)
    L.append(dict(name="net_output", type="Concat", bottom=["c3"], top=["net_output"]))
    x = np.random.default_rng(0).uniform(-0.5, 0.5, (2, 3, 24, 40)).astype(np.float32)
    got, ref = run_graph(ctx, L, x)
    assert got.shape == ref.shape
    assert rel_l2(got, ref) < SMALL_TOL


def test_dense_block_concat_and_pool(ctx):
    L = conv("c1", "image", 64, 3, "relu") + conv("c2", "c1", 128, 3, "relu")
    L.append(dict(name="p1", type="Pooling", bottom=["c2"], top=["p1"], kernel_size=2, stride=2))
    L += conv("c3", "p1", 128, 3, "prelu")
    L += conv("a0", "c3", 96, 3, "prelu") + conv("a1", "a0", 96, 3, "prelu") + conv("a2", "a1", 96, 3, "prelu")
    L.append(dict(name="cat", type="Concat", bottom=["a0", "a1", "a2"], top=["cat"]))
    L += conv("m6", "cat", 256, 1, "prelu") + conv("m7", "m6", 26, 1)
    L.append(dict(name="cat2", type="Concat", bottom=["c3", "m7"], top=["cat2"]))
    L += conv("b0", "cat2", 128, 3, "prelu") + conv("b7", "b0", 52, 1)
    L.append(dict(name="net_output", type="Concat", bottom=["m7", "b7"], top=["net_output"]))
    # odd sizes exercise Caffe's ceil pooling
    x = np.random.default_rng(1).uniform(-0.5, 0.5, (3, 3, 37, 51)).astype(np.float32)
    got, ref = run_graph(ctx, L, x)
    assert got.shape == ref.shape == (3, 78, 19, 26)
    assert rel_l2(got, ref) < SMALL_TOL


@pytest.mark.parametrize("n,h,w", [(2, 64, 96), (1, 368, 368)])
def test_body25_vs_oracle(ctx, n, h, w):
    graph = body25.layers()
    params = synth.he_weights(graph, seed=3)
    x = np.random.default_rng(4).uniform(-0.5, 0.5, (n, 3, h, w)).astype(np.float32)
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(params)
    net.forward(torch.from_numpy(x).cuda())
    got = net.output_numpy()
    ref = body25.forward(x, params, graph=graph)
    assert got.shape == ref.shape == (n, 78, h // 8, w // 8)
    err = rel_l2(got, ref)
    print("BODY_25 %dx%dx%d rel-L2 %.3e" % (n, h, w, err))
    assert err < BODY25_TOL


@pytest.mark.parametrize("hw,acts", [((24, 40), ("relu", "relu")), ((26, 130), ("relu", "prelu")),
                                     ((14, 6), ("prelu", "relu"))])
def test_conv1_fused_matches_unfused(ctx, hw, acts):
    """conv1_1 -> conv1_2 -> pool1 in one kernel (conv1_fused.hip) gives the bits of the three
    separate kernels (same MFMA operands and accumulation order, same epilogue, same max)."""
    L = conv("c1", "image", 64, 3, acts[0]) + conv("c2", "c1", 64, 3, acts[1])
    L.append(dict(name="pool1", type="Pooling", bottom=["c2"], top=["pool1"], pool="MAX",
                  kernel_size=2, stride=2))
    L += conv("c3", "pool1", 32, 3, "relu") + conv("c4", "c3", 16, 1)
    L.append(dict(name="net_output", type="Concat", bottom=["c4"], top=["net_output"]))
    x = np.random.default_rng(7).uniform(-0.5, 0.5, (3, 3) + hw).astype(np.float32)
    outs = []
    for fused in ("1", "0"):
        os.environ["OPK_CONV1_FUSED"] = fused
        try:
            got, ref = run_graph(ctx, L, x, seed=3)
        finally:
            os.environ.pop("OPK_CONV1_FUSED", None)
        assert rel_l2(got, ref) < SMALL_TOL
        outs.append(got)
    np.testing.assert_array_equal(outs[0], outs[1])
