"""CPU: the resize and Caffe-layer restatements against independent fp32 references (torch CPU).

torch's bicubic (align_corners=False) uses the same Keys kernel (A = -0.75), the same
(d + 0.5) * scale - 0.5 source mapping and replicated border taps as OpenCV's INTER_CUBIC, so it is
an independent check of oracle/resize.c up to summation order (1e-5).  Caffe layers are checked
against torch conv2d / max_pool2d(ceil_mode=True).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle


@pytest.mark.parametrize("sh,sw,dh,dw", [(46, 82, 368, 656), (10, 20, 80, 160), (7, 5, 31, 47),
                                         (40, 40, 20, 25), (34, 60, 368, 656)])
def test_resize_vs_torch_bicubic(sh, sw, dh, dw):
    src = np.random.default_rng(sh * 100 + sw).normal(0, 1, (sh, sw)).astype(np.float32)
    got = oracle.resize_cubic(src, dh, dw)
    ref = F.interpolate(torch.from_numpy(src)[None, None], size=(dh, dw), mode="bicubic",
                        align_corners=False)[0, 0].numpy()
    # torch forms the source coordinate in float, OpenCV in double: ~1e-5 differences
    np.testing.assert_allclose(got, ref, atol=6e-5, rtol=1e-5)


def test_resize_constant_and_tables():
    src = np.full((5, 7), 0.3, np.float32)
    got = oracle.resize_cubic(src, 40, 56)
    np.testing.assert_allclose(got, 0.3, atol=1e-6)
    ofs, coef = oracle.cubic_tables(46, 368)
    assert ofs[0] == -1 and ofs[-1] == 45          # floor((0.5)/8 - 0.5), floor((367.5)/8 - 0.5)
    np.testing.assert_allclose(coef.sum(1), 1.0, atol=1e-6)


def test_resize_merge_average():
    rng = np.random.default_rng(5)
    a = rng.normal(0, 1, (2, 10, 20)).astype(np.float32)
    b = rng.normal(0, 1, (2, 5, 10)).astype(np.float32)
    got = oracle.resize_merge([a, b], 40, 80)
    ra = oracle.resize_merge([a], 40, 80)
    rb = oracle.resize_merge([b], 40, 80)
    np.testing.assert_allclose(got, (ra + rb) * np.float32(0.5), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("ci,co,k,h,w", [(3, 16, 3, 13, 17), (32, 24, 3, 9, 30), (40, 8, 1, 7, 7),
                                         (64, 5, 3, 4, 70)])
def test_conv2d_vs_torch(ci, co, k, h, w):
    rng = np.random.default_rng(ci + co)
    x = rng.normal(0, 1, (2, ci, h, w)).astype(np.float32)
    wt = rng.normal(0, 0.1, (co, ci, k, k)).astype(np.float32)
    b = rng.normal(0, 0.1, co).astype(np.float32)
    got = oracle.conv2d(x, wt, b, pad=k // 2, nthreads=2)
    ref = F.conv2d(torch.from_numpy(x), torch.from_numpy(wt), torch.from_numpy(b), padding=k // 2)
    np.testing.assert_allclose(got, ref.numpy(), rtol=1e-4, atol=1e-4)


def test_prelu_relu_maxpool():
    rng = np.random.default_rng(9)
    x = rng.normal(0, 1, (2, 3, 9, 11)).astype(np.float32)
    s = np.float32([0.25, 0.1, 0.5])
    got = oracle.prelu(x.copy(), s)
    ref = F.prelu(torch.from_numpy(x), torch.from_numpy(s)).numpy()
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(oracle.relu(x.copy()), np.maximum(x, 0))
    mp = oracle.maxpool(x)                            # ceil sizing: 9x11 -> 5x6
    ref = F.max_pool2d(torch.from_numpy(x), 2, 2, ceil_mode=True).numpy()
    assert mp.shape == (2, 3, 5, 6)
    np.testing.assert_array_equal(mp, ref)
