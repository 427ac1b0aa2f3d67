"""GPU parity: resizeAndMerge / NMS / PAF scores / connector through libopk_hip.so vs the oracle.

Bar: bit-exact (the HIP kernels follow the CPU path's float operation order).
"""
import numpy as np
import pytest
import torch

import oracle
from openpose_amd import pose_tables as pt
from openpose_amd.api import dev_switches
from tests.fields import noise_field, people_field, smooth_noise_field

pytestmark = pytest.mark.gpu


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


def _peaks_equal(gpu, ref):
    """Same count per part and identical (x, y, score) for every valid slot."""
    assert gpu.shape == ref.shape
    for c in range(ref.shape[0]):
        n = int(ref[c, 0, 0])
        assert int(gpu[c, 0, 0]) == n, "part %d: count %d vs %d" % (c, gpu[c, 0, 0], n)
        np.testing.assert_array_equal(gpu[c, 1:n + 1], ref[c, 1:n + 1], err_msg="part %d" % c)


@pytest.mark.parametrize("sh,sw,dh,dw", [(46, 82, 368, 656), (46, 46, 368, 368), (10, 20, 80, 160),
                                         (7, 5, 31, 47), (34, 60, 368, 656), (40, 40, 20, 25)])
def test_resize_single_scale_bitexact(ctx, sh, sw, dh, dw):
    src = smooth_noise_field(2 * 5, sh, sw, seed=sh * 1000 + sw).reshape(2, 5, sh, sw)
    out = torch.empty((2, 5, dh, dw), device="cuda")
    ctx.resize_and_merge(out, [_dev(src)])
    got = out.cpu().numpy()
    for b in range(2):
        ref = oracle.resize_merge([src[b]], dh, dw)
        np.testing.assert_array_equal(got[b], ref)


def test_resize_multiscale_bitexact(ctx):
    # config 4 geometry: 656x368, 480x272, 320x176, 160x80 nets -> outputs /8, merged at 368x656
    shapes = [(46, 82), (34, 60), (22, 40), (10, 20)]
    srcs = [smooth_noise_field(78, h, w, seed=i) for i, (h, w) in enumerate(shapes)]
    out = torch.empty((1, 78, 368, 656), device="cuda")
    ctx.resize_and_merge(out, [_dev(s[None]) for s in srcs])
    ref = oracle.resize_merge(srcs, 368, 656)
    np.testing.assert_array_equal(out.cpu().numpy()[0], ref)


@pytest.mark.parametrize("kind", ["people", "noise", "noise_sorted", "noise_dense"])
def test_nms_bitexact(ctx, kind):
    if kind == "people":
        f = np.stack([people_field(5, 368, 656, seed=s) for s in (1, 2)])
    elif kind == "noise":
        f = np.stack([noise_field(78, 64, 96, seed=s) for s in (3, 4)])
    elif kind == "noise_sorted":   # 128..1024 peaks per part: candidate sort + maxPeaks truncation
        f = np.stack([noise_field(25, 100, 100, seed=s, levels=5, density=1.0) for s in (6, 7)])
    else:   # > 1024 peaks per part (kNmsCandidates): the ordered re-scan fallback
        f = np.stack([noise_field(78, 200, 200, seed=s, levels=5, density=1.0) for s in (5,)])
    n = f.shape[0]
    peaks = torch.zeros((n, 25, 128, 3), device="cuda")
    ctx.nms(peaks, _dev(f), 0.05, (0.25, 0.5))
    got = peaks.cpu().numpy()
    for b in range(n):
        ref = oracle.nms(f[b], 0.05, 128, (0.25, 0.5))
        _peaks_equal(got[b], ref)


def test_nms_tiny_maps(ctx):
    # degenerate widths/heights exercise the overlapping border classes
    for h, w in [(1, 1), (2, 3), (3, 3), (4, 5), (5, 4), (6, 7)]:
        f = noise_field(25, h, w, seed=h * 10 + w, levels=4, density=1.0)
        peaks = torch.zeros((1, 25, 128, 3), device="cuda")
        ctx.nms(peaks, _dev(f[None]), 0.05)
        _peaks_equal(peaks.cpu().numpy()[0], oracle.nms(f, 0.05, 128))


@pytest.mark.parametrize("spl", [1, 0])
def test_paf_scores_bitexact(ctx, spl):
    """Dense pair scores (materialised map: the sources read through L2) against the oracle's
    getScoreAB table, one sample per lane (default) and one line per lane (PAF_SPL=0)."""
    with dev_switches(PAF_SPL=spl):
        _paf_scores_bitexact(ctx)


def _paf_scores_bitexact(ctx):
    f = people_field(6, 368, 656, seed=7)
    pk = oracle.nms(f, 0.05, 128, (0.25, 0.25))
    scores = torch.zeros((1, 26, 127, 127), device="cuda")
    ctx.paf_scores(scores, _dev(f[None]), _dev(pk[None]))
    got = scores.cpu().numpy()[0]
    ref = oracle.pair_scores(f, pk, pt.BODY25_PAIRS, pt.BODY25_MAP_IDX)
    for q in range(26):
        na = int(pk[pt.BODY25_PAIRS[2 * q], 0, 0])
        nb = int(pk[pt.BODY25_PAIRS[2 * q + 1], 0, 0])
        np.testing.assert_array_equal(got[q, :na, :nb], ref[q, :na, :nb], err_msg="pair %d" % q)


@pytest.mark.parametrize("n_people,seed", [(1, 11), (5, 12), (20, 13), (0, 14)])
def test_connect_body_parts_exact(ctx, n_people, seed):
    f = people_field(n_people, 368, 656, seed=seed)
    pk = oracle.nms(f, 0.05, 128, (0.255216, 0.255216))
    kp, ks = ctx.connect_body_parts(_dev(f), _dev(pk), scale=1.959128)
    rk, rs = oracle.connect(f, pk, scale=1.959128)
    np.testing.assert_array_equal(kp, rk)
    np.testing.assert_array_equal(ks, rs)


def test_connect_noise_many_peaks(ctx):
    f = noise_field(78, 120, 160, seed=21, levels=6, density=0.7)
    f[26:] = f[26:] * 2 - 1   # PAF channels in [-1, 1]
    pk = oracle.nms(f, 0.05, 128, (0.25, 0.25))
    kp, ks = ctx.connect_body_parts(_dev(f), _dev(pk))
    rk, rs = oracle.connect(f, pk)
    np.testing.assert_array_equal(kp, rk)
    np.testing.assert_array_equal(ks, rs)
