"""Heat-map semantics of the reference's CUDA build (OPK_MAPS_CUDA): resizeAndMergeGpu
(src/openpose/net/resizeAndMergeBase.cu, include/openpose_private/gpu/cuda.hu:92-145) and nmsGpu
(src/openpose/net/nmsBase.cu:50-90,161-240) beside the CPU build's (the default).

CPU tests pin the oracle restatements (oracle/resize.c, oracle/nms.c) with known answers derived
from the reference source; GPU tests hold libopk_hip.so to them bit for bit.  Parity with a real
CUDA build is unpinned (no CUDA toolchain here; nvcc's contraction of the cubic polynomial cannot be
reproduced), see include/opk.h OPK_MAPS_CUDA."""
import numpy as np
import pytest

import oracle
from openpose_amd import synth


def catmull_rom64(src, xs, ys):
    """float64 restatement of bicubicInterpolate (clamped base, A = -0.5) for one pixel."""
    h, w = src.shape

    def idx(v, n):
        i1 = min(max(int(np.floor(v)), 0), n - 1)
        return [max(0, i1 - 1), i1, min(n - 1, i1 + 1), min(n - 1, min(n - 1, i1 + 1) + 1)], v - i1

    xi, dx = idx(xs, w)
    yi, dy = idx(ys, h)

    def cub(v, d):
        v0, v1, v2, v3 = v
        return ((-0.5 * v0 + 1.5 * v1 - 1.5 * v2 + 0.5 * v3) * d ** 3 +
                (v0 - 2.5 * v1 + 2 * v2 - 0.5 * v3) * d ** 2 - 0.5 * (v0 - v2) * d + v1)

    return cub([cub([float(src[r, c]) for c in xi], dx) for r in yi], dy)


def test_cuda_resize_constant_and_linear():
    const = np.full((2, 6, 10), 0.75, np.float32)
    np.testing.assert_array_equal(oracle.resize_merge_cuda([const], 48, 80), 0.75)
    # Catmull-Rom reproduces a ramp away from the clamped border: x_src = (x + 0.5) / 8 - 0.5
    ramp = np.broadcast_to(np.arange(10, dtype=np.float32), (1, 6, 10)).copy()
    out = oracle.resize_merge_cuda([ramp], 48, 80)[0]
    x = np.arange(12, 68)
    np.testing.assert_allclose(out[20, x], (x + 0.5) / 8 - 0.5, atol=2e-6)
    # at the left border the base column is clamped to 0 and dx goes negative (cuda.hu:96-101)
    assert out[20, 0] == pytest.approx(catmull_rom64(ramp[0], 0.5 / 8 - 0.5, 20.5 / 8 - 0.5), abs=1e-6)


def test_cuda_resize_matches_float64_restatement():
    rng = np.random.default_rng(1)
    src = rng.normal(size=(1, 7, 9)).astype(np.float32)
    out = oracle.resize_merge_cuda([src], 56, 72)[0]
    for y, x in [(0, 0), (3, 70), (55, 71), (27, 33), (8, 1)]:
        assert out[y, x] == pytest.approx(catmull_rom64(src[0], (x + 0.5) / 8 - 0.5, (y + 0.5) / 8 - 0.5),
                                          abs=2e-5)


def test_cuda_resize_reference_errors_and_identity():
    src = np.random.default_rng(2).normal(size=(1, 6, 10)).astype(np.float32)
    assert oracle.resize_merge_cuda([src], 42, 70) is None        # x7: "only implemented for 8x"
    np.testing.assert_array_equal(oracle.resize_merge_cuda([src], 6, 10), src)   # fillKernel
    assert oracle.resize_merge_cuda([src], 7, 10) is None         # same ratio 1, other size


def test_cuda_multiscale_average():
    """resizeAndAddAndAverageKernel: source i scaled by (W / w0) / (r_i / r_0), sum / N."""
    rng = np.random.default_rng(3)
    a = rng.normal(size=(1, 6, 10)).astype(np.float32)
    b = rng.normal(size=(1, 3, 5)).astype(np.float32)
    ratios = [1.0, 0.5]
    out = oracle.resize_merge_cuda([a, b], 48, 80, ratios)[0]
    for y, x in [(0, 0), (10, 40), (47, 79), (24, 3)]:
        va = catmull_rom64(a[0], (x + 0.5) / 8 - 0.5, (y + 0.5) / 8 - 0.5)
        vb = catmull_rom64(b[0], (x + 0.5) / 16 - 0.5, (y + 0.5) / 16 - 0.5)
        assert out[y, x] == pytest.approx((va + vb) / 2, abs=2e-5)


def test_cuda_nms_rules():
    """nmsRegisterKernel: interior only, strict 8-neighbour maximum; nmsCpu differs on the first
    inner ring (>= with outside = threshold) and on plateaus there."""
    h, w = 12, 16
    f = np.zeros((1, h, w), np.float32)
    f[0, 5, 7] = 0.9                    # ordinary interior peak: both
    f[0, 1, 3] = 0.8                    # first inner ring, strict maximum: both
    f[0, 8, 1] = f[0, 8, 2] = 0.7       # plateau touching column 1: nmsCpu takes (x=1), nmsGpu none
    f[0, 0, 10] = 0.95                  # outer border: neither
    cpu = oracle.nms(f, 0.05, 8, channels=1)
    gpu = oracle.nms(f, 0.05, 8, channels=1, cuda=True)

    def found(p):
        return sorted((int(round(p[0, i, 1])), int(round(p[0, i, 0]))) for i in range(1, int(p[0, 0, 0]) + 1))

    # (8, 1) registers under nmsCpu; its 7x7 centroid lies between the plateau's two pixels
    assert found(cpu) == [(1, 3), (5, 7), (8, 2)] and int(cpu[0, 0, 0]) == 3
    assert cpu[0, 3, 0] == 1.5 and cpu[0, 3, 1] == 8.0
    assert found(gpu) == [(1, 3), (5, 7)]


def test_cuda_nms_centroid_is_fused():
    """The centroid sums are fmaf (nvcc --fmad): the same interior peaks as nmsCpu, positions equal
    to within rounding and bit-different for some fields."""
    rng = np.random.default_rng(4)
    yy, xx = np.mgrid[0:60, 0:90].astype(np.float32)
    diff = 0
    for k in range(20):
        f = np.zeros((1, 60, 90), np.float32)
        for _ in range(4):
            cy, cx = rng.uniform(10, 50), rng.uniform(10, 80)
            f[0] += rng.uniform(0.3, 1.0) * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / rng.uniform(2, 8))
        f = f.astype(np.float32)
        cpu = oracle.nms(f, 0.05, 32, channels=1)
        gpu = oracle.nms(f, 0.05, 32, channels=1, cuda=True)
        n = int(cpu[0, 0, 0])
        assert int(gpu[0, 0, 0]) == n
        np.testing.assert_array_equal(cpu[0, 1:n + 1, 2], gpu[0, 1:n + 1, 2])   # same peaks
        np.testing.assert_allclose(cpu[0, 1:n + 1, :2], gpu[0, 1:n + 1, :2], atol=1e-4)
        diff += int(np.any(cpu[0, 1:n + 1, :2] != gpu[0, 1:n + 1, :2]))
    assert diff > 0


# ---- GPU: libopk_hip.so against the restatements ----------------------------------------------
def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


@pytest.mark.gpu
def test_gpu_cuda_resize_bitexact(ctx):
    import torch
    from openpose_amd.api import MAPS_CUDA
    rng = np.random.default_rng(5)
    src = rng.normal(size=(2, 3, 46, 82)).astype(np.float32)
    out = torch.empty((2, 3, 368, 656), device="cuda")
    ctx.resize_and_merge(out, [_dev(src)], semantics=MAPS_CUDA)
    got = out.cpu().numpy()
    for f in range(2):
        np.testing.assert_array_equal(got[f], oracle.resize_merge_cuda([src[f]], 368, 656))
    # several scales (scaleInputToNetInputs of a 3-scale -1x368 run on 1280x720)
    srcs = [rng.normal(size=(1, 4, 46, 82)).astype(np.float32),
            rng.normal(size=(1, 4, 35, 62)).astype(np.float32),
            rng.normal(size=(1, 4, 23, 41)).astype(np.float32)]
    ratios = [0.5104312, 0.3828234, 0.2552156]
    out = torch.empty((1, 4, 368, 656), device="cuda")
    ctx.resize_and_merge(out, [_dev(s) for s in srcs], semantics=MAPS_CUDA, scale_ratios=ratios)
    np.testing.assert_array_equal(out.cpu().numpy()[0],
                                  oracle.resize_merge_cuda([s[0] for s in srcs], 368, 656, ratios))
    from openpose_amd._lib import OpkError
    with pytest.raises(OpkError):   # x7 single source: the reference's "only 8x" error
        ctx.resize_and_merge(torch.empty((1, 4, 322, 574), device="cuda"), [_dev(srcs[0])],
                             semantics=MAPS_CUDA)


@pytest.mark.gpu
def test_gpu_cuda_nms_bitexact(ctx):
    import torch
    from openpose_amd.api import MAPS_CUDA
    rng = np.random.default_rng(6)
    fields = np.stack([synth.overlay(4, 46, 82, seed=30 + k)[:26] for k in range(2)])
    heat = np.stack([oracle.resize_merge_cuda([fl], 368, 656) for fl in fields])
    heat += rng.normal(0, 0.02, heat.shape).astype(np.float32)
    heat[1, 3, 100:104, 1] = 0.9          # plateau on the first inner column
    peaks = torch.zeros((2, 25, 128, 3), device="cuda")
    ctx.nms(peaks, _dev(heat), 0.05, (0.25, 0.5), semantics=MAPS_CUDA)
    got = peaks.cpu().numpy()
    for f in range(2):
        ref = oracle.nms(heat[f], 0.05, 128, (0.25, 0.5), cuda=True)
        for c in range(25):
            n = int(ref[c, 0, 0])
            assert int(got[f, c, 0, 0]) == n
            np.testing.assert_array_equal(got[f, c, 1:n + 1], ref[c, 1:n + 1])


@pytest.mark.gpu
def test_gpu_pose_pipeline_cuda_maps(ctx):
    """The pose pipeline with OPK_MAPS_CUDA: lazy Catmull-Rom heat maps, nmsGpu rules, PAF samples
    of the same maps, CPU connector -- bit-exact to the oracle chain on injected net outputs."""
    from openpose_amd.api import MAPS_CUDA, PoseExtractor
    fields = np.stack([synth.overlay(k + 2, 46, 82, seed=700 + k) +
                       np.random.default_rng(k).normal(0, 0.01, (78, 46, 82)).astype(np.float32)
                       for k in range(3)]).astype(np.float32)
    pose = PoseExtractor(ctx, None)
    pose.set_map_semantics(MAPS_CUDA)
    net_out = _dev(fields)
    pose.forward_net_output(net_out, (656, 368), (1280, 720))
    s = pose.scale_net_to_output()
    off = float(np.float32(0.5 / np.float64(s)))
    gpu_peaks = pose.peaks_numpy()
    gpu_heat = pose.heatmaps_numpy()
    for k in range(3):
        heat = oracle.resize_merge_cuda([fields[k]], 368, 656)
        np.testing.assert_array_equal(gpu_heat[k], heat)
        peaks = oracle.nms(heat, 0.05, 128, (off, off), cuda=True)
        for c in range(25):
            n = int(peaks[c, 0, 0])
            assert int(gpu_peaks[k, c, 0, 0]) == n
            np.testing.assert_array_equal(gpu_peaks[k, c, 1:n + 1], peaks[c, 1:n + 1])
        rk, rs = oracle.connect(heat, peaks, scale=s)
        kp, ks = pose.keypoints(k)
        assert len(kp) >= 1
        np.testing.assert_array_equal(kp, rk)
        np.testing.assert_array_equal(ks, rs)
