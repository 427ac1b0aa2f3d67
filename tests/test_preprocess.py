"""Frame -> net input (ScaleAndSizeExtractor + CvMatToOpInput).

CPU: the oracle restatement (oracle/preprocess.c) against known answers from the reference's
configurations (SURVEY.md §8 shape table) and against an independent float evaluation of the same
warp; the product's host-side size/scale logic (opk_scale_and_size, no GPU) against the oracle.
GPU: opk_cvmat_to_input and the raw-frame pose path bit-exact against the oracle.
The arithmetic is OpenCV's (absent here): parity unpinned.
"""
import numpy as np
import pytest

import oracle
from openpose_amd import api


# ---- CPU -----------------------------------------------------------------------------------------

def test_scale_and_size_known_answers():
    # BASELINE configs 2/3: 1280x720 at -1x368 -> 656x368, scaleInputToNetInput 0.5104312
    s, z = oracle.scale_and_size((1280, 720))
    assert z == [(656, 368)] and abs(s[0] - 0.5104312) < 1e-7
    # config 4: --scale_number 4 --scale_gap 0.25 (SURVEY.md §8 shape table)
    _, z = oracle.scale_and_size((1280, 720), scale_number=4, scale_gap=0.25)
    assert z == [(656, 368), (480, 272), (320, 176), (160, 80)]
    # config 1: a 368x368 frame
    s, z = oracle.scale_and_size((368, 368))
    assert z == [(368, 368)] and s[0] == 1.0
    # dynamic behaviour caps the width at 16:9 (portrait and ultra-wide frames)
    assert oracle.scale_and_size((4000, 720))[1] == [(656, 368)]
    assert oracle.scale_and_size((4000, 720), dynamic_behavior=-1)[1] == [(2048, 368)]
    with pytest.raises(ValueError):
        oracle.scale_and_size((1280, 720), net_resolution=(-1, -1))
    with pytest.raises(ValueError):
        oracle.scale_and_size((1280, 720), scale_number=6, scale_gap=0.25)


def test_scale_and_size_product_matches_oracle():
    rng = np.random.default_rng(0)
    for _ in range(300):
        size = (int(rng.integers(16, 4000)), int(rng.integers(16, 3000)))
        res = [(-1, 368), (656, -1), (-1, int(rng.integers(16, 1000))), (int(rng.integers(16, 1000)), -1)][
            int(rng.integers(0, 4))]
        dyn = float(rng.choice([1.0, -1.0, 0.75]))
        sn = int(rng.integers(1, 5))
        gap = float(rng.choice([0.25, 0.1, 0.3]))
        try:
            ref = oracle.scale_and_size(size, res, dyn, sn, gap)
        except ValueError:
            with pytest.raises(api._lib.OpkError):
                api.scale_and_size(size, res, dyn, sn, gap)
            continue
        got = api.scale_and_size(size, res, dyn, sn, gap)
        assert got[1] == ref[1]
        assert got[0] == [float(v) for v in ref[0]]


def test_warp_weight_tables():
    lin = oracle.warp_weight_table(False).astype(np.int64)
    a = np.arange(32)
    # bilinear: exact products (32 - f) * (32 - g) * 32 ...; every entry sums to 32768
    exp = np.zeros((32, 32, 2, 2), np.int64)
    exp[:, :, 0, 0] = np.outer(32 - a, 32 - a) * 32
    exp[:, :, 0, 1] = np.outer(32 - a, a) * 32
    exp[:, :, 1, 0] = np.outer(a, 32 - a) * 32
    exp[:, :, 1, 1] = np.outer(a, a) * 32
    # fraction 0: 1.0 saturates to 32767 and initInterTab2D's correction adds the unit to tap
    # (1, 1) -- the same rounding for every pixel value
    exp[0, 0] = [[32767, 0], [0, 1]]
    np.testing.assert_array_equal(lin, exp)
    v = np.arange(256)
    for v11 in (0, 255):
        assert ((32767 * v + v11 + 16384) >> 15 == v).all()
    cub = oracle.warp_weight_table(True).astype(np.int64)
    assert (cub.sum(axis=(2, 3)) == 32768).all()
    assert cub[0, 0, 1, 1] == 32767 and cub[0, 0, 2, 2] == 1
    # cubic: the rounded outer product of the A = -0.75 kernel; the correction absorbs up to 16
    # half-unit roundings into one tap
    x = a / 32.0
    A = -0.75
    c = np.stack([((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A,
                  ((A + 2) * x - (A + 3)) * x * x + 1,
                  ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1], 1)
    c = np.concatenate([c, 1 - c.sum(1, keepdims=True)], 1)
    ref = np.einsum("ik,jl->ijkl", c, c) * 32768
    assert np.abs(cub - ref).max() <= 8.0


def test_cvmat_identity_and_padding():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    # scale 1, same size: the copy branch of resizeFixedAspectRatio
    out = oracle.cvmat_to_input(img, 1.0, 53, 37)
    np.testing.assert_array_equal(out, img.transpose(2, 0, 1).astype(np.float32) / 256 - 0.5)
    # scale 1 into a larger canvas: zero border (-0.5 after normalisation)
    out = oracle.cvmat_to_input(img, 1.0, 64, 48)
    np.testing.assert_array_equal(out[:, :37, :53], img.transpose(2, 0, 1) / 256.0 - 0.5)
    assert (out[:, 37:, :] == -0.5).all() and (out[:, :, 53:] == -0.5).all()
    raw = oracle.cvmat_to_input(img, 1.0, 53, 37, normalize=0)
    np.testing.assert_array_equal(raw, img.transpose(2, 0, 1).astype(np.float32))


def _float_bilinear(img, scale, dw, dh):
    """Independent float evaluation of the inverse map x / scale (zero border)."""
    h, w, _ = img.shape
    src = np.zeros((h + 2, w + 2, 3))
    src[:h, :w] = img
    ys = np.arange(dh) / scale
    xs = np.arange(dw) / scale
    y0 = np.floor(ys).astype(int)
    x0 = np.floor(xs).astype(int)
    fy = (ys - y0)[:, None, None]
    fx = (xs - x0)[None, :, None]
    ok_y = (y0 >= 0) & (y0 < h + 1)
    ok_x = (x0 >= 0) & (x0 < w + 1)
    y0c = np.clip(y0, 0, h + 1)
    x0c = np.clip(x0, 0, w + 1)
    y1c = np.clip(y0 + 1, 0, h + 1)
    x1c = np.clip(x0 + 1, 0, w + 1)
    v = ((1 - fy) * (1 - fx) * src[y0c][:, x0c] + (1 - fy) * fx * src[y0c][:, x1c]
         + fy * (1 - fx) * src[y1c][:, x0c] + fy * fx * src[y1c][:, x1c])
    return v * ok_y[:, None, None] * ok_x[None, :, None]


def test_cvmat_downscale_close_to_float_bilinear():
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (72, 128, 3), dtype=np.uint8)
    s, [(dw, dh)] = oracle.scale_and_size((128, 72), (-1, 48))
    out = oracle.cvmat_to_input(img, s[0], dw, dh, normalize=0)
    ref = _float_bilinear(img, s[0], dw, dh).transpose(2, 0, 1)
    # 5-bit fractions (<= 1/64 px position error) and 15-bit weights: a few units at most
    assert np.abs(out - ref).max() <= 6.0
    assert np.abs(out - ref).mean() < 1.0


def test_cvmat_constant_image():
    img = np.full((90, 160, 3), 77, np.uint8)
    for size, res in (((160, 90), (-1, 48)), ((160, 90), (-1, 256))):   # linear, cubic
        s, [(dw, dh)] = oracle.scale_and_size(size, res)
        out = oracle.cvmat_to_input(img, s[0], dw, dh, normalize=0)
        # destinations whose every tap (x/s - 1 .. x/s + 2) lies inside the frame
        lo = int(2 * s[0]) + 1
        iw, ih = int((160 - 3) * s[0]), int((90 - 3) * s[0])
        assert (out[:, lo:ih, lo:iw] == 77).all()


# ---- GPU -----------------------------------------------------------------------------------------

def _frames(n, h, w, seed):
    import torch
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randint(0, 256, (n, h, w, 3), generator=g, dtype=torch.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize("size,res,sn", [((1280, 720), (-1, 368), 1), ((1280, 720), (-1, 368), 4),
                                         ((160, 90), (-1, 368), 1), ((333, 251), (208, -1), 2),
                                         ((640, 480), (-1, 368), 1)])
def test_gpu_cvmat_to_input_bitexact(ctx, size, res, sn):
    import torch
    frames = _frames(2, size[1], size[0], 3)
    dev = frames.cuda()
    scales, sizes = api.scale_and_size(size, res, 1.0, sn, 0.25)
    for s, (w, h) in zip(scales, sizes):
        out = torch.empty((2, 3, h, w), device="cuda")
        ctx.cvmat_to_input(out, dev, s)
        got = out.cpu().numpy()
        for f in range(2):
            ref = oracle.cvmat_to_input(frames[f].numpy(), s, w, h)
            np.testing.assert_array_equal(got[f], ref)


@pytest.mark.gpu
@pytest.mark.parametrize("size", [(256, 144), (160, 90)])   # linear and cubic (upscaling) warps
def test_gpu_pose_forward_frames_equals_prepared_input(ctx, size):
    import torch
    from oracle import body25
    from openpose_amd import synth
    from openpose_amd.api import Net, PoseExtractor
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(synth.he_weights(body25.layers(), seed=0, out_scale=0.02))
    pose = PoseExtractor(ctx, net)
    pose.set_input((-1, 128))
    scales, [(w, h)] = api.scale_and_size(size, (-1, 128))
    n = 3
    frames = _frames(n, size[1], size[0], 5)
    ov = np.stack([synth.overlay(3, h // 8, w // 8, seed=f) for f in range(n)])
    pose.set_overlay(torch.from_numpy(ov).cuda())
    pose.forward_frames(frames.cuda())
    x = pose.net_input_numpy()
    ref_x = np.stack([oracle.cvmat_to_input(frames[f].numpy(), scales[0], w, h) for f in range(n)])
    np.testing.assert_array_equal(x, ref_x)
    got = [pose.keypoints(f) for f in range(n)]
    # the same net input through the float entry point: identical people
    pose2 = PoseExtractor(ctx, net)
    pose2.set_overlay(torch.from_numpy(ov).cuda())
    pose2.forward(torch.from_numpy(ref_x).cuda(), size)
    for f in range(n):
        kp, ks = pose2.keypoints(f)
        np.testing.assert_array_equal(got[f][0], kp)
        np.testing.assert_array_equal(got[f][1], ks)
    assert sum(len(g[1]) for g in got) > 0


@pytest.mark.gpu
def test_gpu_pose_frames_rewritten_between_submits(ctx):
    """Pipelined raw-frame submits that reuse ONE device frame buffer, refilled on the context
    stream (torch's current stream) before every submit, as a serving loop would: each batch must
    see its own frames (the warp had run on a side stream ordered only after the previous
    nets).  Every batch's people equal a synchronous forward of the same frames with all device
    work on the context stream (POST_STREAM=0), bit for bit."""
    import torch
    from oracle import body25
    from openpose_amd import synth
    from openpose_amd.api import Net, PoseExtractor, dev_switches
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(synth.he_weights(body25.layers(), seed=3, out_scale=0.02))
    size, n, batches = (256, 144), 3, 5
    _, [(w, h)] = api.scale_and_size(size, (-1, 128))
    ov = torch.from_numpy(np.stack([synth.overlay(3, h // 8, w // 8, seed=40 + f)
                                    for f in range(n)])).cuda()
    host = [_frames(n, size[1], size[0], 100 + b).pin_memory() for b in range(batches)]

    def people(pose):
        return [pose.keypoints(f) for f in range(n)]

    ref = []
    with dev_switches(POST_STREAM=0):
        pose = PoseExtractor(ctx, net)
        pose.set_input((-1, 128))
        pose.set_overlay(ov)
        for b in range(batches):
            pose.forward_frames(host[b].cuda())
            ref.append(people(pose))
        pose.close()
    # the frames matter: the batches' scores differ (the net output shifts the refined peaks)
    assert any(not np.array_equal(ref[0][f][1], ref[1][f][1]) for f in range(n))

    pose = PoseExtractor(ctx, net)
    pose.set_input((-1, 128))
    pose.set_overlay(ov)
    buf = torch.empty_like(host[0], device="cuda")
    got = []
    for b in range(batches):
        buf.copy_(host[b], non_blocking=True)   # queued on the context stream behind batch b-1
        pose.submit_frames(buf)
        if pose.pending() == 2:
            pose.collect()
            got.append(people(pose))
    while pose.pending():
        pose.collect()
        got.append(people(pose))
    assert len(got) == batches
    for b in range(batches):
        for f in range(n):
            np.testing.assert_array_equal(got[b][f][0], ref[b][f][0])
            np.testing.assert_array_equal(got[b][f][1], ref[b][f][1])


@pytest.mark.gpu
@pytest.mark.parametrize("delay_us", [0, 30000])
def test_gpu_pose_direct_forward_between_submit_and_collect(ctx, delay_us):
    """a batch's post-processing runs on the pipeline's side stream and reads
    the net output; a direct forward of the SAME net and shape queued on the context stream after
    the submit (opk_net_forward) writes that same buffer.  It must wait for the post-processing
    (NetHip::note_reader).  The dev hook POST_DELAY_US holds the post-processing stream for 30 ms
    before it reads anything, so a missing wait corrupts the batch deterministically, not by
    timing luck.  Also: the pipelined submits with the delay (batch i+1's nets on the other output
    buffer) and opk_sync covering the side stream."""
    import torch
    from oracle import body25
    from openpose_amd import synth
    from openpose_amd.api import Net, PoseExtractor, dev_switches
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(synth.he_weights(body25.layers(), seed=5, out_scale=0.02))
    size, n = (256, 144), 2
    _, [(w, h)] = api.scale_and_size(size, (-1, 128))
    ov = torch.from_numpy(np.stack([synth.overlay(3, h // 8, w // 8, seed=60 + f)
                                    for f in range(n)])).cuda()
    frames = [_frames(n, size[1], size[0], 200 + b).cuda() for b in range(3)]

    def people(pose):
        return [pose.keypoints(f) for f in range(n)]

    with dev_switches(POST_STREAM=0):   # reference: everything on the context stream
        pose = PoseExtractor(ctx, net)
        pose.set_input((-1, 128))
        pose.set_overlay(ov)
        ref = []
        for b in range(3):
            pose.forward_frames(frames[b])
            ref.append(people(pose))
        pose.close()
    assert not all(np.array_equal(ref[0][f][1], ref[1][f][1]) for f in range(n))

    with dev_switches(POST_DELAY_US=delay_us):
        pose = PoseExtractor(ctx, net)
        pose.set_input((-1, 128))
        pose.set_overlay(ov)
        # 1. submit, then a direct forward of the same shape (batch 1's net input), then collect
        pose.submit_frames(frames[0])
        x0 = torch.from_numpy(pose.net_input_numpy()).cuda()   # (synchronises the context stream)
        net.forward(torch.flip(x0, dims=[3]).contiguous())     # another input, same shape
        pose.collect()
        got0 = people(pose)
        for f in range(n):
            np.testing.assert_array_equal(got0[f][0], ref[0][f][0])
            np.testing.assert_array_equal(got0[f][1], ref[0][f][1])
        # 2. pipelined submits (alternating output buffers) under the delay
        got = []
        for b in range(3):
            pose.submit_frames(frames[b])
            if pose.pending() == 2:
                pose.collect()
                got.append(people(pose))
        while pose.pending():
            pose.collect()
            got.append(people(pose))
        for b in range(3):
            for f in range(n):
                np.testing.assert_array_equal(got[b][f][0], ref[b][f][0])
                np.testing.assert_array_equal(got[b][f][1], ref[b][f][1])
        # 3. opk_sync waits for the side stream too: with the post-processing held for 30 ms
        #    after the nets, a sync right after the submit takes at least that long
        import time
        pose.submit_frames(frames[2])
        t0 = time.perf_counter()
        ctx.sync()
        if delay_us:
            assert time.perf_counter() - t0 >= 0.8 * delay_us * 1e-6
        pose.collect()
        for f in range(n):
            np.testing.assert_array_equal(people(pose)[f][1], ref[2][f][1])
        pose.close()
