"""Face / hand keypoint extraction on the GPU (op::FaceExtractorCaffe / op::HandExtractorCaffe
forwardPass) against the oracle (oracle/extract.py, oracle.warp_affine_inv, oracle.resize_merge),
bit-exact:
  - every crop: its 2x3 inverse map and its net input (warpAffine INTER_LINEAR | WARP_INVERSE_MAP +
    uCharCvMatToFloatPtr) equal the oracle's for the same rectangle;
  - keypoints: resize x8 + per-part maximum + M (x, y) of the net output the library computed,
    restated on the CPU, equal the library's keypoints (the net itself is checked against the fp32
    oracle in test_gpu_net.py::test_reference_cpm_nets_vs_oracle).
Weights are seeded random (no checkpoints offline); frames are random BGR uint8.
"""
import numpy as np
import pytest
import torch

import oracle.extract as ox
from openpose_amd import _lib, synth
from openpose_amd.api import FACE, HAND, KeypointExtractor, Net
from tests import cpm_graphs, prototxt

pytestmark = pytest.mark.gpu


def _net(ctx, name, seed):
    graph = prototxt.parse(prototxt.emit(cpm_graphs.GRAPHS[name]()))
    net = Net(ctx, name)
    net.set_params(synth.he_weights(graph, seed=seed, out_scale=0.05))
    return net


def _frames(n, h, w, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (n, h, w, 3), dtype=torch.uint8, generator=g)


def _check_crops(ex, frames_np, frame_of, want_ms):
    crops = ex.crops()
    assert len(crops) == len(want_ms)
    w, h = ex.net_resolution
    for (m, x), (f, want) in zip(crops, zip(frame_of, want_ms)):
        np.testing.assert_array_equal(m, want)
        np.testing.assert_array_equal(x, ox.oracle.warp_affine_inv(frames_np[f], want, w, h))


def test_face_extractor_matches_oracle(ctx):
    net = _net(ctx, "builtin:FACE", seed=3)
    ex = KeypointExtractor(ctx, net, FACE, (368, 368))
    frames = _frames(2, 360, 480, seed=1)
    rects = np.array([[100.5, 60.25, 150.0, 150.0],    # inside
                      [-30.0, 250.0, 140.0, 140.0],    # runs off the left / bottom edge
                      [10.0, 10.0, 40.0, 40.0],        # too small (<= 40): skipped, zeros
                      [300.75, 20.5, 97.5, 97.5],
                      [200.0, 100.0, 233.0, 233.0]], np.float32)
    frame_of = np.array([0, 1, 0, 1, 0], np.int32)
    ex.set_heatmaps(7)   # --heatmaps_add_parts --heatmaps_scale 3 (UnsignedChar)
    kp = ex.forward(frames.cuda(), rects, frame_of)
    parts = ex.parts
    assert parts == 70 and kp.shape == (5, 70, 3)
    hm = ex.heatmaps_numpy()
    assert hm.shape == (5, 70, 368, 368)
    valid = [0, 1, 3, 4]   # four crops: one batch of 4, the net output holds all of them
    want_ms = [ox.face_affine(rects[i], 368) for i in valid]
    assert ox.face_affine(rects[2], 368) is None
    fr = frames.numpy()
    _check_crops(ex, fr, frame_of[valid], want_ms)
    out = net.output_numpy()
    assert out.shape == (4, 71, 46, 46)
    for j, i in enumerate(valid):
        want = ox.keypoints_from_output(out[j], want_ms[j], parts)
        np.testing.assert_array_equal(kp[i], want)
        np.testing.assert_array_equal(hm[i], ox.crop_heatmaps(out[j], parts, 7))
    assert not kp[2].any() and not hm[2].any()


@pytest.mark.parametrize("res,scales", [((368, 368), 1), ((320, 256), 2)])
def test_hand_extractor_matches_oracle(ctx, res, scales):
    net = _net(ctx, "builtin:HAND", seed=5)
    ex = KeypointExtractor(ctx, net, HAND, res)
    if scales > 1:
        ex.set_scales(scales, 0.4)
    frames = _frames(1, 300, 400, seed=2)
    rects = np.array([[[50.5, 40.0, 80.0, 80.0], [250.25, 120.0, 61.0, 61.0]],
                      [[350.0, -20.0, 90.0, 90.0], [0.0, 0.0, 3.0, 3.0]]],   # last: area <= 10
                     np.float32)
    mode = 5 if scales > 1 else 8   # PlusMinusOne / NoScale
    ex.set_heatmaps(mode)
    kp = ex.forward(frames.cuda(), rects)
    parts = ex.parts
    assert parts == 21 and kp.shape == (2, 2, 21, 3)
    hm = ex.heatmaps_numpy()
    assert hm.shape == (2, 2, 21, res[1], res[0])
    side = min(res)
    crops, owners = [], []
    for hand in range(2):
        for p in range(2):
            r = rects[p, hand]
            if not ox.hand_valid(r):
                continue
            for rs in ox.hand_scale_rects(r, scales, 0.4):
                crops.append(ox.hand_affine(rs, side, mirror=hand == 0))
                owners.append((hand, p))
    assert len(crops) == 3 * scales
    fr = frames.numpy()
    _check_crops(ex, fr, [0] * len(crops), crops)
    out = net.output_numpy()
    # 3 crops = batches of 2 + 1 (single scale) or 6 = 4 + 2: check the last batch's crops
    # against its net output, and every crop's input above
    nb = out.shape[0]
    first = len(crops) - nb
    best = {}
    for j in range(first, len(crops)):
        est = ox.keypoints_from_output(out[j - first], crops[j], parts)
        o = owners[j]
        if o not in best or ox.average_score(est) > ox.average_score(best[o]):
            best[o] = est
    for (hand, p), est in best.items():
        if all(owners[j] != (hand, p) for j in range(first)):   # owner's crops all in the batch
            np.testing.assert_array_equal(kp[hand, p], est)
    # heat maps: the LAST scale's crop of each rectangle (handExtractorCaffe.cpp:433-441)
    for j in range(first, len(crops)):
        last = j == len(crops) - 1 or owners[j + 1] != owners[j]
        if last:
            hand, p = owners[j]
            np.testing.assert_array_equal(hm[hand, p], ox.crop_heatmaps(out[j - first], parts, mode))
    assert not kp[1, 1].any() and not hm[1, 1].any()


def test_batches_are_independent(ctx):
    """Crops split into power-of-two batches give the same keypoints as smaller calls of the same
    batch sizes (the offsets of the batched warp / net / maximum are right)."""
    net = _net(ctx, "builtin:FACE", seed=4)
    ex = KeypointExtractor(ctx, net, FACE, (368, 368))
    ex.set_max_batch(4)
    frames = _frames(1, 300, 420, seed=6).cuda()
    rng = np.random.default_rng(0)
    rects = np.zeros((6, 4), np.float32)
    rects[:, :2] = rng.uniform(-20, 200, (6, 2))
    rects[:, 2] = rects[:, 3] = rng.uniform(50, 180, 6)
    kp = ex.forward(frames, rects)            # batches of 4 + 2
    kp4 = ex.forward(frames, rects[:4])       # one batch of 4
    kp2 = ex.forward(frames, rects[4:])       # one batch of 2
    np.testing.assert_array_equal(kp[:4], kp4)
    np.testing.assert_array_equal(kp[4:], kp2)


def test_extractor_errors(ctx):
    net = _net(ctx, "builtin:FACE", seed=3)
    ex = KeypointExtractor(ctx, net, FACE, (368, 368))
    frames = _frames(1, 100, 100, seed=1).cuda()
    with pytest.raises(_lib.OpkError, match="squared"):
        ex.forward(frames, np.array([[0, 0, 50, 60]], np.float32))
    with pytest.raises(_lib.OpkError, match="frame index"):
        ex.forward(frames, np.array([[0, 0, 50, 50]], np.float32), np.array([1], np.int32))
    with pytest.raises(_lib.OpkError):
        ex.set_scales(2, 0.4)                 # a hand option
    with pytest.raises(_lib.OpkError):
        KeypointExtractor(ctx, net, FACE, (360, 368))
    assert ex.forward(frames, np.zeros((0, 4), np.float32)).shape == (0, 70, 3)
