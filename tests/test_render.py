"""GPU renderers: renderPoseKeypointsGpu / renderFaceKeypointsGpu / renderHandKeypointsGpu and the
heat-map renders of src/openpose/pose/renderPose.cu (renderKeypointsOld,
include/openpose_private/utilities/render.hu:209-383; renderBodyPartHeatMap(s),
renderPartAffinities, renderPose.cu:419-527).

CPU tests pin the tables (the reference's *_RENDER_GPU macros, compiled here by
tools/gen_render_tables.py) and the oracle restatement (oracle/render.c) with known answers derived
from the reference source, plus the C-ABI's error behaviour.  GPU tests hold libopk_hip.so to the
oracle: bit-exact everywhere except, for keypoints, on the pixels where a limb's ellipse test sits
within 1e-4 of its boundary (the oracle marks them; atan2f / sinf / cosf of glibc and of the HIP
device library may differ by an ulp there), and for PAF colours (atan2f), which are compared to
1e-3 of 255.  Parity with a CUDA build of the reference is unpinned (no CUDA toolchain here)."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _inc_tables():
    """The product's render_tables.inc, parsed."""
    with open(os.path.join(ROOT, "openpose_amd", "csrc", "host", "render_tables.inc")) as f:
        text = f.read()
    arrays = {}
    for kind, name, body in re.findall(r"static const (unsigned|float) (\w+)\[\] = \{([^}]*)\};",
                                       text):
        vals = [v.strip().rstrip("f") for v in body.split(",") if v.strip()]
        arrays[name] = [int(v) for v in vals] if kind == "unsigned" else [float(v) for v in vals]
    rows = re.findall(r'\{"(\w+)", (\w+), (\d+), (\w+), (\d+), (\w+), (\d+)\}', text)
    return {r[0]: dict(pairs=arrays[r[1]], npairs=int(r[2]), scales=arrays[r[3]],
                       nscales=int(r[4]), colors=arrays[r[5]], ncolors=int(r[6])) for r in rows}


def test_render_tables_match_golden():
    gold = oracle.render_tables()
    inc = _inc_tables()
    assert set(inc) == set(gold)
    for name, g in gold.items():
        t = inc[name]
        assert t["pairs"] == g["pairs"] and t["npairs"] * 2 == len(g["pairs"]), name
        assert np.array_equal(np.float32(t["scales"]), np.float32(g["scales"])), name
        assert np.array_equal(np.float32(t["colors"]), np.float32(g["colors"])), name
        assert t["ncolors"] * 3 == len(g["colors"]) and t["nscales"] == len(g["scales"])
    # spot values of poseParametersRender.hpp: BODY_25's first pair / color, BODY_135's scales
    assert gold["BODY_25"]["pairs"][:4] == [1, 8, 1, 2]
    assert gold["BODY_25"]["colors"][:3] == [255.0, 0.0, 85.0]
    assert len(gold["BODY_135"]["scales"]) == 135 and gold["BODY_135"]["scales"][17] == 0.0
    assert gold["FACE"]["colors"] == [255.0, 255.0, 255.0]


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libref_render.so")),
                    reason="reference render tables not built (needs /root/reference)")
def test_render_tables_match_reference_build():
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_render.so"))
    gold = list(oracle.render_tables().values())
    for i, g in enumerate(gold):
        pairs = np.zeros(4096, np.uint32)
        scales = np.zeros(4096, np.float32)
        colors = np.zeros(4096, np.float32)
        counts = np.zeros(3, np.int32)
        assert lib.ref_render_table(i, pairs.ctypes.data_as(ctypes.c_void_p),
                                    scales.ctypes.data_as(ctypes.c_void_p),
                                    colors.ctypes.data_as(ctypes.c_void_p),
                                    counts.ctypes.data_as(ctypes.c_void_p), 4096) == 0
        assert list(pairs[:counts[0]]) == g["pairs"]
        assert np.array_equal(scales[:counts[1]], np.float32(g["scales"]))
        assert np.array_equal(colors[:counts[2]], np.float32(g["colors"]))


def _limb_person(parts=25):
    kp = np.zeros((1, parts, 3), np.float32)
    kp[0, 1] = (30, 60, 0.9)
    kp[0, 8] = (90, 60, 0.9)
    return kp


def test_oracle_keypoints_known_answer():
    """One horizontal BODY_25 limb (pair 1-8) on a black 120x120 frame: radius 1.2, line width
    1.0, scale 0.33 (box 60 px wide), so bSqrt = 0.1089 and the ellipse is the row y = 60 from x =
    30 to 90; the circles (maxr2 = 0.157) are the two keypoint pixels.  Colors: BODY_25 index 8 and
    1 are both (255, 0, 0)."""
    frame = np.zeros((120, 120, 3), np.float32)
    out, amb = oracle.render_keypoints(frame, _limb_person(), "BODY_25", threshold=0.05, alpha=0.6)
    a = np.float32(0.6)
    once = np.float32(1 - a) * np.float32(0) + a * np.float32(255)
    twice = np.float32(1 - a) * once + a * np.float32(255)
    want = np.zeros_like(frame)
    want[60, 30:91, 2] = once
    want[60, 30, 2] = twice
    want[60, 90, 2] = twice
    np.testing.assert_array_equal(out, want)
    # the two row ends sit exactly on the ellipse (judge = 1): marked ambiguous
    assert amb[60, 30] and amb[60, 90] and amb.sum() >= 2


def test_oracle_keypoints_rules():
    frame = np.full((120, 120, 3), 100.0, np.float32)
    # below-threshold parts draw nothing
    kp = _limb_person()
    kp[0, 8, 2] = 0.05
    out, _ = oracle.render_keypoints(frame, kp, "BODY_25", threshold=0.05)
    changed = np.argwhere(np.any(out != frame, axis=2))
    assert [tuple(v) for v in changed] == [(60, 30)]   # only part 1's circle
    # blend_original false clears the frame first, even with nobody to draw
    out, _ = oracle.render_keypoints(frame, np.zeros((0, 25, 3), np.float32), "BODY_25",
                                     blend=False)
    assert not out.any()


def test_oracle_heat_map_colormap_known_answers():
    """A constant heat map interpolates to itself; getColorHeatMap at 0.25 is (255, 128, 0) into
    (R, G, B) = target (+2, +1, +0); |v| for the distance render."""
    frame = np.full((16, 24, 3), 10.0, np.float32)
    heat = np.full((2, 4, 6), 0.25, np.float32)
    heat[1] = -0.25
    out = oracle.render_heat_map(frame, heat, 4.0, 0, alpha=0.5)
    a = np.float32(0.5)
    mix = lambda c: np.float32(1 - a) * np.float32(10) + a * np.float32(c)
    np.testing.assert_array_equal(out[..., 2], mix(255.0))
    np.testing.assert_array_equal(out[..., 1], mix(np.float32(256.0) * np.float32(0.125) * 4))
    np.testing.assert_array_equal(out[..., 0], mix(0.0))
    # negative values truncate to 0 -> 256 * 0.5 in the first channel; abs gives 0.25 again
    out = oracle.render_heat_map(frame, heat, 4.0, 1, alpha=0.5)
    np.testing.assert_array_equal(out[..., 2], mix(128.0))
    out2 = oracle.render_heat_map(frame, heat, 4.0, 1, alpha=0.5, abs_value=True)
    np.testing.assert_array_equal(out2[..., 1], mix(128.0))


def test_oracle_heat_maps_and_pafs_known_answers():
    frame = np.zeros((8, 8, 3), np.float32)
    heat = np.zeros((3, 8, 8), np.float32)
    heat[2, 3, 5] = 2.0        # saturates to 1; COCO color 2 = (255, 85, 0)
    out = oracle.render_heat_maps(frame, heat, 1.0, 3, alpha=1.0)
    assert tuple(out[3, 5]) == (0.0, 85.0, 255.0) and np.count_nonzero(out) == 2
    # PAF (-1, 0): atan2(0, 1) = 0 -> fk 0.5 -> v 27.5 -> (0, 255 (1 - 2.5 / 11), 255), radius 1
    paf = np.zeros((2, 4, 4), np.float32)
    paf[0] = -1.0
    out = oracle.render_pafs(np.zeros((4, 4, 3), np.float32), paf, 1.0, 0, 1, alpha=1.0)
    g = np.float32(255.0) * (np.float32(1) - (np.float32(27.5) - 15 - 6 - 4) / np.float32(11))
    np.testing.assert_array_equal(out[..., 2], 0.0)
    np.testing.assert_allclose(out[..., 1], g, rtol=1e-6)
    np.testing.assert_array_equal(out[..., 0], 255.0)
    # zero vectors: fk from atan2(-0, -0) = -pi -> 0; radius 0 -> no colour
    out = oracle.render_pafs(np.zeros((4, 4, 3), np.float32), np.zeros((2, 4, 4), np.float32), 1.0,
                             0, 1, alpha=1.0)
    assert not out.any()


def test_render_abi_errors_host_only():
    """renderPoseKeypointsGpu's and checkAlpha's errors, raised before any device work."""
    from openpose_amd.api import Context
    OPK_ERR_ARG = 1   # include/opk.h
    ctx = Context.host_only()
    L = ctx.L
    fake = ctypes.c_void_p(64)
    cases = [
        (lambda: L.opk_render_pose_keypoints(ctx.h, fake, 2, 1, 64, 64, fake, 0.05, 1, 1, 0.6),
         "googlyEyes not compatible with MPI"),
        (lambda: L.opk_render_pose_keypoints(ctx.h, fake, 0, 128, 64, 64, fake, 0.05, 0, 1, 0.6),
         "POSE_MAX_PEOPLE = 127"),
        (lambda: L.opk_render_pose_keypoints(ctx.h, fake, 15, 1, 64, 64, fake, 0.05, 0, 1, 0.6),
         "Invalid Model"),
        (lambda: L.opk_render_pose_heat_map(ctx.h, fake, 64, 64, fake, 8, 8, 1.0, 0, 1.5),
         "Alpha must be in the range [0, 1]"),
        (lambda: L.opk_render_pose_pafs(ctx.h, fake, 0, 64, 64, fake, 8, 8, 1.0, -0.1),
         "Alpha must be in the range [0, 1]"),
    ]
    for call, msg in cases:
        assert call() == OPK_ERR_ARG
        assert msg in L.opk_last_error().decode()
    # nothing to draw: no device work, success even on a host-only context
    assert L.opk_render_pose_keypoints(ctx.h, fake, 0, 0, 64, 64, None, 0.05, 0, 1, 0.6) == 0
    assert L.opk_render_face_keypoints(ctx.h, fake, 64, 64, None, 0, 0.4, 0.6) == 0
    assert L.opk_render_hand_keypoints(ctx.h, fake, 64, 64, None, 0, 0.2, 0.6) == 0


# ---- GPU parity ---------------------------------------------------------------------------------
def people_on(w, h, n, parts, seed, spread=0.15):
    """n synthetic people: a centre and parts scattered around it (some below threshold)."""
    rng = np.random.default_rng(seed)
    kp = np.zeros((n, parts, 3), np.float32)
    for p in range(n):
        cx, cy = rng.uniform(0.1, 0.9) * w, rng.uniform(0.1, 0.9) * h
        r = spread * min(w, h) * rng.uniform(0.5, 1.5)
        kp[p, :, 0] = cx + rng.uniform(-r, r, parts)
        kp[p, :, 1] = cy + rng.uniform(-r, r, parts)
        kp[p, :, 2] = rng.uniform(0, 1, parts)
    kp[..., 2][kp[..., 2] < 0.15] = 0.0
    return kp


def _frame(h, w, seed):
    return np.random.default_rng(seed).uniform(0, 255, (h, w, 3)).astype(np.float32)


def _check_keypoints(got, want, amb):
    diff = np.any(got != want, axis=2)
    bad = diff & (amb == 0)
    assert not bad.any(), "%d unambiguous pixels differ, first %s" % (bad.sum(), np.argwhere(bad)[:5])
    assert amb.mean() < 0.01
    print("keypoints: %d px, %d ambiguous, %d of them differ" % (
        amb.size, int(amb.sum()), int((diff & (amb != 0)).sum())))


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,n,googly,blend", [(320, 240, 6, False, True), (321, 203, 12, True, True),
                                                (160, 120, 3, False, False), (96, 64, 0, False, False)])
def test_gpu_pose_keypoints_body25(w, h, n, googly, blend):
    import torch
    from openpose_amd.api import Context
    ctx = Context(0)
    frame = _frame(h, w, 1)
    kp = people_on(w, h, n, 25, seed=n + w)
    want, amb = oracle.render_keypoints(frame, kp, "BODY_25", threshold=0.05, alpha=0.6,
                                        blend=blend, eyes=(15, 16) if googly else (-1, -1))
    f = torch.from_numpy(frame).cuda()
    ctx.render_pose_keypoints(f, torch.from_numpy(kp).cuda() if n else None, 0, threshold=0.05,
                              googly_eyes=googly, blend_original=blend, alpha=0.6)
    ctx.sync()
    got = f.cpu().numpy()
    if n == 0 and blend:
        np.testing.assert_array_equal(got, frame)
    _check_keypoints(got, want, amb)
    if n:
        assert np.any(got != frame)


@pytest.mark.gpu
def test_gpu_pose_keypoints_every_model():
    import torch
    from openpose_amd.api import Context
    ctx = Context(0)
    w, h = 200, 150
    for model, (table, stable, parts, eyes) in sorted(oracle.RENDER_POSE.items()):
        frame = _frame(h, w, model)
        kp = people_on(w, h, 4, parts, seed=model)
        googly = eyes[0] >= 0
        want, amb = oracle.render_keypoints(frame, kp, table, scales_table=stable, threshold=0.05,
                                            eyes=eyes if googly else (-1, -1))
        f = torch.from_numpy(frame).cuda()
        ctx.render_pose_keypoints(f, torch.from_numpy(kp).cuda(), model, threshold=0.05,
                                  googly_eyes=googly)
        ctx.sync()
        _check_keypoints(f.cpu().numpy(), want, amb)


@pytest.mark.gpu
def test_gpu_face_and_hand_keypoints():
    import torch
    from openpose_amd.api import Context
    ctx = Context(0)
    w, h = 256, 192
    frame = _frame(h, w, 7)
    face = people_on(w, h, 5, 70, seed=3, spread=0.08)
    want, amb = oracle.render_keypoints(frame, face, "FACE", radius_div=120.0, line_div=250.0,
                                        threshold=0.4)
    f = torch.from_numpy(frame).cuda()
    ctx.render_face_keypoints(f, torch.from_numpy(face).cuda(), threshold=0.4)
    ctx.sync()
    _check_keypoints(f.cpu().numpy(), want, amb)
    hands = people_on(w, h, 6, 21, seed=4, spread=0.06)
    want, amb = oracle.render_keypoints(frame, hands, "HAND", radius_div=100.0, line_div=80.0,
                                        threshold=0.2)
    f = torch.from_numpy(frame).cuda()
    ctx.render_hand_keypoints(f, torch.from_numpy(hands).cuda(), threshold=0.2)
    ctx.sync()
    _check_keypoints(f.cpu().numpy(), want, amb)


@pytest.mark.gpu
def test_gpu_pose_keypoints_full_hd_crowd():
    """1920x1080 with 127 people (POSE_MAX_PEOPLE): crowded tiles, person compaction past one
    wave."""
    import torch
    from openpose_amd.api import Context
    ctx = Context(0)
    w, h = 1920, 1080
    frame = _frame(h, w, 11)
    kp = people_on(w, h, 127, 25, seed=12, spread=0.08)
    want, amb = oracle.render_keypoints(frame, kp, "BODY_25", threshold=0.05)
    f = torch.from_numpy(frame).cuda()
    ctx.render_pose_keypoints(f, torch.from_numpy(kp).cuda(), 0, threshold=0.05)
    ctx.sync()
    _check_keypoints(f.cpu().numpy(), want, amb)


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [8.0, 1.7, 0.9])
def test_gpu_heat_map_renders(scale):
    import torch
    from openpose_amd.api import Context
    ctx = Context(0)
    rng = np.random.default_rng(int(scale * 10))
    hh, hw = 23, 37
    heat = rng.uniform(-0.3, 1.2, (78, hh, hw)).astype(np.float32)
    w, h = int(hw * scale) + 3, int(hh * scale) + 2   # a little past the map: border clamps
    frame = _frame(h, w, 5)
    hd = torch.from_numpy(heat).cuda()
    for part, dist in ((3, False), (25, False), (7, True)):
        want = oracle.render_heat_map(frame, heat, scale, part, alpha=0.7, abs_value=dist)
        f = torch.from_numpy(frame).cuda()
        ctx.render_heat_map(f, hd, scale, part, alpha=0.7, distance=dist)
        ctx.sync()
        np.testing.assert_array_equal(f.cpu().numpy(), want)
    want = oracle.render_heat_maps(frame, heat, scale, 25, alpha=0.7)
    f = torch.from_numpy(frame).cuda()
    ctx.render_heat_maps(f, hd, scale, 0, alpha=0.7)
    ctx.sync()
    np.testing.assert_array_equal(f.cpu().numpy(), want)
    # PAFs: one (bilinear) and all 26 from channel 26 (BODY_25: 25 parts + background)
    for part, count in ((30, 1), (None, 26)):
        want = oracle.render_pafs(frame, heat, scale, 26 if part is None else part, count, alpha=0.7)
        f = torch.from_numpy(frame).cuda()
        ctx.render_pafs(f, hd, scale, part=part, alpha=0.7)
        ctx.sync()
        got = f.cpu().numpy()
        print("pafs x%d: max |diff| %.3g" % (count, float(np.abs(got - want).max())))
        np.testing.assert_allclose(got, want, rtol=0, atol=0.255 * count / 26 + 0.01)
