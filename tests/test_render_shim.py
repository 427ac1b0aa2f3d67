"""The render drop-in (integration/renderHip.cpp, replacing src/openpose/pose/renderPose.cu,
face/renderFace.cu and hand/renderHand.cu): it compiles against the reference's own headers with
-Wall -Wextra -Werror, and a driver built against them (tests/render_driver.cpp) calls
renderPoseKeypointsGpu / renderPoseHeatMapGpu / renderPosePAFsGpu / renderFaceKeypointsGpu with the
reference signatures on the GPU -- results identical to the C-ABI path (tests/test_render.py pins
that path to the oracle).  The driver is built where /root/reference exists (build_render_driver(),
also run by __graft_entry__.build()) and travels with the tree."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "_bin", "render_driver")


@pytest.mark.skipif(not os.path.isdir("/root/reference/include"), reason="no reference tree")
def test_render_shim_compiles_against_reference_headers():
    r = subprocess.run(["g++", "-std=c++14", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
                        "-I/root/reference/include", "-I" + os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "integration", "renderHip.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def build_render_driver():
    """Compile tests/_bin/render_driver (needs the reference headers and libopk_hip.so)."""
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    cmd = ["g++", "-std=c++14", "-O1", "-Wall", "-Wextra", "-Werror",
           "-I/root/reference/include", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "integration"),
           os.path.join(ROOT, "integration", "renderHip.cpp"),
           os.path.join(ROOT, "tests", "render_driver.cpp"),
           "-L" + os.path.join(ROOT, "openpose_amd"), "-lopk_hip",
           "-Wl,-rpath,$ORIGIN/../../openpose_amd", "-o", BIN]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return BIN


@pytest.mark.skipif(not os.path.isdir("/root/reference/include"), reason="no reference tree")
def test_render_driver_builds():
    assert os.path.exists(build_render_driver())


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(BIN), reason="driver not built (needs the reference headers)")
def test_render_shim_matches_abi():
    import torch
    from openpose_amd.api import Context
    from tests.test_render import people_on

    w, h, hw, hh = 232, 176, 29, 22
    rng = np.random.default_rng(9)
    frame = rng.uniform(0, 255, (h, w, 3)).astype(np.float32)
    pose = people_on(w, h, 5, 25, seed=21)
    face = people_on(w, h, 3, 70, seed=22, spread=0.05)
    heat = rng.uniform(-0.5, 1.0, (78, hh, hw)).astype(np.float32)
    with tempfile.TemporaryDirectory() as d:
        np.array([w, h, 5, hw, hh, 3], np.int32).tofile(os.path.join(d, "meta.i32"))
        frame.tofile(os.path.join(d, "frame.f32"))
        pose.tofile(os.path.join(d, "pose.f32"))
        heat.tofile(os.path.join(d, "heat.f32"))
        face.tofile(os.path.join(d, "face.f32"))
        r = subprocess.run([BIN, d], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and "render ok" in r.stdout, r.stderr + r.stdout
        outs = {k: np.fromfile(os.path.join(d, "out_%s.f32" % k), np.float32).reshape(h, w, 3)
                for k in ("pose", "heat", "pafs", "face")}
    ctx = Context(0)
    hd = torch.from_numpy(heat).cuda()
    scale = np.float32(w) / np.float32(hw)

    def run(fn):
        f = torch.from_numpy(frame).cuda()
        fn(f)
        ctx.sync()
        return f.cpu().numpy()

    want = {
        "pose": run(lambda f: ctx.render_pose_keypoints(f, torch.from_numpy(pose).cuda(), 0,
                                                        threshold=0.05, googly_eyes=True)),
        "heat": run(lambda f: ctx.render_heat_map(f, hd, float(scale), 3, alpha=0.7)),
        "pafs": run(lambda f: ctx.render_pafs(f, hd, float(scale), alpha=0.7)),
        "face": run(lambda f: ctx.render_face_keypoints(f, torch.from_numpy(face).cuda(),
                                                        threshold=0.4)),
    }
    for k in outs:
        np.testing.assert_array_equal(outs[k], want[k], err_msg=k)
        assert np.any(outs[k] != frame), k
