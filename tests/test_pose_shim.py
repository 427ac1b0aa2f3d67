"""The pose drop-in (integration/openpose_hip_shim.cpp) run through the reference's own call
sequence by a linked C++ driver (tests/pose_driver.cpp; reference symbols that need OpenCV are backed
by tests/shim_backing.cpp), against the C-ABI pipeline (openpose_amd.api) on the same inputs:

* PoseExtractorHip through a PoseExtractorNet* on a worker thread (1 scale with a property pushed,
  4 scales, --upsampling_ratio 4), destroyed on the main thread after the join (the Wrapper's order);
* the poseNetOutput injection path;
* makeNetHip in addCaffeNetOnThread's order (output blob taken before the first forward, read
  after forwards of two shapes);
* resizeAndMergeGpu -> nmsGpu -> connectBodyPartsGpu with the reference signatures (the CUDA
  build's map semantics, the shim's default), float and double instantiations;
* two worker threads with one extractor each, forwarding concurrently: same keypoints as one.

The driver is built here where /root/reference is present (__graft_entry__.build() does it too) and
runs on the GPU box from tests/_bin (no reference code is compiled into it).
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "_bin", "pose_driver")
# reference symbols of code paths the driver never takes (face / hand extractors, CvMatToOpInput):
# their definitions need OpenCV (core/matrix.cpp, face/faceExtractorNet.cpp, hand/handExtractorNet.cpp)
ALLOWED_UNRESOLVED = ("op::Matrix::", "op::FaceExtractorNet::", "op::HandExtractorNet::",
                      "typeinfo for op::FaceExtractorNet", "typeinfo for op::HandExtractorNet")


def build_pose_driver():
    """Compile tests/_bin/pose_driver (needs the reference headers and libopk_hip.so)."""
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    cmd = ["g++", "-std=c++14", "-O1", "-Wall", "-Wextra", "-Werror",
           "-I/root/reference/include", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "integration"),
           os.path.join(ROOT, "integration", "openpose_hip_shim.cpp"),
           os.path.join(ROOT, "integration", "arrayCpuGpuHip.cpp"),
           os.path.join(ROOT, "tests", "shim_backing.cpp"),
           os.path.join(ROOT, "tests", "pose_driver.cpp"),
           "-L" + os.path.join(ROOT, "openpose_amd"), "-lopk_hip", "-lpthread",
           "-Wl,-rpath,$ORIGIN/../../openpose_amd",
           "-Wl,--unresolved-symbols=ignore-all", "-o", BIN]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    nm = subprocess.run(["nm", "-C", "--undefined-only", BIN], capture_output=True, text=True)
    missing = [l.split(None, 1)[1] for l in nm.stdout.splitlines()
               if "op::" in l and " U " in l]
    bad = [m for m in missing if not m.startswith(ALLOWED_UNRESOLVED)]
    assert not bad, "unresolved reference symbols on the tested path: %s" % bad
    return BIN


@pytest.mark.skipif(not os.path.isdir("/root/reference/include"), reason="no reference tree")
def test_pose_driver_builds():
    assert os.path.exists(build_pose_driver())


def _inputs(d):
    """Synthetic BODY_25 weights as a .caffemodel, net inputs of 1 and 4 scales, a net output."""
    from oracle import body25
    from openpose_amd import synth
    from openpose_amd.api import scale_and_size
    from tests import caffemodel_writer as cw
    graph = body25.layers()
    params = synth.he_weights(graph, seed=31, out_scale=0.02)
    path = os.path.join(d, "model.caffemodel")
    with open(path, "wb") as f:
        f.write(cw.body25_caffemodel(params, graph))
    producer = (640, 360)
    scales, sizes = scale_and_size(producer, (-1, 368), 1.0, 4, 0.25)
    rng = np.random.default_rng(32)
    xs = [rng.uniform(-0.5, 0.5, (1, 3, h, w)).astype(np.float32) for (w, h) in sizes]
    for i, x in enumerate(xs):
        x.tofile(os.path.join(d, "in_s%d.f32" % i))
    np.array(scales, np.float64).tofile(os.path.join(d, "scales.f64"))
    oh, ow = sizes[0][1] // 8, sizes[0][0] // 8
    field = (synth.overlay(5, oh, ow, seed=33) +
             rng.normal(0, 0.01, (78, oh, ow))).astype(np.float32)
    field.tofile(os.path.join(d, "netout.f32"))
    meta = [sizes[0][1], sizes[0][0], 4] + [v for (w, h) in sizes for v in (h, w)] + \
        [producer[0], producer[1], oh, ow]
    np.array(meta, np.int32).tofile(os.path.join(d, "meta.i32"))
    return path, producer, scales, sizes, xs, field


def _read(d, name, dtype=np.float32):
    return np.fromfile(os.path.join(d, name), dtype)


def _result(d, tag, parts=25):
    meta = _read(d, tag + "_meta.f32")
    n = int(meta[0])
    kp = _read(d, tag + "_kp.f32").reshape(n, parts, 3) if n else np.zeros((0, parts, 3), np.float32)
    sc = _read(d, tag + "_sc.f32") if n else np.zeros(0, np.float32)
    return kp, sc, float(meta[1])


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(BIN), reason="driver not built (needs the reference headers)")
def test_pose_shim_matches_abi(ctx):
    import torch
    from openpose_amd.api import Net, PoseExtractor

    with tempfile.TemporaryDirectory() as d:
        path, producer, scales, sizes, xs, field = _inputs(d)
        s_fns = np.float32(2.0)
        s_fns.tofile(os.path.join(d, "fns_scale.f32"))
        r = subprocess.run([BIN, d], capture_output=True, text=True, timeout=180)
        assert r.returncode == 0 and "pose driver ok" in r.stdout, r.stderr + r.stdout

        net = Net(ctx, "builtin:BODY_25", caffemodel=path)
        dev = [torch.from_numpy(x).cuda() for x in xs]

        # 1. one scale, NMS threshold pushed through PoseExtractorNet::set
        pose = PoseExtractor(ctx, net)
        pose.set_property(0, 0.06)
        pose.forward(dev[0], producer)
        kp, sc = pose.keypoints(0)
        gk, gs, gscale = _result(d, "single")
        np.testing.assert_array_equal(gk, kp)   # synthetic weights: usually nobody; maps below
        np.testing.assert_array_equal(gs, sc)
        assert gscale == np.float32(pose.scale_net_to_output())
        hs = _read(d, "single_heatsize.i32", np.int32)
        heat = pose.heatmaps_numpy()
        assert list(hs) == [1, 78, heat.shape[2], heat.shape[3]]
        np.testing.assert_array_equal(_read(d, "single_heat.f32").reshape(heat.shape[1:]), heat[0])
        np.testing.assert_array_equal(_read(d, "single_cand.f32").reshape(25, 128, 3),
                                      pose.peaks_numpy()[0])
        # 4 scales
        pose.forward_multi(dev, producer)
        kp, sc = pose.keypoints(0)
        gk, gs, _ = _result(d, "multi")
        np.testing.assert_array_equal(gk, kp)
        np.testing.assert_array_equal(gs, sc)
        pose.close()

        # 2. --upsampling_ratio 4
        p4 = PoseExtractor(ctx, net)
        p4.set_upsampling_ratio(4.0)
        p4.forward(dev[0], producer)
        kp, sc = p4.keypoints(0)
        gk, gs, gscale = _result(d, "up4")
        np.testing.assert_array_equal(gk, kp)
        np.testing.assert_array_equal(gs, sc)
        assert gscale == np.float32(p4.scale_net_to_output())
        h4 = _read(d, "up4_heatsize.i32", np.int32)
        assert list(h4) == [1, 78, 4 * (sizes[0][1] // 8), 4 * (sizes[0][0] // 8)]
        p4.close()

        # 3. injection
        pi = PoseExtractor(ctx, None)
        pi.forward_net_output(torch.from_numpy(field[None]).cuda(), sizes[0], producer)
        kp, sc = pi.keypoints(0)
        gk, gs, _ = _result(d, "inject")
        assert len(kp) >= 1
        np.testing.assert_array_equal(gk, kp)
        np.testing.assert_array_equal(gs, sc)
        pi.close()

        # 4. NetHip output blob, live across forwards of two shapes
        assert list(_read(d, "net_before.i32", np.int32)) == [1, 78, 1, 1]
        net.forward(dev[0])
        np.testing.assert_array_equal(_read(d, "net_out0.f32"), net.output_numpy().ravel())
        net.forward(dev[1])
        o1 = net.output_numpy()
        assert list(_read(d, "net_after.i32", np.int32)) == list(o1.shape)
        np.testing.assert_array_equal(_read(d, "net_out1.f32"), o1.ravel())

        # 5. the *Gpu functions (CUDA-build semantics) vs the C-ABI calls they wrap
        H, W = sizes[0][1], sizes[0][0]
        src = torch.from_numpy(field[None]).cuda()
        heat = torch.empty((1, 78, H, W), device="cuda")
        ctx.resize_and_merge(heat, [src], semantics=1, scale_ratios=[1.0])
        peaks = torch.zeros((1, 25, 128, 3), device="cuda")
        off = float(np.float32(0.5 / np.float64(s_fns)))
        ctx.nms(peaks, heat, 0.05, (off, off), semantics=1)
        np.testing.assert_array_equal(_read(d, "fns_peaks.f32").reshape(25, 128, 3), peaks.cpu().numpy()[0])
        kp, sc = ctx.connect_body_parts(heat, peaks, scale=float(s_fns))
        n = int(_read(d, "fns_meta.f32")[0])
        assert n == len(kp) and n >= 1
        np.testing.assert_array_equal(_read(d, "fns_kp.f32").reshape(n, 25, 3), kp)
        np.testing.assert_array_equal(_read(d, "fns_sc.f32"), sc)
        # 5b. the double instantiations (the reference instantiates all three for double): the float
        # kernels between device conversions, so exactly the float results, widened
        np.testing.assert_array_equal(_read(d, "fns64_heat.f64", np.float64).reshape(78, H, W),
                                      heat.cpu().numpy()[0].astype(np.float64))
        np.testing.assert_array_equal(_read(d, "fns64_peaks.f64", np.float64).reshape(25, 128, 3),
                                      peaks.cpu().numpy()[0].astype(np.float64))
        assert int(_read(d, "fns64_meta.f64", np.float64)[0]) == n
        np.testing.assert_array_equal(_read(d, "fns64_kp.f64", np.float64).reshape(n, 25, 3),
                                      kp.astype(np.float64))
        np.testing.assert_array_equal(_read(d, "fns64_sc.f64", np.float64), sc.astype(np.float64))

        # 6. two concurrent Wrapper threads: every repetition equals the single-thread result
        gk, gs, _ = _result(d, "single")
        for t in range(2):
            for rep in range(3):
                tk, ts, _ = _result(d, "thread%d_%d" % (t, rep))
                np.testing.assert_array_equal(tk, gk)
                np.testing.assert_array_equal(ts, gs)
                np.testing.assert_array_equal(_read(d, "thread%d_%d_heat.f32" % (t, rep)),
                                              _read(d, "single_heat.f32"))


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(BIN), reason="driver not built (needs the reference headers)")
def test_pose_shim_split_precision_env(ctx):
    """OPENPOSE_HIP_PRECISION=split puts every net the drop-in creates into OPK_PRECISION_SPLIT: the
    makeNetHip output blob and PoseExtractorHip's heat maps / peaks / keypoints equal the C-ABI run
    with Net.set_precision(PRECISION_SPLIT), bit for bit; an unknown value fails through op::error."""
    import torch
    from openpose_amd.api import PRECISION_SPLIT, Net, PoseExtractor

    with tempfile.TemporaryDirectory() as d:
        path, producer, scales, sizes, xs, field = _inputs(d)
        np.float32(2.0).tofile(os.path.join(d, "fns_scale.f32"))
        env = dict(os.environ, OPENPOSE_HIP_PRECISION="split")
        r = subprocess.run([BIN, d], capture_output=True, text=True, timeout=180, env=env)
        assert r.returncode == 0 and "pose driver ok" in r.stdout, r.stderr + r.stdout

        net = Net(ctx, "builtin:BODY_25", caffemodel=path)
        net.set_precision(PRECISION_SPLIT)
        dev = [torch.from_numpy(x).cuda() for x in xs]
        pose = PoseExtractor(ctx, net)
        pose.set_property(0, 0.06)
        pose.forward(dev[0], producer)
        kp, sc = pose.keypoints(0)
        gk, gs, _ = _result(d, "single")
        np.testing.assert_array_equal(gk, kp)
        np.testing.assert_array_equal(gs, sc)
        heat = pose.heatmaps_numpy()
        np.testing.assert_array_equal(_read(d, "single_heat.f32").reshape(heat.shape[1:]), heat[0])
        np.testing.assert_array_equal(_read(d, "single_cand.f32").reshape(25, 128, 3),
                                      pose.peaks_numpy()[0])
        pose.close()
        net.forward(dev[0])
        split_out = net.output_numpy().ravel()
        np.testing.assert_array_equal(_read(d, "net_out0.f32"), split_out)
        # and it is the split net, not the fp16 one
        n16 = Net(ctx, "builtin:BODY_25", caffemodel=path)
        n16.forward(dev[0])
        assert not np.array_equal(n16.output_numpy().ravel(), split_out)

        bad = dict(os.environ, OPENPOSE_HIP_PRECISION="fp32")
        r = subprocess.run([BIN, d], capture_output=True, text=True, timeout=180, env=bad)
        assert r.returncode != 0 and "OPENPOSE_HIP_PRECISION must be fp16 or split" in r.stderr, \
            r.stderr + r.stdout
