"""GPU: every conv kernel launch of the BODY_25 forward at the bench geometry, checked layer by
layer against the fp16-storage emulation (oracle/fp16.py) fed with the GPU's OWN fp16 input of
that layer -- so the only freedom left is the fp32 summation order, and a wrong kernel (a wrong
lane, fragment, tap, bias or pooling partner) cannot hide in the whole-net tolerance.

Geometry: the bench's (bench.py): BODY_25 at 656x368 with the tile-aligned batch
(tile_aligned_batch: 130 frames on a 256-CU MI355X), so every kernel instantiation the bench
launches -- conv1_fused, conv3w<128/96>, conv3w8<128, 1/2/4> with and without the pooled epilogue,
conv_head<512/256, 2/4>, the 16-wave conv3 1x1 tiles -- runs here with the bench's grid and tile
walk.  Frames 0, n//2 - 1 (64 at 130 frames) and the last one are checked (first, middle,
last tile rounds).

Bound per output element (oracle/fp16.py): |gpu - ref| <= 2 ulp16(ref) + C_ACC * S,
S = sum |w x| + |b|.  C_ACC = 2^-16 (one conv) / 2^-14 (kernels with an fp16 intermediate on
chip, whose 1-ulp intermediate differences reach the second conv).  Biases and PReLU slopes are
random (non-zero biases, slopes in (0.05, 0.5)).  Reference layers:
models/pose/body_25/pose_deploy.prototxt, NetCaffe::forwardPass (netCaffe.cpp:248).
"""
import numpy as np
import pytest
import torch

from oracle import body25
from oracle import fp16 as emu
from openpose_amd import synth
from openpose_amd.api import Net, dev_switches

pytestmark = pytest.mark.gpu

C_ACC = 2.0 ** -16          # one conv per kernel
C_ACC_CHAINED = 2.0 ** -14  # conv1_1 -> conv1_2 and Mconv6 -> Mconv7 inside one kernel
NET_H, NET_W = 368, 656


def random_params(graph, seed):
    """He weights + non-zero biases + PReLU slopes in (0.05, 0.5) (all in [0, 1]: the max
    epilogue the bench runs)."""
    params = synth.he_weights(graph, seed=seed)
    rng = np.random.default_rng(seed + 1)
    out = {}
    for name, (w, b, s) in params.items():
        b = rng.normal(0.0, 0.05, b.shape).astype(np.float32)
        if s is not None:
            s = rng.uniform(0.05, 0.5, s.shape).astype(np.float32)
        out[name] = (w, b, s)
    return out


@pytest.fixture(scope="module")
def bench_net(ctx):
    from bench import tile_aligned_batch
    n = tile_aligned_batch(torch.cuda.get_device_properties(0).multi_processor_count)
    graph = body25.layers()
    params = random_params(graph, 21)
    x = np.random.default_rng(22).uniform(-0.5, 0.5, (n, 3, NET_H, NET_W)).astype(np.float32)
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(params)
    with dev_switches(LAUNCH_LOG=1):
        net.forward(torch.from_numpy(x).cuda())
    log = net.launch_log()
    frames = [0, n // 2 - 1, n - 1]
    yield dict(net=net, graph=graph, params=params, x=x, n=n, log=log, frames=frames)
    net.close()


def test_launch_log_covers_the_bench_kernels(bench_net):
    """The forward launches one kernel per fused unit, and the instantiations are the bench's:
    the fused first layers, both stage-layer kernels, the 8-wave kernel with 1, 2 and 4 n-blocks
    with and without the pooled epilogue, and both head widths."""
    log = bench_net["log"]
    kernels = {k.split("<")[0] for _, k in log}
    assert {"conv1_fused_kernel", "conv3w_kernel", "conv3w8_kernel", "conv_head_kernel"} <= kernels
    inst = {k for _, k in log}
    for nb in (1, 2, 4):
        assert any(k.startswith("conv3w8_kernel<128,%d,0," % nb) for k in inst), nb
    for nb in (1, 2):
        assert any(k.startswith("conv3w8_kernel<128,%d,1," % nb) for k in inst), nb
    for bn in (128, 96):
        assert any(k.startswith("conv3w_kernel<%d," % bn) for k in inst), bn
    for n1 in (512, 256):
        assert any(k.startswith("conv_head_kernel<%d," % n1) for k in inst), n1
    # every conv of the graph is in exactly one launch
    named = [c for layer, _ in log for c in layer.split("+") if c != "pool"]
    convs = [l["name"] for l in bench_net["graph"] if l["type"] == "Convolution"]
    assert sorted(named) == sorted(convs)
    print("%d launches, %d instantiations: %s" % (len(log), len(inst), sorted(inst)))


def _check_unit(bench_net, layer, kernel):
    net, graph, params = bench_net["net"], bench_net["graph"], bench_net["params"]
    u = emu.unit_from_launch(graph, layer)
    chained = len(u["convs"]) > 1
    worst = (0.0, 0.0, 0.0)
    for f in bench_net["frames"]:
        if u["input"] == "image":
            x = bench_net["x"][f:f + 1]
        else:
            x = net.blob(u["input"], (f, 1))
        got = net.blob(u["output"], (f, 1))
        ref, tol = emu.unit(u, x, params, C_ACC_CHAINED if chained else C_ACC)
        assert got.shape == ref.shape, (layer, got.shape, ref.shape)
        d = np.abs(got - ref)
        bad = d > tol
        if bad.any():
            i = np.unravel_index(np.argmax(d - tol), d.shape)
            raise AssertionError("%s (%s) frame %d: %d of %d elements beyond the bound; worst at %s: "
                                 "gpu %r ref %r tol %r" % (layer, kernel, f, int(bad.sum()), d.size,
                                                           i, float(got[i]), float(ref[i]),
                                                           float(tol[i])))
        # in ulp16 where the output rounding dominates the bound (no cancellation)
        ulp = emu.ulp16(ref)
        dom = tol <= 3 * ulp
        ulps = float((d[dom] / ulp[dom]).max()) if dom.any() else 0.0
        worst = tuple(max(a, b) for a, b in zip(worst, (ulps, float((d / tol).max()),
                                                        float(np.abs(ref).max()))))
    return worst


def test_every_launch_within_fp16_bound(bench_net, record_property):
    """Each launch of the bench forward against the fp16-storage emulation of its layers, fed with
    the GPU's own input blob (frames 0, middle, last).  Also the fp32 net_output slices of the two
    final heads."""
    rows = []
    for layer, kernel in bench_net["log"]:
        w = _check_unit(bench_net, layer, kernel)
        rows.append((layer, kernel) + w)
    for layer, kernel, ulps, frac, amax in rows:
        print("%-40s %-30s %.2f ulp16 (rounding-dominated elements)  %.3f of bound  |ref| <= %.3g"
              % (layer, kernel, ulps, frac, amax))
    record_property("max_ulp16", max(r[2] for r in rows))
    record_property("max_frac_of_bound", max(r[3] for r in rows))
    # net_output (fp32): the last heads' slices against the emulation from their own inputs
    net, graph, params = bench_net["net"], bench_net["graph"], bench_net["params"]
    off = 0
    for b in [l for l in graph if l["top"][0] == "net_output"][0]["bottom"]:
        head = [lay for lay, _ in bench_net["log"] if lay.endswith("+" + b)]
        assert len(head) == 1, b
        u = emu.unit_from_launch(graph, head[0])
        u = dict(u, fp32_output=True)
        for f in bench_net["frames"]:
            ref, tol = emu.unit(u, net.blob(u["input"], (f, 1)), params, C_ACC_CHAINED)
            got = net.blob("net_output", (f, 1))[:, off:off + ref.shape[1]]
            assert (np.abs(got - ref) <= tol).all(), (b, f)
        off += ref.shape[1]
    assert off == 78


# ---- split precision (opk_net_set_precision OPK_PRECISION_SPLIT) --------------------------------
# The same bench geometry in split precision: every conv launch -- conv_image<split>, the 8-wave
# conv3w8 split instantiations (96 / 128 channels, 2 and 4 n-blocks), conv3_kernel split for the
# rest -- against the exact (float64) conv of the GPU's own hi + lo input blob (oracle/split.py).
# fp32 accumulation + dropped lo*lo + weight residue (oracle/split.py); the worst launch measured
# 0.041 of 2^-16 (round 6, r6b), so 2^-19 keeps ~3x headroom -- a missing or misplaced pass
# (~2^-11 S) is 250x beyond it
C_SPLIT = 2.0 ** -19


@pytest.fixture(scope="module")
def split_net(ctx):
    from bench import tile_aligned_batch
    from openpose_amd.api import PRECISION_SPLIT
    n = tile_aligned_batch(torch.cuda.get_device_properties(0).multi_processor_count)
    graph = body25.layers()
    params = random_params(graph, 31)
    x = np.random.default_rng(32).uniform(-0.5, 0.5, (n, 3, NET_H, NET_W)).astype(np.float32)
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(params)
    net.set_precision(PRECISION_SPLIT)
    with dev_switches(LAUNCH_LOG=1):
        net.forward(torch.from_numpy(x).cuda())
    log = net.launch_log()
    yield dict(net=net, graph=graph, params=params, x=x, n=n, log=log, frames=[0, n - 1])
    net.close()


def test_split_launch_log_uses_fused_kernels(split_net):
    """Split precision runs the 8-wave persistent kernel's split instantiations for the 512-position
    layers (1, 2 and 4 n-blocks of 128, 96 and 64 channels; pool1 / pool2 / pool3 in the epilogue),
    the first conv on conv_image<split> and the 1x1 head pairs on conv_head<split>; every conv
    kernel is a split instantiation and every conv is launched (the 64-channel full-resolution
    layer as frame runs)."""
    inst = {k for _, k in split_net["log"]}
    for nb in (1, 2, 4):
        assert any(k.startswith("conv3w8_kernel<128,%d,0," % nb) and k.endswith(",split>") for k in inst), nb
    for nb in (1, 2):   # conv2_2 + pool2, conv3_4 + pool3: the split pooled epilogue
        assert any(k.startswith("conv3w8_kernel<128,%d,1," % nb) and k.endswith(",split>") for k in inst), nb
    # conv1_2 + pool1 on the 64-channel tile
    assert any(k.startswith("conv3w8_kernel<64,1,1,") and k.endswith(",split>") for k in inst)
    assert any(k.startswith("conv3w8_kernel<96,1,0,") and k.endswith(",split>") for k in inst)
    assert "conv_image_kernel<split>" in inst
    # the Mconv6 + Mconv7 pairs on conv_head_kernel's split instantiations (N1 = 256 and 512)
    for n1 in (256, 512):
        assert any(k.startswith("conv_head_kernel<%d," % n1) and k.endswith(",split>") for k in inst), n1
    # (and so no conv of the bench net is left on the generic conv3_kernel)
    assert not any(k.startswith("conv3_kernel") for k in inst), inst
    convk = [k for k in inst if k.startswith(("conv3", "conv_image", "conv_head"))]
    assert all("split" in k for k in convk), convk
    assert not any(k.startswith(("conv3w_", "conv1_fused")) for k in inst), inst
    # (the full-resolution layers of 130 frames run as frame runs: several launches, one layer)
    named = {c for layer, _ in split_net["log"] for c in layer.split("+") if c != "pool"}
    convs = [l["name"] for l in split_net["graph"] if l["type"] == "Convolution"]
    assert sorted(named) == sorted(convs)
    print("%d launches: %s" % (len(split_net["log"]), sorted(inst)))


def test_split_every_launch_within_bound(split_net, record_property):
    """Each conv launch of the split-precision bench forward against the float64 conv of the GPU's
    own hi + lo input blob (frames 0 and last): |gpu - ref| <= 2^-19 S + 2^-21 |ref| + 2^-24."""
    from oracle import split as sp
    net, graph, params = split_net["net"], split_net["graph"], split_net["params"]
    worst = 0.0
    rows = []
    for layer, kernel in split_net["log"]:
        if layer == "pool":
            continue
        u = emu.unit_from_launch(graph, layer)
        frac = 0.0
        for f in split_net["frames"]:
            x = split_net["x"][f:f + 1] if u["input"] == "image" else net.blob(u["input"], (f, 1))
            ref, tol = sp.unit(u, x, params, C_SPLIT)
            got = net.blob(u["output"], (f, 1))   # (hi + lo; net_output heads: fp32)
            assert got.shape == ref.shape, (layer, got.shape, ref.shape)
            d = np.abs(got.astype(np.float64) - ref)
            bad = d > tol
            if bad.any():
                i = np.unravel_index(np.argmax(d - tol), d.shape)
                raise AssertionError("%s (%s) frame %d: %d of %d elements beyond the split bound; "
                                     "worst at %s: gpu %r ref %r tol %r"
                                     % (layer, kernel, f, int(bad.sum()), d.size, i, float(got[i]),
                                        float(ref[i]), float(tol[i])))
            frac = max(frac, float((d / tol).max()))
        rows.append((layer, kernel, frac))
        worst = max(worst, frac)
    for layer, kernel, frac in rows:
        print("%-40s %-40s %.3f of bound" % (layer, kernel, frac))
    record_property("report_max_frac_of_split_bound", round(worst, 4))
    record_property("report_split_worst_launch", max(rows, key=lambda r: r[2])[:2])

