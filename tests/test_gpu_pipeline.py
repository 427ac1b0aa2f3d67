"""GPU: whole hot path through libopk_hip.so against the committed fixtures and the oracle.

* connector fixtures hold the REFERENCE's own connector outputs (oracle/_ref): the GPU pipeline
  (GPU NMS -> GPU PAF integrals -> host assembly) must reproduce them bit for bit;
* NMS / resize fixtures: bit-exact; CNN fixture: relative L2 < 2e-2 (fp16 MFMA vs fp32);
* end-to-end on 656x368 frames: GPU keypoints vs the fp32 CPU pipeline within 1e-3 net-input
  pixels (north_star tolerance; x, y are reported in 1280x720 frame pixels = net pixels x
  scaleNetToOutput 1.959), scores within 1e-3, identical people and found parts.
"""
import glob
import os

import numpy as np
import pytest
import torch

import oracle
from oracle import body25
from openpose_amd import synth
from openpose_amd.api import Net, PoseExtractor, dev_switches
from openpose_amd.pose_tables import BODY_135, CONNECT_GPU
from tests.golden.make_golden import connector_field

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KEYPOINT_TOL = 1e-3


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "connector_*.npz"))),
                         ids=lambda p: os.path.basename(p))
def test_gpu_connector_matches_reference_fixture(ctx, path):
    g = np.load(path, allow_pickle=False)
    f = connector_field(str(g["kind"]), int(g["n_people"]), int(g["seed"]), int(g["h"]), int(g["w"]))
    scale = float(g["scale"])
    off = float(np.float32(0.5 / scale))
    peaks = torch.zeros((1, 25, 128, 3), device="cuda")
    heat = _dev(f[None])
    ctx.nms(peaks, heat, 0.05, (off, off))
    np.testing.assert_array_equal(peaks.cpu().numpy()[0], g["peaks"])
    kp, ks = ctx.connect_body_parts(heat, peaks, scale=scale,
                                    maximize_positives=bool(g["maximize_positives"]))
    np.testing.assert_array_equal(kp, g["keypoints"])
    np.testing.assert_array_equal(ks, g["scores"])


@pytest.mark.parametrize("name", ["people", "noise", "plateau"])
def test_gpu_nms_fixture(ctx, name):
    g = np.load(os.path.join(GOLDEN, "nms_%s.npz" % name), allow_pickle=False)
    peaks = torch.zeros((1, 25, 128, 3), device="cuda")
    ctx.nms(peaks, _dev(g["field"][None]), 0.05, (0.25, 0.5))
    got, ref = peaks.cpu().numpy()[0], g["peaks"]
    for c in range(25):
        n = int(ref[c, 0, 0])
        assert int(got[c, 0, 0]) == n
        np.testing.assert_array_equal(got[c, 1:n + 1], ref[c, 1:n + 1])


def test_gpu_resize_fixture(ctx):
    g = np.load(os.path.join(GOLDEN, "resize.npz"), allow_pickle=False)
    out = torch.empty((1, 2, 80, 160), device="cuda")
    ctx.resize_and_merge(out, [_dev(g["src"][None])])
    np.testing.assert_array_equal(out.cpu().numpy()[0], g["out"])
    ctx.resize_and_merge(out, [_dev(g["ms_src%d" % i][None]) for i in range(3)])
    np.testing.assert_array_equal(out.cpu().numpy()[0], g["ms_out"])


def test_gpu_cnn_fixture(ctx):
    g = np.load(os.path.join(GOLDEN, "cnn_body25_64x96.npz"), allow_pickle=False)
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(synth.he_weights(body25.layers(), seed=int(g["weight_seed"])))
    net.forward(_dev(g["input"]))
    got, ref = net.output_numpy(), g["net_output"]
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 2e-2


def test_pose_injection_batch_bitexact(ctx):
    """poseNetOutput path (poseExtractorCaffe.cpp:249-262) on 3 frames at once."""
    fields = np.stack([synth.overlay(k + 2, 46, 82, seed=600 + k) +
                       np.random.default_rng(k).normal(0, 0.01, (78, 46, 82)).astype(np.float32)
                       for k in range(3)]).astype(np.float32)
    pose = PoseExtractor(ctx, None)
    net_out = _dev(fields)   # stays alive: heat maps are evaluated lazily from it
    pose.forward_net_output(net_out, (656, 368), (1280, 720))
    s = pose.scale_net_to_output()
    assert abs(s - 1.959128) < 1e-5                  # poseExtractorCaffe.cpp:306-310
    off = float(np.float32(0.5 / np.float64(s)))
    gpu_peaks = pose.peaks_numpy()
    gpu_heat = pose.heatmaps_numpy()                 # materialised on request
    for k in range(3):
        heat = oracle.resize_merge([fields[k]], 368, 656)
        peaks = oracle.nms(heat, 0.05, 128, (off, off))
        rk, rs = oracle.connect(heat, peaks, scale=s)
        kp, ks = pose.keypoints(k)
        assert len(kp) >= 1
        np.testing.assert_array_equal(kp, rk)
        np.testing.assert_array_equal(ks, rs)
        for c in range(25):
            n = int(peaks[c, 0, 0])
            assert int(gpu_peaks[k, c, 0, 0]) == n
            np.testing.assert_array_equal(gpu_peaks[k, c, 1:n + 1], peaks[c, 1:n + 1])
        np.testing.assert_array_equal(gpu_heat[k], heat)


def test_end_to_end_keypoints_within_tolerance(ctx):
    """CNN (fp16 MFMA) + overlay + resize + NMS + connector vs the fp32 CPU pipeline, 656x368."""
    graph = body25.layers()
    params = synth.he_weights(graph, seed=7, out_scale=0.02)
    x = np.random.default_rng(8).uniform(-0.5, 0.5, (2, 3, 368, 656)).astype(np.float32)
    ov = np.stack([synth.overlay(5, 46, 82, seed=900 + k) for k in range(2)]).astype(np.float32)
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(params)
    pose = PoseExtractor(ctx, net)
    ovd = _dev(ov)
    pose.set_overlay(ovd)
    pose.forward(_dev(x), (1280, 720))
    s = pose.scale_net_to_output()
    off = float(np.float32(0.5 / np.float64(s)))
    for k in range(2):
        out = body25.forward(x[k:k + 1], params, graph=graph)[0] + ov[k]
        heat = oracle.resize_merge([out], 368, 656)
        peaks = oracle.nms(heat, 0.05, 128, (off, off))
        rk, rs = oracle.connect(heat, peaks, scale=s)
        kp, ks = pose.keypoints(k)
        assert kp.shape == rk.shape and len(kp) >= 3
        np.testing.assert_array_equal(kp[..., 2] > 0, rk[..., 2] > 0)   # same parts found
        assert np.abs(kp[..., :2] - rk[..., :2]).max() / s <= KEYPOINT_TOL
        assert np.abs(ks - rs).max() <= KEYPOINT_TOL


# Stated parity bounds at full strength (random He weights, out_scale 1, no overlay: every peak
# comes from the CNN, ~2,400 peaks per frame, many of them near-ties of neighbouring pixels).
# fp16 storage of ~100 layers' activations moves the net output by rel-L2 ~2e-3, which flips the
# order of pixels whose fp32 values differ by less than that: those peaks move by one pixel.
# Measured (round 5, profiles/round5/): rel-L2 1.5e-3, 90.4 % of 18,658 fp32 peaks at the
# identical pixel, 97.5 % within 1 px, people 348 vs 346 (the bench's parity block on its own
# frames: 93.6 % / 98.3 %).
UNSCALED_REL_L2 = 5e-3
UNSCALED_PEAKS_IDENTICAL = 0.88   # fraction of fp32 peaks detected at the identical pixel
UNSCALED_PEAKS_WITHIN_1PX = 0.96
UNSCALED_PEOPLE_DELTA = 0.03      # |people - fp32 people| / fp32 people


def _unscaled_parity(ctx, precision=None):
    """Full-strength heads (out_scale 1, no overlay) at 656x368, two frames: (1) post-processing
    isolated, bit-exact; (2) the CNN's drift against the fp32 oracle through the whole chain.
    Returns the measured quantities."""
    from oracle import parity
    graph = body25.layers()
    params = synth.he_weights(graph, seed=31, out_scale=1.0)
    x = np.random.default_rng(32).uniform(-0.5, 0.5, (2, 3, 368, 656)).astype(np.float32)
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(params)
    if precision is not None:
        net.set_precision(precision)
    pose = PoseExtractor(ctx, net)
    pose.forward(_dev(x), (1280, 720))
    s = pose.scale_net_to_output()
    off = float(np.float32(0.5 / np.float64(s)))
    gpu_outs = net.output_numpy()
    stats = {"fp32_peaks": 0, "same": 0.0, "near": 0.0, "shift": 0.0, "kshift": 0.0,
             "people": 0, "people32": 0, "num": 0.0, "den": 0.0, "exact": 0}
    for k in range(2):
        gpu_out = gpu_outs[k]
        gpu_peaks = pose.peaks_numpy()[k]
        kp, ks = pose.keypoints(k)

        heat = oracle.resize_merge([gpu_out], 368, 656)
        peaks = oracle.nms(heat, 0.05, 128, (off, off))
        rk, rs = oracle.connect(heat, peaks, scale=s)
        for c in range(25):
            n = int(peaks[c, 0, 0])
            assert int(gpu_peaks[c, 0, 0]) == n
            np.testing.assert_array_equal(gpu_peaks[c, 1:n + 1], peaks[c, 1:n + 1])
        np.testing.assert_array_equal(kp, rk)
        np.testing.assert_array_equal(ks, rs)

        ref_out = body25.forward(x[k:k + 1], params, graph=graph)[0]
        stats["num"] += float(np.sum((gpu_out.astype(np.float64) - ref_out) ** 2))
        stats["den"] += float(np.sum(ref_out.astype(np.float64) ** 2))
        heat32 = oracle.resize_merge([ref_out], 368, 656)
        total, same, near = parity.compare_peaks(parity.peak_mask(heat32, 0.05, 25),
                                                 parity.peak_mask(heat, 0.05, 25))
        peaks32 = oracle.nms(heat32, 0.05, 128, (off, off))
        rk32, _ = oracle.connect(heat32, peaks32, scale=s)
        kshift, _ = parity.keypoint_shift(rk32, kp, radius=2.0 * s)
        stats["exact"] += parity.people_identical(rk32, kp, 1e-3 * s)
        stats["fp32_peaks"] += total
        stats["same"] += same * total
        stats["near"] += near * total
        stats["shift"] = max(stats["shift"], parity.refined_shift(peaks32, gpu_peaks))
        stats["kshift"] = max(stats["kshift"], kshift)
        stats["people"] += len(kp)
        stats["people32"] += len(rk32)
    total = stats["fp32_peaks"]
    return {"net_rel_l2": (stats["num"] / stats["den"]) ** 0.5, "fp32_peaks": total,
            "peak_index_identical": stats["same"] / total, "peaks_within_1px": stats["near"] / total,
            "max_refined_peak_shift_px": stats["shift"], "max_keypoint_shift_px": stats["kshift"],
            "people_gpu_fp32": (stats["people"], stats["people32"]),
            "people_identical_1e-3": stats["exact"] / max(stats["people32"], 1)}


def _report(record_property, m, tag=""):
    for k, v in m.items():
        record_property("report_" + tag + k, round(v, 6) if isinstance(v, float) else v)


def test_end_to_end_unscaled_heads(ctx, record_property):
    """Full-strength heads (out_scale 1, no overlay) at 656x368, two frames, fp16 precision.

    (1) post-processing isolated: the oracle's resize -> NMS -> connector run on the GPU's OWN net
        output must give the GPU pipeline's peaks and keypoints bit for bit;
    (2) fp16-vs-fp32 CNN drift, measured and bounded: the same chain on the fp32 oracle net
        output; the fraction of fp32 NMS peaks (nmsCpu's integer pixels, oracle/parity.py) the GPU
        finds at the identical pixel and within 1 heat-map pixel, the largest refined-peak and
        keypoint shifts and the people counts are printed at the end of the run (conftest:
        report_*) and checked against the UNSCALED_* bounds above.
    poseExtractorCaffe.cpp:246-333 is the chain both sides follow."""
    m = _unscaled_parity(ctx)
    _report(record_property, m)
    assert m["net_rel_l2"] < UNSCALED_REL_L2
    assert m["fp32_peaks"] > 0 and m["peak_index_identical"] >= UNSCALED_PEAKS_IDENTICAL
    assert m["peaks_within_1px"] >= UNSCALED_PEAKS_WITHIN_1PX
    p, p32 = m["people_gpu_fp32"]
    assert abs(p - p32) / max(p32, 1) <= UNSCALED_PEOPLE_DELTA


# Split precision (opk_net_set_precision OPK_PRECISION_SPLIT): the same field, the same chain.
SPLIT_REL_L2 = 5e-5
SPLIT_PEAKS_IDENTICAL = 0.998
SPLIT_PEOPLE_IDENTICAL = 0.95   # fp32 people reproduced with every keypoint within 1e-3 net px


def test_end_to_end_unscaled_heads_split_precision(ctx, record_property):
    """The full-strength field of test_end_to_end_unscaled_heads with the net in split precision
    (fp16 hi/lo pairs, three MFMA passes): the north star's "peak indices bit-exact, keypoints
    within 1e-3 of the CPU reference" on a CNN-driven field, measured and bounded (SPLIT_*)."""
    from openpose_amd.api import PRECISION_SPLIT
    m = _unscaled_parity(ctx, PRECISION_SPLIT)
    _report(record_property, m, "split_")
    assert m["net_rel_l2"] < SPLIT_REL_L2
    assert m["peak_index_identical"] >= SPLIT_PEAKS_IDENTICAL
    assert m["people_identical_1e-3"] >= SPLIT_PEOPLE_IDENTICAL


def test_pose_submit_collect_pipeline(ctx):
    """Two batches in flight (opk_pose_submit / opk_pose_collect) give the synchronous results."""
    def fields(seed):
        return np.stack([synth.overlay(3, 46, 82, seed=seed + k) +
                         np.random.default_rng(seed + k).normal(0, 0.01, (78, 46, 82))
                         for k in range(2)]).astype(np.float32)

    fa, fb = fields(700), fields(800)
    sync = PoseExtractor(ctx, None)
    ref = []
    for f in (fa, fb):
        d = _dev(f)
        sync.forward_net_output(d, (656, 368), (1280, 720))
        ref.append([sync.keypoints(k) for k in range(2)])
    pipe = PoseExtractor(ctx, None)
    da, db = _dev(fa), _dev(fb)
    pipe.submit_net_output(da, (656, 368), (1280, 720))
    pipe.submit_net_output(db, (656, 368), (1280, 720))
    assert pipe.pending() == 2
    for r in ref:
        assert pipe.collect() == 2
        for k in range(2):
            kp, ks = pipe.keypoints(k)
            np.testing.assert_array_equal(kp, r[k][0])
            np.testing.assert_array_equal(ks, r[k][1])
    assert pipe.pending() == 0


GPU_CONN = sorted(glob.glob(os.path.join(GOLDEN, "gpuconn_*.npz")))


@pytest.mark.parametrize("path", GPU_CONN, ids=lambda p: os.path.basename(p))
def test_gpu_connector_gpu_semantics_matches_reference_fixture(ctx, path):
    """connectBodyPartsGpu semantics (any model): GPU NMS + GPU PAF integrals + global-sort
    assembly reproduce the reference's own outputs (random-score fixtures: CPU tests only)."""
    g = np.load(path, allow_pickle=False)
    kind = str(g["kind"])
    if not kind.startswith("people"):
        pytest.skip("random pair scores have no heat map")
    t = oracle.pose_tables()[int(g["model"])]
    h, w = int(g["h"]), int(g["w"])
    sk = synth.people_model(t, int(g["n_people"]), h, w, int(g["seed"]))
    sc = h / 368.0
    f = synth.render_field(sk, h, w, sigma=max(1.0, 7.0 * sc), paf_width=max(1.0, 6.0 * sc), table=t)
    if kind == "people_noface":
        f[65:t["parts"]] = 0
    scale = float(g["scale"])
    off = float(np.float32(0.5 / scale))
    peaks = torch.zeros((1, t["parts"], 128, 3), device="cuda")
    heat = _dev(f[None])
    ctx.nms(peaks, heat, 0.05, (off, off))
    np.testing.assert_array_equal(peaks.cpu().numpy()[0], g["peaks"])
    kp, ks = ctx.connect_body_parts(heat, peaks, pose_model=int(g["model"]), scale=scale,
                                    maximize_positives=bool(g["maximize_positives"]),
                                    semantics=CONNECT_GPU)
    np.testing.assert_array_equal(kp, g["keypoints"])
    np.testing.assert_array_equal(ks, g["scores"])


@pytest.mark.parametrize("spl", [1, 0])
@pytest.mark.parametrize("model,people", [(BODY_135, 20), (0, 5), (0, 20)])
def test_pose_injection_gpu_semantics(ctx, model, people, spl):
    """BODY_135 through the poseNetOutput injection path -- 439 x 46 x 82
    net output, 20 synthetic people, GPU-path connector -- bit-exact against the oracle chain
    (resize -> NMS -> getScoreAB table -> global-sort assembly); BODY_25 with the same semantics.
    5 people: every pair's line integrals read the sources through L2; 20 people (>= 64 candidate
    lines per pair): through the planes staged in LDS (paf.hip).  spl: the line integrals with one
    sample per lane (the default) and with one line per lane (PAF_SPL=0)."""
    with dev_switches(PAF_SPL=spl):
        _pose_injection_gpu_semantics(ctx, model, people)


def _pose_injection_gpu_semantics(ctx, model, people):
    t = oracle.pose_tables()[model]
    C = t["parts"] + int(t["bkg"]) + len(t["map_idx"])
    fields = np.stack([synth.overlay(people, 46, 82, seed=1500 + k, table=t) +
                       np.random.default_rng(k).normal(0, 0.01, (C, 46, 82)).astype(np.float32)
                       for k in range(2)]).astype(np.float32)
    pose = PoseExtractor(ctx, None, pose_model=model, semantics=CONNECT_GPU)
    net_out = _dev(fields)
    pose.forward_net_output(net_out, (656, 368), (1280, 720))
    s = pose.scale_net_to_output()
    off = float(np.float32(0.5 / np.float64(s)))
    gpu_peaks = pose.peaks_numpy()
    assert gpu_peaks.shape == (2, t["parts"], 128, 3)
    for k in range(2):
        heat = oracle.resize_merge([fields[k]], 368, 656)
        peaks = oracle.nms(heat, 0.05, 128, (off, off), channels=t["parts"])
        np.testing.assert_array_equal(gpu_peaks[k], peaks)
        ps = oracle.pair_scores_table(heat, peaks, t)
        rk, rs = oracle.connect_gpu_semantics(ps, peaks, t, scale=s)
        kp, ks = pose.keypoints(k)
        assert len(kp) >= 1
        np.testing.assert_array_equal(kp, rk)
        np.testing.assert_array_equal(ks, rs)


def test_pose_injection_mixed_record_lengths(ctx):
    """One BODY_135 batch whose frames' PAF records are longer than the eagerly copied head
    (kRecordHead floats: 20+ people) and shorter (0-3 people) in alternation: the long records come
    over in one 2-D copy spanning short frames too, the frames are assembled by the worker pool in
    any order; every frame bit-exact against the oracle chain, over two batches in flight."""
    t = oracle.pose_tables()[BODY_135]
    C = t["parts"] + int(t["bkg"]) + len(t["map_idx"])
    people = [1, 20, 0, 25, 3, 20]
    fields = np.stack([synth.overlay(p, 46, 82, seed=4100 + k, table=t) +
                       np.random.default_rng(k).normal(0, 0.01, (C, 46, 82)).astype(np.float32)
                       for k, p in enumerate(people)]).astype(np.float32)
    pose = PoseExtractor(ctx, None, pose_model=BODY_135, semantics=CONNECT_GPU)
    order = [np.arange(len(people)), np.arange(len(people))[::-1]]
    devs = [_dev(np.ascontiguousarray(fields[o])) for o in order]
    for d in devs:
        pose.submit_net_output(d, (656, 368), (1280, 720))
    ref = {}
    for o in order:
        pose.collect()
        s = pose.scale_net_to_output()
        off = float(np.float32(0.5 / np.float64(s)))
        for k, src in enumerate(o):
            if src not in ref:
                heat = oracle.resize_merge([fields[src]], 368, 656)
                peaks = oracle.nms(heat, 0.05, 128, (off, off), channels=t["parts"])
                ps = oracle.pair_scores_table(heat, peaks, t)
                ref[src] = oracle.connect_gpu_semantics(ps, peaks, t, scale=s)
            kp, ks = pose.keypoints(k)
            np.testing.assert_array_equal(kp, ref[src][0])
            np.testing.assert_array_equal(ks, ref[src][1])
            assert (len(kp) > 0) == (people[src] > 0)


def _multiscale_case(ctx, nscales, gap, seed, nms_stream=1, nms_walk=None, frames=2):
    """--scale_number nscales --scale_gap gap through opk_pose_forward_multi, sizes from
    ScaleAndSizeExtractor (scaleAndSizeExtractor.cpp:74-88); merged heat maps (resizeAndMergeCpu
    average, resizeAndMergeBase.cpp:55-106), peaks and people bit-identical to the oracle chain fed
    with the same per-scale net outputs.  nms_stream=0: the windowed lazy NMS instead of the
    streaming walk (dev switch; the same candidates)."""
    from openpose_amd.api import dev_switches, scale_and_size
    _, net_sizes = scale_and_size((1280, 720), (-1, 368), 1.0, nscales, gap)
    sizes = [(h, w) for (w, h) in net_sizes]
    graph = body25.layers()
    params = synth.he_weights(graph, seed=seed, out_scale=0.02)
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(params)
    rng = np.random.default_rng(seed + 1)
    xs = [rng.uniform(-0.5, 0.5, (frames, 3, h, w)).astype(np.float32) for h, w in sizes]
    outs = []
    for x in xs:
        net.forward(_dev(x))
        outs.append(net.output_numpy())
    assert [o.shape[2:] for o in outs] == [(h // 8, w // 8) for h, w in sizes]
    # the overlay rides on scale 0 only: scaled so that the average over the scales keeps people
    ov = np.stack([synth.overlay(4, 46, 82, seed=2300 + k) for k in range(frames)]).astype(np.float32)
    ov *= np.float32(max(1.0, nscales / 4.0))
    pose = PoseExtractor(ctx, net)
    ovd = _dev(ov)
    pose.set_overlay(ovd)
    sw = dict(NMS_STREAM=nms_stream)
    if nms_walk is not None:
        sw["NMS_WALK"] = nms_walk
    with dev_switches(**sw):
        pose.forward_multi([_dev(x) for x in xs], (1280, 720))
    s = pose.scale_net_to_output()
    assert abs(s - 1.959128) < 1e-5
    off = float(np.float32(0.5 / np.float64(s)))
    gpu_heat = pose.heatmaps_numpy()
    gpu_peaks = pose.peaks_numpy()
    for k in range(frames):
        heat = oracle.resize_merge([outs[0][k] + ov[k]] + [o[k] for o in outs[1:]], 368, 656)
        np.testing.assert_array_equal(gpu_heat[k], heat)
        peaks = oracle.nms(heat, 0.05, 128, (off, off))
        np.testing.assert_array_equal(gpu_peaks[k], peaks)
        rk, rs = oracle.connect(heat, peaks, scale=s)
        kp, ks = pose.keypoints(k)
        assert len(kp) >= 1
        np.testing.assert_array_equal(kp, rk)
        np.testing.assert_array_equal(ks, rs)


def test_multiscale_config4_bitexact(ctx):
    """four scales (nets 656x368, 480x272, 320x176, 160x80) through
    opk_pose_forward_multi, bit-identical to the oracle chain (the 4-source streaming NMS walk)."""
    from openpose_amd.api import scale_and_size
    assert scale_and_size((1280, 720), (-1, 368), 1.0, 4, 0.25)[1] == \
        [(656, 368), (480, 272), (320, 176), (160, 80)]
    _multiscale_case(ctx, 4, 0.25, 21)


@pytest.mark.parametrize("nscales,gap,nms_stream", [(2, 0.25, 1), (3, 0.25, 1), (6, 0.15, 1),
                                                    (2, 0.25, 0), (3, 0.3, 0), (4, 0.25, 0)])
def test_multiscale_other_scale_numbers_bitexact(ctx, nscales, gap, nms_stream):
    """--scale_number 2 / 3 (the 2- and 3-source streaming NMS walks) and 6 (more than 4 sources:
    the windowed lazy NMS), and the windowed kernel for 2-4 sources (NMS_STREAM=0)."""
    _multiscale_case(ctx, nscales, gap, 40 + nscales, nms_stream)


@pytest.mark.parametrize("walk", [0, 8])
@pytest.mark.parametrize("nscales", [1, 4])
def test_nms_walk_variants_bitexact(ctx, walk, nscales):
    """Both streaming NMS walks -- the two-columns-per-lane walk (nms_detect_walk2_kernel, the
    default) and the one-column ring walk (NMS_WALK=0) -- give the oracle's peaks and people, with
    1 and 4 sources (the other tests run the default)."""
    _multiscale_case(ctx, nscales, 0.25, 90 + nscales, 1, walk)


def test_collect_copy_sizes_adapt(ctx):
    """collect() copies the first rows of every part's peak block and the first floats of every
    frame's records, sized from the previous batches: a batch with far more peaks / longer records
    than the last one (1 person, then 24 with noise peaks, then 1 again, on BODY_25 and the GPU-path
    connector over BODY_135) is fetched whole where needed -- peaks, candidates and people
    bit-exact against the oracle chain for every batch."""
    for model, sem in ((0, None), (BODY_135, CONNECT_GPU)):
        t = oracle.pose_tables()[model]
        C = t["parts"] + int(t["bkg"]) + len(t["map_idx"])
        pose = PoseExtractor(ctx, None, pose_model=model, **({"semantics": sem} if sem is not None else {}))
        for k, people in enumerate((1, 24, 1)):
            rng = np.random.default_rng(6100 + k)
            fields = np.stack([synth.overlay(people, 46, 82, seed=6100 + 10 * k + f, table=t) +
                               rng.normal(0, 0.03 if people > 1 else 0.005, (C, 46, 82))
                               for f in range(2)]).astype(np.float32)
            pose.forward_net_output(_dev(fields), (656, 368), (1280, 720))
            s = pose.scale_net_to_output()
            off = float(np.float32(0.5 / np.float64(s)))
            gpu_peaks = pose.peaks_numpy()
            for f in range(2):
                heat = oracle.resize_merge([fields[f]], 368, 656)
                peaks = oracle.nms(heat, 0.05, 128, (off, off), channels=t["parts"])
                np.testing.assert_array_equal(gpu_peaks[f], peaks)
                if sem is None:
                    rk, rs = oracle.connect(heat, peaks, scale=s)
                else:
                    rk, rs = oracle.connect_gpu_semantics(oracle.pair_scores_table(heat, peaks, t),
                                                          peaks, t, scale=s)
                kp, ks = pose.keypoints(f)
                np.testing.assert_array_equal(kp, rk)
                np.testing.assert_array_equal(ks, rs)
                cand = pose.candidates(f)   # (read from the host copy of the peaks)
                counts = peaks[:, 0, 0].astype(int)
                for part in range(t["parts"]):
                    np.testing.assert_array_equal(cand[part][:, 2], peaks[part, 1:counts[part] + 1, 2])
        pose.close()


@pytest.mark.parametrize("kind", ["spikes", "borderline_noise", "plateau", "negative"])
def test_nms_cold_windows_bitexact(ctx, kind):
    """The walk's cold-window skip (nms_detect_walk2_kernel COLD: a source window whose rows are
    bounded by th is not evaluated) on fields built around its bound: isolated one-pixel spikes just
    above the threshold in an otherwise zero map (hot windows next to cold ones), noise whose window
    maxima straddle th / 1.375, a plateau at th / 1.375 +- 1 ulp, and negative fields (the bound is
    on |h|).  Peaks bit-identical to the oracle's nmsCpu, and to the walk with the skip off."""
    rng = np.random.default_rng({"spikes": 1, "borderline_noise": 2, "plateau": 3, "negative": 4}[kind])
    shape = (2, 78, 46, 82)
    th = np.float32(0.05)
    if kind == "spikes":
        f = np.zeros(shape, np.float32)
        for _ in range(600):
            k, c, y, x = rng.integers(0, 2), rng.integers(0, 25), rng.integers(0, 46), rng.integers(0, 82)
            f[k, c, y, x] = rng.uniform(0.04, 0.2)
    elif kind == "borderline_noise":
        f = rng.normal(0, th / 1.375 / 2.5, shape).astype(np.float32)
    elif kind == "plateau":
        b = np.float32(th / np.float32(1.375))
        f = np.full(shape, b, np.float32)
        f += rng.choice(np.array([0, 1, -1], np.float32), shape) * np.spacing(b)
        f[:, :, 20:26, 30:40] += np.float32(0.02) * rng.random((2, 78, 6, 10), np.float32)
    else:
        f = -np.abs(rng.normal(0, 0.06, shape)).astype(np.float32)
        f[:, :, 10:14, 10:14] = np.float32(0.3) * rng.random((2, 78, 4, 4), np.float32)
    got = {}
    for cold in (1, 0):
        pose = PoseExtractor(ctx, None)
        with dev_switches(NMS_COLD=cold):
            pose.forward_net_output(_dev(f), (656, 368), (1280, 720))
        got[cold] = pose.peaks_numpy()
        s = pose.scale_net_to_output()
        pose.close()
    off = float(np.float32(0.5 / np.float64(s)))
    np.testing.assert_array_equal(got[1], got[0])
    found = 0
    for k in range(2):
        peaks = oracle.nms(oracle.resize_merge([f[k]], 368, 656), 0.05, 128, (off, off))
        np.testing.assert_array_equal(got[1][k], peaks)
        found += int(peaks[:, 0, 0].sum())
    assert found > 0


def test_nms_one_frame(ctx):
    """A batch of one frame (25 planes) through the streaming walk: peaks and people the oracle's."""
    _multiscale_case(ctx, 1, 0.25, 97, 1, 8, frames=1)


def _resize_get_scale_factor(init, target):
    """resizeGetScaleFactor (src/openpose/utilities/openCv.cpp:182-195)"""
    return min((target[0] - 1) / float(init[0] - 1), (target[1] - 1) / float(init[1] - 1))


@pytest.mark.parametrize("ratio", [4.0, 2.5, 16.0, 1.0])
def test_upsampling_ratio_bitexact(ctx, ratio):
    """--upsampling_ratio (flags.hpp:136): the heat maps are round(h * r - 1) + 1 rows of the
    46 x 82 net output (ResizeAndMergeCaffe::Reshape, resizeAndMergeCaffe.cpp:77-81, with
    reshapePoseExtractorCaffe's netFactor = r, poseExtractorCaffe.cpp:47-54), NMS and the connector
    run at that size, and scaleNetToOutput comes from mNetOutputSize = round(r / 8 x net input)
    (poseExtractorCaffe.cpp:281-310).  Bit-identical to the oracle chain at that size."""
    rng = np.random.default_rng(77)
    fields = np.stack([synth.overlay(5, 46, 82, seed=7700 + k) +
                       rng.normal(0, 0.01, (78, 46, 82)) for k in range(2)]).astype(np.float32)
    pose = PoseExtractor(ctx, None)
    pose.set_upsampling_ratio(ratio)
    pose.forward_net_output(_dev(fields), (656, 368), (1280, 720))
    f32 = np.float32
    H = int(np.round(f32(46) * f32(ratio) - f32(1))) + 1
    W = int(np.round(f32(82) * f32(ratio) - f32(1))) + 1
    r = f32(ratio) / f32(8)
    out = (int(r * f32(656) + f32(0.5)), int(r * f32(368) + f32(0.5)))
    sp = _resize_get_scale_factor((1280, 720), out)
    net = (int(sp * 1280 + 0.5), int(sp * 720 + 0.5))
    s = f32(_resize_get_scale_factor(net, (1280, 720)))
    assert pose.scale_net_to_output() == s
    off = float(np.float32(0.5 / np.float64(s)))
    gpu_heat = pose.heatmaps_numpy()
    assert gpu_heat.shape == (2, 78, H, W)
    gpu_peaks = pose.peaks_numpy()
    for k in range(2):
        heat = oracle.resize_merge([fields[k]], H, W)
        np.testing.assert_array_equal(gpu_heat[k], heat)
        peaks = oracle.nms(heat, 0.05, 128, (off, off))
        np.testing.assert_array_equal(gpu_peaks[k], peaks)
        rk, rs = oracle.connect(heat, peaks, scale=float(s))
        kp, ks = pose.keypoints(k)
        assert len(kp) >= 1 or ratio < 2
        np.testing.assert_array_equal(kp, rk)
        np.testing.assert_array_equal(ks, rs)
    # the CUDA build's resize accepts x8 only for one source (resizeAndMergeBase.cu:276-300)
    if ratio not in (1.0, 8.0):
        from openpose_amd._lib import OpkError
        pose.set_map_semantics(1)
        with pytest.raises(OpkError, match="8x resize"):
            pose.forward_net_output(_dev(fields), (656, 368), (1280, 720))


def test_two_threads_own_contexts_concurrent(ctx):
    """The drop-in's threading model in-process (wrapperAuxiliary.hpp:328-337: one worker thread per
    --num_gpu, each with its own PoseExtractor): two host threads, each with its own opk context on
    its own stream, net and PoseExtractor, forward concurrently (ctypes drops the GIL in every
    library call) and every repetition gives the single-thread keypoints, peaks and heat maps."""
    import threading
    from openpose_amd.api import Context
    graph = body25.layers()
    params = synth.he_weights(graph, seed=61, out_scale=0.02)
    rng = np.random.default_rng(62)
    x = rng.uniform(-0.5, 0.5, (2, 3, 368, 656)).astype(np.float32)
    ov = np.stack([synth.overlay(4, 46, 82, seed=6300 + k) for k in range(2)]).astype(np.float32)

    def run(c, reps):
        net = Net(c, "builtin:BODY_25")
        net.set_params(params)
        pose = PoseExtractor(c, net)
        pose.set_overlay(_dev(ov))
        res = []
        for _ in range(reps):
            pose.forward(_dev(x), (1280, 720))
            res.append(([pose.keypoints(k) for k in range(2)], pose.peaks_numpy().copy(),
                        pose.heatmaps_numpy().copy()))
        pose.close()
        net.close()
        return res

    ref = run(ctx, 1)[0]
    assert sum(len(kp) for kp, _ in ref[0]) >= 2
    results, errors = {}, []
    start = threading.Barrier(2)

    def worker(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                c = Context(0, s)
                start.wait()
                results[t] = run(c, 3)
                c.close()
        except Exception as e:   # re-raised on the main thread below
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors
    for t in range(2):
        assert len(results[t]) == 3
        for kps, peaks, heat in results[t]:
            for (kp, ks), (rk, rs) in zip(kps, ref[0]):
                np.testing.assert_array_equal(kp, rk)
                np.testing.assert_array_equal(ks, rs)
            np.testing.assert_array_equal(peaks, ref[1])
            np.testing.assert_array_equal(heat, ref[2])


def test_net_destroyed_before_its_pose_extractor(ctx):
    """Net.close() while a PoseExtractor still refers to the net.  The extractor's
    calls that need the net raise (NetHip::liveness), and destroying the extractor afterwards
    -- whose destructor used to call into the dead net (forget_reader_events) -- is safe."""
    from openpose_amd._lib import OpkError
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(synth.he_weights(net.convs(), seed=3, out_scale=0.02))
    pose = PoseExtractor(ctx, net)
    x = torch.rand((1, 3, 64, 96), device="cuda") - 0.5
    pose.forward(x, (96, 64))
    pose.submit(x, (96, 64))   # leaves a post-processing reading the net's output buffer
    pose.collect()
    net.close()
    with pytest.raises(OpkError, match="destroyed before"):
        pose.forward(x, (96, 64))
    pose.close()
    ctx.sync()
