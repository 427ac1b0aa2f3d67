"""CPU: the oracle (and the product's host assembly) against the committed golden fixtures.

connector_* fixtures hold the REFERENCE connector's outputs (bodyPartConnectorBase.cpp compiled from
/root/reference, tests/golden/make_golden.py); the others pin the oracle's restatements so the GPU
box, which has no reference tree, checks against the same numbers.
"""
import glob
import hashlib
import os

import numpy as np
import pytest

import oracle
from oracle import body25
from openpose_amd import api, synth
from tests.golden.make_golden import connector_field

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CONNECTOR = sorted(glob.glob(os.path.join(GOLDEN, "connector_*.npz")))


def _load(path):
    return np.load(path, allow_pickle=False)


@pytest.mark.parametrize("path", CONNECTOR, ids=[os.path.basename(p) for p in CONNECTOR])
def test_connector_oracle_matches_reference_fixture(path):
    g = _load(path)
    f = connector_field(str(g["kind"]), int(g["n_people"]), int(g["seed"]), int(g["h"]), int(g["w"]))
    assert hashlib.sha256(f.tobytes()).hexdigest() == str(g["field_sha"]), "input regeneration drifted"
    scale = float(g["scale"])
    off = np.float32(0.5 / scale)
    pk = oracle.nms(f, 0.05, 128, (off, off))
    np.testing.assert_array_equal(pk, g["peaks"])
    kp, ks = oracle.connect(f, pk, scale=scale, maximize_positives=bool(g["maximize_positives"]))
    np.testing.assert_array_equal(kp, g["keypoints"])
    np.testing.assert_array_equal(ks, g["scores"])


@pytest.mark.parametrize("path", CONNECTOR, ids=[os.path.basename(p) for p in CONNECTOR])
def test_product_host_assembly_matches_reference_fixture(path):
    """libopk_hip.so's host assembly (opk_assemble_people) fed the getScoreAB table."""
    g = _load(path)
    f = connector_field(str(g["kind"]), int(g["n_people"]), int(g["seed"]), int(g["h"]), int(g["w"]))
    pk = g["peaks"]
    from openpose_amd import pose_tables as pt
    scores = oracle.pair_scores(f, pk, pt.BODY25_PAIRS, pt.BODY25_MAP_IDX)
    kp, ks = api.assemble_people(scores, pk, scale=float(g["scale"]),
                                 maximize_positives=bool(g["maximize_positives"]))
    np.testing.assert_array_equal(kp, g["keypoints"])
    np.testing.assert_array_equal(ks, g["scores"])


@pytest.mark.parametrize("name", ["people", "noise", "plateau"])
def test_nms_fixture(name):
    g = _load(os.path.join(GOLDEN, "nms_%s.npz" % name))
    np.testing.assert_array_equal(oracle.nms(g["field"], 0.05, 128, (0.25, 0.5)), g["peaks"])


def test_resize_fixture():
    g = _load(os.path.join(GOLDEN, "resize.npz"))
    np.testing.assert_array_equal(oracle.resize_merge([g["src"]], 80, 160), g["out"])
    ms = oracle.resize_merge([g["ms_src0"], g["ms_src1"], g["ms_src2"]], 80, 160)
    np.testing.assert_array_equal(ms, g["ms_out"])
    np.testing.assert_array_equal(oracle.resize_merge([g["ragged_src"]], 72, 166), g["ragged_out"])
    with oracle.resize_order("3.x"):
        np.testing.assert_array_equal(oracle.resize_merge([g["src"]], 80, 160), g["out_opencv3"])


def test_resize_orders_differ_only_in_the_vertical_sum():
    """OpenCV 4.x (SIMD body h0b0 + (h1b1 + (h2b2 + h3b3))) and 3.x (left to right) agree to a few
    ulp, differ somewhere in the last bits, and agree exactly on the 4.x scalar tail columns."""
    g = _load(os.path.join(GOLDEN, "resize.npz"))
    a, b = g["out"], g["out_opencv3"]
    assert not np.array_equal(a, b)
    np.testing.assert_allclose(a, b, rtol=0, atol=4 * np.finfo(np.float32).eps * np.abs(a).max())
    src = g["ragged_src"]
    four = g["ragged_out"]
    with oracle.resize_order("3.x"):
        three = oracle.resize_merge([src], 72, 166)
    np.testing.assert_array_equal(four[..., 164:], three[..., 164:])   # 166 % 4 == 2 tail columns


def test_cnn_fixture():
    g = _load(os.path.join(GOLDEN, "cnn_body25_64x96.npz"))
    graph = body25.layers()
    params = synth.he_weights(graph, seed=int(g["weight_seed"]))
    out = body25.forward(g["input"], params, graph=graph)
    # fp32 summation order depends on the thread count only through tiling: allow rounding noise
    np.testing.assert_allclose(out, g["net_output"], rtol=1e-4, atol=1e-5)
