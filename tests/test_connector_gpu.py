"""CPU: the connectBodyPartsGpu people assembly (any pose model, BODY_135 included) and the pose
tables of every model.

gpuconn_*.npz hold the REFERENCE's own outputs (pafVectorIntoPeopleVector,
removePeopleBelowThresholdsAndFillFaces compiled from /root/reference into oracle/_ref;
tests/golden/make_golden.py); pose_tables.json is the reference's poseParameters.cpp run here
(tools/gen_pose_tables.py).  The BODY_135 face-fragment merge runs the reference's code too, with
its one helper from the OpenCV-dependent keypoint.cpp -- getKeypointsRoi(Rectangle, Rectangle),
plain arithmetic -- restated in oracle/ref_driver.cpp (round 5); the gpuconn_b135_*_face fixtures
reach that branch (make_golden.py checks it).
"""
import glob
import os

import numpy as np
import pytest

import oracle
from openpose_amd import api
from openpose_amd.pose_tables import BODY_135, CONNECT_CPU, CONNECT_GPU
from tests.golden.make_golden import dense_scores, gpu_connector_inputs

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = sorted(glob.glob(os.path.join(GOLDEN, "gpuconn_*.npz")))


def _load(path):
    g = np.load(path, allow_pickle=False)
    return g, dense_scores(g["score_idx"], g["score_val"], int(g["npairs"]))


def test_pose_tables_match_reference():
    for t in oracle.pose_tables():
        got = api.pose_model_info(t["id"])
        assert got["parts"] == t["parts"] and got["bkg"] == t["bkg"], t["name"]
        assert got["pairs"] == t["pairs"], t["name"]
        assert got["map_idx"] == t["map_idx"], t["name"]
        assert got["heat_channels"] == t["parts"] + int(t["bkg"]) + len(t["map_idx"])
        assert np.float32(got["nms_threshold"]) == np.float32(t["nms_threshold"])
        assert np.float32(got["inter_threshold"]) == np.float32(t["inter_threshold"])
    assert api.pose_model_info(BODY_135)["heat_channels"] == 439


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p)[8:-4] for p in CASES])
def test_gpu_assembly_oracle_matches_reference_fixture(path):
    g, ps = _load(path)
    t = oracle.pose_tables()[int(g["model"])]
    kp, ks = oracle.connect_gpu_semantics(ps, g["peaks"], t, scale=float(g["scale"]),
                                          maximize_positives=bool(g["maximize_positives"]))
    np.testing.assert_array_equal(kp, g["keypoints"])
    np.testing.assert_array_equal(ks, g["scores"])


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p)[8:-4] for p in CASES])
def test_gpu_assembly_product_matches_reference_fixture(path):
    g, ps = _load(path)
    kp, ks = api.assemble_people(ps, g["peaks"], pose_model=int(g["model"]),
                                 scale=float(g["scale"]),
                                 maximize_positives=bool(g["maximize_positives"]),
                                 semantics=CONNECT_GPU)
    np.testing.assert_array_equal(kp, g["keypoints"])
    np.testing.assert_array_equal(ks, g["scores"])


@pytest.mark.parametrize("kind,n,seed", [("people", 3, 131), ("people", 8, 132), ("random", 0, 133)])
def test_body135_face_merge_product_matches_oracle(kind, n, seed):
    """Inputs with face-only fragments (the getKeypointsRoi branch): product vs oracle, and vs the
    reference compiled here when it is (build container)."""
    t = oracle.pose_tables()[BODY_135]
    pk, ps = gpu_connector_inputs(t, kind, n, seed, 184, 328)
    for maxpos in (False, True):
        ref = oracle.connect_gpu_semantics(ps, pk, t, scale=1.959128, maximize_positives=maxpos)
        got = api.assemble_people(ps, pk, pose_model=BODY_135, scale=1.959128,
                                  maximize_positives=maxpos, semantics=CONNECT_GPU)
        np.testing.assert_array_equal(got[0], ref[0])
        np.testing.assert_array_equal(got[1], ref[1])
        if oracle.ref_lib() is not None:
            assert oracle.face_merge_reached(ps, pk, t, maximize_positives=maxpos)
            live = oracle.connect_gpu_semantics(ps, pk, t, use_reference=True, scale=1.959128,
                                                maximize_positives=maxpos)
            np.testing.assert_array_equal(got[0], live[0])
            np.testing.assert_array_equal(got[1], live[1])


@pytest.mark.skipif(oracle.ref_lib() is None, reason="needs /root/reference (oracle/_ref)")
def test_body135_face_merge_random_vs_reference_live():
    """80 BODY_135 inputs with face peaks (people fields and random scores, both
    maximize_positives settings), nearly all reaching the face-fragment merge: product and oracle
    equal the reference bit for bit."""
    t = oracle.pose_tables()[BODY_135]
    reached = 0
    for kind, n in (("people", 3), ("people", 8), ("random", 0), ("random", 0)):
        for seed in range(10):
            pk, ps = gpu_connector_inputs(t, kind, n, 6000 + 37 * seed + n, 184, 328)
            for maxpos in (False, True):
                reached += oracle.face_merge_reached(ps, pk, t, maximize_positives=maxpos)
                live = oracle.connect_gpu_semantics(ps, pk, t, use_reference=True, scale=1.5,
                                                    maximize_positives=maxpos)
                got = api.assemble_people(ps, pk, pose_model=BODY_135, scale=1.5,
                                          maximize_positives=maxpos, semantics=CONNECT_GPU)
                orc = oracle.connect_gpu_semantics(ps, pk, t, scale=1.5, maximize_positives=maxpos)
                for a in (got, orc):
                    np.testing.assert_array_equal(a[0], live[0])
                    np.testing.assert_array_equal(a[1], live[1])
    assert reached >= 60


@pytest.mark.skipif(oracle.ref_lib() is None, reason="needs /root/reference (oracle/_ref)")
@pytest.mark.parametrize("model", [0, 1, 2, 4, 7, 10, 11, 12, 13, 14])
def test_gpu_assembly_random_vs_reference_live(model):
    """Random peaks/scores for many models against the reference compiled here (build container
    only; the GPU box has no /root/reference)."""
    t = oracle.pose_tables()[model]
    checked = 0
    for seed in range(20):
        pk, ps = gpu_connector_inputs(t, "random", 0, 1000 + seed, 184, 328)
        ref = oracle.connect_gpu_semantics(ps, pk, t, use_reference=True, scale=1.5)
        got = api.assemble_people(ps, pk, pose_model=model, scale=1.5, semantics=CONNECT_GPU)
        orc = oracle.connect_gpu_semantics(ps, pk, t, scale=1.5)
        for a in (got, orc):
            np.testing.assert_array_equal(a[0], ref[0])
            np.testing.assert_array_equal(a[1], ref[1])
        checked += 1
    assert checked >= 10


@pytest.mark.parametrize("model", [0, 14])
def test_gpu_assembly_ties_product_matches_oracle(model):
    """Scores and peak values quantised to a few levels: most connections tie on (total, paf), so
    the order comes from the (pair, i, j) tail of the reference's std::greater tuple -- the
    product's radix sort over packed keys must reproduce it (and the reference, when built)."""
    t = oracle.pose_tables()[model]
    for seed in range(6):
        pk, ps = gpu_connector_inputs(t, "random_noface" if t["parts"] >= 135 else "random", 0,
                                      2000 + seed, 184, 328)
        ps = np.where(ps > 0, np.ceil(ps * 4) / 4, 0).astype(np.float32)
        pk = pk.copy()
        pk[:, 1:, 2] = np.where(pk[:, 1:, 2] > 0, np.ceil(pk[:, 1:, 2] * 2) / 2, 0)
        ref = oracle.connect_gpu_semantics(ps, pk, t, scale=1.5)
        got = api.assemble_people(ps, pk, pose_model=model, scale=1.5, semantics=CONNECT_GPU)
        np.testing.assert_array_equal(got[0], ref[0])
        np.testing.assert_array_equal(got[1], ref[1])
        if oracle.ref_lib() is not None:
            live = oracle.connect_gpu_semantics(ps, pk, t, use_reference=True, scale=1.5)
            if live is not None:
                np.testing.assert_array_equal(got[0], live[0])
                np.testing.assert_array_equal(got[1], live[1])


def test_cpu_semantics_rejects_models_the_reference_cpu_path_rejects():
    """connectBodyPartsCpu accepts BODY_25 / COCO_18 / MPI_15 only (bodyPartConnectorBase.cpp:165-167)."""
    t = oracle.pose_tables()[BODY_135]
    pk, ps = gpu_connector_inputs(t, "random_noface", 0, 5, 100, 100)
    with pytest.raises(api.OpkError if hasattr(api, "OpkError") else RuntimeError):
        api.assemble_people(ps, pk, pose_model=BODY_135, semantics=CONNECT_CPU)
