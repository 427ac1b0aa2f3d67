"""Output contract: getHeatMapsCopy scale modes, getCandidatesCopy,
KeypointScaler, KeepTopNPeople -- product (libopk_hip) against the oracle restatements
(oracle/output.py).  CPU tests call the host C-ABI functions; GPU tests the pose pipeline."""
import numpy as np
import pytest

from oracle import output as O
from openpose_amd import api


@pytest.mark.parametrize("mode", range(7))
def test_scale_keypoints_matches_oracle(mode):
    rng = np.random.default_rng(mode)
    kp = rng.uniform(0, 1280, (7, 25, 3)).astype(np.float32)
    kp[..., 2] = rng.uniform(0, 1, (7, 25))
    args = dict(scale_input_to_output=0.75, scale_net_to_output=1.959128, producer_size=(1280, 720))
    got = api.scale_keypoints(kp, mode, **args)
    np.testing.assert_array_equal(got, O.scale_keypoints(kp, mode, **args))
    np.testing.assert_array_equal(got[..., 2], kp[..., 2])   # scores untouched
    if mode == O.INPUT_RESOLUTION:
        np.testing.assert_array_equal(got, kp)


def test_scale_keypoints_rejects_unknown_mode():
    with pytest.raises(api._lib.OpkError):
        api.scale_keypoints(np.zeros((1, 25, 3)), 7)   # UnsignedChar: not a keypoint scale


@pytest.mark.parametrize("seed", range(6))
def test_keep_top_n_people_matches_oracle(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 30))
    kp = rng.uniform(0, 500, (n, 25, 3)).astype(np.float32)
    kp[..., 2] = rng.uniform(0, 1, (n, 25)) * (rng.uniform(0, 1, (n, 25)) > 0.3)
    scores = rng.uniform(0, 1, n).astype(np.float32)
    if seed % 2:   # ties at the threshold: identical people
        kp[n // 2:] = kp[0]
        scores[n // 2:] = scores[0]
    for m in (0, 1, n // 2, n - 1, n, n + 3):
        got, gi = api.keep_top_n_people(kp, scores, m)
        ref, ri = O.keep_top_n_people(kp, scores, m)
        np.testing.assert_array_equal(got, ref)
        np.testing.assert_array_equal(gi, ri)


def test_keep_top_n_people_edge_cases():
    got, idx = api.keep_top_n_people(np.zeros((0, 25, 3), np.float32), np.zeros(0, np.float32), 2)
    assert got.shape[0] == 0 and idx.shape[0] == 0
    # people with no keypoint above 0.05 have area 0: ranked last
    kp = np.zeros((3, 25, 3), np.float32)
    kp[1, :2] = [[10, 10, 0.9], [50, 80, 0.9]]
    got, idx = api.keep_top_n_people(kp, np.array([0.9, 0.1, 0.8], np.float32), 1)
    assert list(idx) == [1]


@pytest.mark.gpu
@pytest.mark.parametrize("types,mode", [(7, 8), (7, 5), (7, 3), (7, 7), (1, 7), (4, 3), (2, 5),
                                        (5, 0), (6, 7)])
def test_gpu_heatmaps_copy_and_candidates(ctx, types, mode):
    import torch
    import oracle
    from openpose_amd import synth
    from openpose_amd.api import PoseExtractor
    h, w = 23, 41
    rng = np.random.default_rng(types * 10 + mode)
    field = (rng.standard_normal((2, 78, h, w)) * 0.3).astype(np.float32)
    for f in range(2):
        field[f] += synth.overlay(3, h, w, seed=f)
    pose = PoseExtractor(ctx, None)
    pose.forward_net_output(torch.from_numpy(field).cuda(), (w * 8, h * 8), (w * 8, h * 8))
    got = pose.heatmaps_copy(types, mode)
    for f in range(2):
        heat = oracle.resize_merge([field[f]], h * 8, w * 8)
        ref = O.heatmaps_copy(heat, 25, True, 52, types, mode)
        np.testing.assert_array_equal(got[f], ref)
    s = pose.scale_net_to_output()
    peaks = pose.peaks_numpy()
    for f in range(2):
        for a, b in zip(pose.candidates(f), O.candidates(peaks[f], s)):
            np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_gpu_heatmaps_copy_rejects_bkg_without_background(ctx):
    import torch
    from openpose_amd.api import PoseExtractor
    from openpose_amd.pose_tables import BODY_135, CONNECT_GPU
    pose = PoseExtractor(ctx, None, pose_model=BODY_135, semantics=CONNECT_GPU)
    field = torch.zeros((1, 439, 10, 12), device="cuda")
    pose.forward_net_output(field, (96, 80), (96, 80))
    with pytest.raises(api._lib.OpkError, match="heatmaps_add_bkg"):
        pose.heatmaps_copy(2, 8)


# ---- people JSON (--write_json): savePeopleJson, fileStream.cpp:306-344 ----------------------
def test_people_json_known_answer():
    """Hand-derived from the reference source: JsonOfstream writes `"key":` then the values through
    std::ostream (%g); humanReadable = false in WPeopleJsonSaver (wPeopleJsonSaver.hpp:68)."""
    kp = np.array([[[1.5, 2.0, 0.25], [0.0, 0.0, 0.0]]], np.float32)
    text = api.people_json(api.datum_keypoint_vector(kp))
    assert text == ('{"version":1.3,"people":[{"person_id":[-1],"pose_keypoints_2d":[1.5,2,0.25,0,0,0],'
                    '"face_keypoints_2d":[],"hand_left_keypoints_2d":[],"hand_right_keypoints_2d":[],'
                    '"pose_keypoints_3d":[],"face_keypoints_3d":[],"hand_left_keypoints_3d":[],'
                    '"hand_right_keypoints_3d":[]}]}')
    assert api.people_json([(None, "pose_keypoints_2d")]) == \
        '{"version":1.3,"people":[]}'
    cand = [[[10.0, 20.0, 0.5]], [], [[1e-7, 123456789.0, 1.0], [0.1, 0.2, 0.3]]]
    assert api.people_json([(None, "pose_keypoints_2d")], cand) == \
        ('{"version":1.3,"people":[],"part_candidates":[{"0":[10,20,0.5],"1":[],'
         '"2":[1e-07,1.23457e+08,1,0.1,0.2,0.3]}]}')


@pytest.mark.parametrize("human", [False, True])
@pytest.mark.parametrize("seed", range(4))
def test_people_json_matches_oracle(seed, human, tmp_path):
    rng = np.random.default_rng(seed)
    people = [0, 1, 3, 7][seed]
    kp = rng.uniform(0, 1280, (people, 25, 3)).astype(np.float32)
    kp[..., 2] = rng.uniform(0, 1, (people, 25))
    kp[:, ::4] = 0                                        # parts not found
    face = rng.uniform(-1, 1, (people, 70, 3)).astype(np.float32) if seed % 2 else None
    hands = (rng.normal(0, 1e3, (people, 21, 3)).astype(np.float32), None)
    vec = api.datum_keypoint_vector(kp, face, hands)
    cand = ([[list(rng.uniform(0, 500, 3)) for _ in range(rng.integers(0, 4))] for _ in range(25)]
            if seed >= 2 else None)
    text = api.people_json(vec, cand, human_readable=human)
    assert text == O.people_json(vec, cand, human_readable=human)
    path = str(tmp_path / ("%d_keypoints.json" % seed))
    api.save_people_json(path, vec, cand, human_readable=human)
    with open(path) as f:
        saved = f.read()
    assert saved == text
    if not human:
        import json
        d = json.loads(text)
        assert d["version"] == 1.3 and len(d["people"]) == people
        for p in range(people):
            np.testing.assert_allclose(d["people"][p]["pose_keypoints_2d"], kp[p].reshape(-1),
                                       rtol=1e-5)


def test_people_json_rejects_bad_arrays():
    with pytest.raises(api._lib.OpkError):    # getNumberDimensions() != 1 && != 3
        api.people_json([(np.zeros((2, 3), np.float32), "pose_keypoints_2d")])
    with pytest.raises(api._lib.OpkError):    # fewer people than the widest array
        api.people_json([(np.zeros((3, 25, 3), np.float32), "a"),
                         (np.zeros((2, 25, 3), np.float32), "b")])
    with pytest.raises(api._lib.OpkError):
        api.save_people_json("/nonexistent_dir/x.json", [(None, "pose_keypoints_2d")])
