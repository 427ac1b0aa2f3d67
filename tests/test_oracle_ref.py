"""CPU: pin the connector restatement to the reference's own code (oracle/_ref, compiled from
/root/reference/src/openpose/net/bodyPartConnectorBase.cpp and friends by oracle/Makefile).
Skipped where the reference tree is absent (the GPU box): test_golden.py covers it there."""
import numpy as np
import pytest

import oracle
from openpose_amd import api
from openpose_amd import pose_tables as pt
from tests.fields import noise_field, people_field

pytestmark = pytest.mark.skipif(oracle.ref_lib() is None, reason="no /root/reference here")

CASES = [(n, s) for n in (0, 1, 2, 5, 9, 20) for s in (1, 2, 3)]


@pytest.mark.parametrize("n,seed", CASES)
def test_connector_people(n, seed):
    f = people_field(n, 184, 328, seed=1000 + seed * 31 + n)
    pk = oracle.nms(f, 0.05, 128, (0.25, 0.25))
    for maxpos in (False, True):
        ref = oracle.connect(f, pk, use_reference=True, scale=1.959128, maximize_positives=maxpos)
        got = oracle.connect(f, pk, scale=1.959128, maximize_positives=maxpos)
        np.testing.assert_array_equal(got[0], ref[0])
        np.testing.assert_array_equal(got[1], ref[1])


@pytest.mark.parametrize("seed", range(6))
def test_connector_noise_fields(seed):
    """dense candidate sets, ties, short limbs (the near-distance fallback score)"""
    f = noise_field(78, 48, 64, seed=seed, levels=4 + seed, density=0.5 + 0.08 * seed)
    f[26:] = f[26:] * 2 - 1
    pk = oracle.nms(f, 0.05, 128, (0.25, 0.25))
    ref = oracle.connect(f, pk, use_reference=True)
    got = oracle.connect(f, pk)
    np.testing.assert_array_equal(got[0], ref[0])
    np.testing.assert_array_equal(got[1], ref[1])
    # and the product's host assembly fed the same scores
    scores = oracle.pair_scores(f, pk, pt.BODY25_PAIRS, pt.BODY25_MAP_IDX)
    kp, ks = api.assemble_people(scores, pk)
    np.testing.assert_array_equal(kp, ref[0])
    np.testing.assert_array_equal(ks, ref[1])


def test_connector_thresholds_sweep():
    f = people_field(6, 184, 328, seed=77)
    pk = oracle.nms(f, 0.05, 128, (0.25, 0.25))
    for inter_min, inter_th, cnt, score in [(0.95, 0.05, 3, 0.4), (0.5, 0.2, 2, 0.1),
                                            (0.99, 0.5, 8, 0.6), (0.1, 0.01, 1, 0.0)]:
        kw = dict(inter_min_above=inter_min, inter_th=inter_th, min_subset_cnt=cnt,
                  min_subset_score=score)
        ref = oracle.connect(f, pk, use_reference=True, **kw)
        got = oracle.connect(f, pk, **kw)
        np.testing.assert_array_equal(got[0], ref[0])
        np.testing.assert_array_equal(got[1], ref[1])
