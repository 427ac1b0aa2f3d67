"""CPU: known-answer tests for the NMS restatement (nmsBase.cpp:7-170 semantics).

Parity unpinned against the reference binary (nmsBase.cpp needs OpenCV headers, absent here); every
expected value below follows from the reference source text, with the line it exercises.
"""
import numpy as np

import oracle


def peaks_of(field, th=0.05, cap=128, off=(0.0, 0.0)):
    return oracle.nms(field[None].astype(np.float32), th, cap, off, channels=1)[0]


def test_single_interior_peak_and_centroid():
    f = np.zeros((20, 30), np.float32)
    f[10, 12] = 1.0
    f[10, 13] = 0.5
    f[9, 12] = 0.25
    p = peaks_of(f, off=(0.5, 0.25))
    assert p[0, 0] == 1
    # centroid over the 7x7 window of positive scores (nmsBase.cpp:79-106), + offset
    xs = (12 * 1.0 + 13 * 0.5 + 12 * 0.25) / 1.75
    ys = (10 * 1.0 + 10 * 0.5 + 9 * 0.25) / 1.75
    np.testing.assert_allclose(p[1], [xs + 0.5, ys + 0.25, 1.0], rtol=1e-6)


def test_interior_plateau_is_not_a_peak():
    f = np.zeros((20, 30), np.float32)
    f[10, 12] = f[10, 13] = 0.8          # strict '>' on the interior (nmsBase.cpp:31-33)
    assert peaks_of(f)[0, 0] == 0


def test_inner_ring_uses_ge():
    f = np.zeros((20, 30), np.float32)
    f[1, 5] = f[1, 6] = 0.8              # row 1: '>=' (nmsBase.cpp:41-61) -> both register
    p = peaks_of(f)
    assert p[0, 0] == 2
    np.testing.assert_array_equal(p[1:3, 2], np.float32([0.8, 0.8]))


def test_outer_border_rules():
    f = np.zeros((20, 30), np.float32)
    f[5, 0] = 0.9        # x == 0, 2 <= y <= h-3: class 3, never (nmsBase.cpp:66-67)
    f[1, 0] = 0.7        # x == 0 but y == 1: class 2, outside neighbours read as th
    f[0, 15] = 0.6       # y == 0 on a column that is not 1 / w-2: class 3
    f[0, 28] = 0.5       # y == 0, x == w-2: class 2
    p = peaks_of(f)
    assert p[0, 0] == 2
    assert {tuple(np.round(p[i, :2] - 0, 3)) for i in (1, 2)} >= set()
    scores = sorted(p[1:3, 2].tolist())
    np.testing.assert_array_equal(scores, np.float32([0.5, 0.7]))


def test_threshold_is_strict():
    f = np.zeros((20, 30), np.float32)
    f[10, 10] = np.float32(0.05)         # value > threshold required (nmsBase.cpp:20,45)
    f[10, 20] = np.float32(0.0500001)
    p = peaks_of(f, th=0.05)
    assert p[0, 0] == 1 and p[1, 2] == np.float32(0.0500001)


def test_cap_and_raster_order():
    f = np.zeros((40, 40), np.float32)
    ys, xs = np.mgrid[2:38:2, 2:38:2]
    f[ys, xs] = 0.5 + (ys * 40 + xs) / 10000.0     # 324 isolated peaks
    p = peaks_of(f, cap=128)
    assert p[0, 0] == 127                           # targetPeaks-1 kept (nmsBase.cpp:151)
    order = p[1:128, 1] * 1000 + p[1:128, 0]        # raster order: y then x
    assert np.all(np.diff(order) > 0)


def test_refine_ignores_nonpositive_and_clips():
    f = np.full((10, 10), -1.0, np.float32)
    f[1, 1] = 1.0                                   # corner-near peak: window clipped at 0
    p = peaks_of(f)
    assert p[0, 0] == 1
    np.testing.assert_array_equal(p[1], np.float32([1.0, 1.0, 1.0]))
