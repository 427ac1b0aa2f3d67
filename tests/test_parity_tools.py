"""CPU: the parity checker (oracle/parity.py) against the oracle's nmsCpu restatement -- the numpy
peak test must accept exactly the pixels orc_nms counts, border rules included."""
import os

import numpy as np

import oracle
from oracle import parity


def test_peak_mask_matches_oracle_nms():
    rng = np.random.default_rng(0)
    for trial in range(6):
        h, w = (23, 31) if trial % 2 else (40, 17)
        heat = rng.uniform(0, 1, (25, h, w)).astype(np.float32)
        if trial >= 2:   # plateaus: ties decide the strict / non-strict rules
            heat = np.round(heat * 4) / 4
        if trial >= 4:   # sparse maps: peaks on and next to the border
            heat *= rng.uniform(0, 1, heat.shape) > 0.7
        th = 0.05
        mask = parity.peak_mask(heat, th)
        peaks = oracle.nms(heat, th, 128, (0.0, 0.0))
        for c in range(25):
            n = int(peaks[c, 0, 0])
            m = int(mask[c].sum())
            assert n == min(m, 127), (trial, c, n, m)
            if m <= 127:   # the integer pixel of each refined peak is a mask pixel
                ys, xs = np.nonzero(mask[c])
                # raster order, as nmsCpu collects them
                assert list(zip(ys, xs)) == sorted(zip(ys, xs))


def test_compare_peaks_and_keypoint_shift():
    a = np.zeros((2, 10, 10), bool)
    b = np.zeros((2, 10, 10), bool)
    a[0, 3, 3] = a[0, 6, 6] = a[1, 2, 7] = True
    b[0, 3, 3] = b[0, 6, 7] = b[1, 5, 5] = True
    total, same, near = parity.compare_peaks(a, b)
    assert total == 3 and same == 1 / 3 and near == 2 / 3
    r = np.array([[[1, 1, 1], [2, 2, 1]], [[10, 10, 1], [0, 0, 0]]], np.float32)
    g = np.array([[[10.5, 10, 1], [0, 0, 0]], [[1, 1.25, 1], [2, 2, 1]]], np.float32)
    worst, matched = parity.keypoint_shift(r, g)
    assert matched == 2 and abs(worst - 0.5) < 1e-6
    assert parity.keypoint_shift(r, g, radius=0.3) == (0.25, 1)
    assert parity.people_identical(r, g, 0.3) == 1 and parity.people_identical(r, g, 0.6) == 2
    g[0, 1] = [3, 3, 1]   # another part set: never matched
    assert parity.keypoint_shift(r, g) == (0.25, 1)


def test_pmc_provenance_kernel_groups(tmp_path):
    """bench.pmc_provenance: a summary stamped with per-group digests matches the running tree for
    the group whose sources are unchanged and not for a group whose digest differs; without group
    digests it falls back to the whole-tree digest (tools/pmc_stamp.py, tools/pmc_round.sh)."""
    import json
    import bench
    assert set(bench.KERNEL_GROUPS) == {"cnn", "post"}
    kdir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "openpose_amd", "csrc", "kernels")
    for names in bench.KERNEL_GROUPS.values():
        for n in names:
            assert os.path.exists(os.path.join(kdir, n)), n
    full, cnn, post = bench.kernel_src_sha(), bench.kernel_src_sha("cnn"), bench.kernel_src_sha("post")
    assert len({full, cnn, post}) == 3
    p = tmp_path / "report.json"
    p.write_text(json.dumps({"commit": "x", "kernel_src_sha": "0" * 16,
                             "cnn_kernel_src_sha": cnn, "post_kernel_src_sha": "1" * 16}))
    c = bench.pmc_provenance(str(p), "cnn")
    assert c["kernels_match_this_tree"] is True and c["all_kernels_match_this_tree"] is False
    assert bench.pmc_provenance(str(p), "post")["kernels_match_this_tree"] is False
    p.write_text(json.dumps({"commit": "x", "kernel_src_sha": full}))
    assert bench.pmc_provenance(str(p), "cnn")["kernels_match_this_tree"] is True
    # a reader over another tree gives that tree's digest
    assert bench.kernel_src_sha("cnn", read=lambda n: b"") != cnn
