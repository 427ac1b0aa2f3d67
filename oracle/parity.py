"""Keypoint parity of the GPU pipeline against the fp32 CPU path -- TEST INFRASTRUCTURE ONLY.

Used by tests/ and by bench.py's cpu_baseline leg (the CPU reference run) as the checker: the
product never imports it.  It compares what the reference's CPU path produces from a frame with
what the GPU pipeline produced from the same frame, at the stages the north star names:

* the net output (relative L2 of the whole [C, h, w] stack);
* the NMS peak set: the integer pixel of every peak nmsCpu's test accepts (nmsRegisterKernelCPU,
  src/openpose/net/nmsBase.cpp:7-68, restated in numpy below), on the x8 resize of each side's
  own net output -- the fraction of the fp32 path's peaks found at the identical index, and
  within 1 heat-map pixel;
* the refined peaks (nmsAccuratePeakPosition, nmsBase.cpp:70-107) of matched peaks: the largest
  displacement;
* people: counts and, for people matched part by part, the largest keypoint displacement.
"""
import numpy as np


def peak_mask(heat, threshold, parts=None):
    """Boolean [parts, H, W]: nmsCpu's peak test (nmsBase.cpp:17-67) per pixel.  Inner pixels
    (1 < x < w-2, 1 < y < h-2): value > threshold and strictly greater than all 8 neighbours; the
    first inner border (x or y equal to 1 or its mirror, any pixel of those rows/columns): value >
    threshold and >= every neighbour, neighbours outside the map counting as the threshold; the
    outer border otherwise: never."""
    heat = np.asarray(heat, np.float32)
    if parts is not None:
        heat = heat[:parts]
    c, h, w = heat.shape
    t = np.float32(threshold)
    p = np.full((c, h + 2, w + 2), t, np.float32)
    p[:, 1:-1, 1:-1] = heat
    v = heat
    nb = [p[:, 1 + dy:1 + dy + h, 1 + dx:1 + dx + w]
          for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dy or dx]
    gt = np.ones_like(v, bool)
    ge = np.ones_like(v, bool)
    for n in nb:
        gt &= v > n
        ge &= v >= n
    y = np.arange(h)[:, None]
    x = np.arange(w)[None, :]
    inner = (1 < x) & (x < w - 2) & (1 < y) & (y < h - 2)
    edge = ~inner & ((x == 1) | (x == w - 2) | (y == 1) | (y == h - 2))
    above = v > t
    # (an inner pixel reads real neighbours only, so the padding never reaches its test)
    return above & ((inner & gt) | (edge & ge))


def peak_sets(mask):
    """[(y, x) array per part] of a peak mask."""
    return [np.argwhere(m) for m in mask]


def compare_peaks(ref_mask, got_mask, radius=1.0):
    """(reference peaks, identical-index fraction, within-`radius` fraction) of two peak masks of
    the same part stack (Euclidean distance in heat-map pixels, same part)."""
    total = same = near = 0
    for r, g in zip(peak_sets(ref_mask), peak_sets(got_mask)):
        total += len(r)
        if len(r) == 0 or len(g) == 0:
            continue
        d = np.sqrt(((r[:, None, :] - g[None, :, :]).astype(np.float64) ** 2).sum(-1)).min(1)
        same += int((d == 0).sum())
        near += int((d <= radius).sum())
    return total, (same / total if total else 1.0), (near / total if total else 1.0)


def refined_shift(ref_peaks, got_peaks, radius=1.0):
    """Largest displacement between a reference refined peak and the nearest refined peak of the
    same part within `radius` ([parts, 128, 3] blobs: row 0 holds the count)."""
    worst = 0.0
    for c in range(ref_peaks.shape[0]):
        r = ref_peaks[c, 1:int(ref_peaks[c, 0, 0]) + 1, :2]
        g = got_peaks[c, 1:int(got_peaks[c, 0, 0]) + 1, :2]
        if len(r) == 0 or len(g) == 0:
            continue
        d = np.sqrt(((r[:, None, :] - g[None, :, :]) ** 2).sum(-1)).min(1)
        if (d <= radius).any():
            worst = max(worst, float(d[d <= radius].max()))
    return worst


def keypoint_shift(ref_kp, got_kp, radius=2.0):
    """Largest keypoint displacement over people matched greedily (smallest mean distance first)
    among pairs that detect the same parts with a mean distance <= radius, and the number matched.
    kp: [people, parts, 3] (x, y, score; score 0 = part absent), distances in kp units."""
    ref_kp = np.asarray(ref_kp, np.float64)
    got_kp = np.asarray(got_kp, np.float64)
    if len(ref_kp) == 0 or len(got_kp) == 0:
        return 0.0, 0
    pr = ref_kp[:, :, 2] > 0
    pg = got_kp[:, :, 2] > 0
    same_parts = (pr[:, None, :] == pg[None, :, :]).all(-1)
    d = np.sqrt(((ref_kp[:, None, :, :2] - got_kp[None, :, :, :2]) ** 2).sum(-1))   # [R, G, parts]
    cnt = np.maximum(pr.sum(-1), 1)[:, None]
    cost = np.where(same_parts, (d * pr[:, None, :]).sum(-1) / cnt, np.inf)
    worst, matched = 0.0, 0
    used_r, used_g = set(), set()
    for flat in np.argsort(cost, axis=None):
        i, j = divmod(int(flat), cost.shape[1])
        if not cost[i, j] <= radius:
            break
        if i in used_r or j in used_g:
            continue
        used_r.add(i)
        used_g.add(j)
        worst = max(worst, float(np.abs(ref_kp[i, pr[i], :2] - got_kp[j, pr[i], :2]).max()))
        matched += 1
    return worst, matched


def people_identical(ref_kp, got_kp, tol):
    """Number of reference people that some GPU person reproduces exactly: the same parts, every
    keypoint within tol (kp units), one GPU person per reference person."""
    ref_kp = np.asarray(ref_kp, np.float64)
    got_kp = np.asarray(got_kp, np.float64)
    if len(ref_kp) == 0 or len(got_kp) == 0:
        return 0
    pr = ref_kp[:, :, 2] > 0
    pg = got_kp[:, :, 2] > 0
    ok = (pr[:, None, :] == pg[None, :, :]).all(-1)
    diff = np.abs(ref_kp[:, None, :, :2] - got_kp[None, :, :, :2]).max(-1)   # [R, G, parts]
    ok &= np.where(pr[:, None, :], diff <= tol, True).all(-1)
    used, n = set(), 0
    for i in range(len(ref_kp)):
        for j in np.nonzero(ok[i])[0]:
            if int(j) not in used:
                used.add(int(j))
                n += 1
                break
    return n
