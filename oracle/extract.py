"""CPU oracle for face / hand keypoint extraction (TEST INFRASTRUCTURE ONLY; see oracle/oracle.h).

Restates, in float32 / float64 scalar arithmetic as the C++ does:
  FaceDetector::detectFaces            src/openpose/face/faceDetector.cpp:8-15, 22-139
  HandDetector::detectHands            src/openpose/hand/handDetector.cpp:9-57, 135-160
  FaceExtractorCaffe::forwardPass      src/openpose/face/faceExtractorCaffe.cpp:174-280
  HandExtractorCaffe::forwardPass      src/openpose/hand/handExtractorCaffe.cpp:44-100, 306-445
    crop = warpAffine(INTER_LINEAR | WARP_INVERSE_MAP)  -> oracle.warp_affine_inv (preprocess.c)
    ResizeAndMergeCaffe x8 (CPU path)   -> oracle.resize_merge (resize.c)
    MaximumCaffe (maximumBase.cpp:8-42, cv::minMaxLoc: first maximum in raster order)
    keypoint = M (x, y) in double, stored as float
getDistance / getAverageScore are keypoint.cpp:12-26, 352-372.  faceDetector.cpp / handDetector.cpp
compile without OpenCV but need op::Array (array.cpp includes OpenCV), so the detectors are
restatements: parity unpinned, plain float code restated line by line.
"""
import numpy as np

import oracle

f32 = np.float32
FACE_PARTS, HAND_PARTS = 70, 21
# PoseKey indices of the detector keypoint table (tests/golden/pose_tables.json "detector_keys")
NECK, NOSE, LEAR, REAR, LEYE, REYE, LWRIST, LELBOW, LSHOULDER, RWRIST, RELBOW, RSHOULDER = range(12)


def _dist(p, a, b):   # getDistance (float)
    dx = f32(p[a, 0] - p[b, 0])
    dy = f32(p[a, 1] - p[b, 1])
    return f32(np.sqrt(f32(dx * dx + dy * dy)))


def face_rect(p, keys, threshold=f32(0.25)):
    """getFaceFromPoseKeypoints for one person p [parts, 3] -> (x, y, w, h) float32."""
    neck, nose, lear, rear, leye, reye = (keys[i] for i in (NECK, NOSE, LEAR, REAR, LEYE, REYE))
    above = {k: bool(p[k, 2] > threshold) for k in (neck, nose, lear, rear, leye, reye)}
    tx = ty = size = f32(0)
    counter = 0
    if nose == lear and lear == rear:   # MPI: face and neck given
        if above[neck] and above[nose]:
            tx, ty = f32(p[nose, 0]), f32(p[nose, 1])
            size = f32(f32(1.33) * _dist(p, neck, nose))
    else:
        if above[neck] and above[nose]:
            if (above[leye] == above[lear] and above[reye] == above[rear]
                    and above[leye] != above[reye]):
                eye, ear = (leye, lear) if above[leye] else (reye, rear)
                tx = f32(tx + f32(f32(f32(p[eye, 0] + p[ear, 0]) + p[nose, 0]) / f32(3)))
                ty = f32(ty + f32(f32(f32(p[eye, 1] + p[ear, 1]) + p[nose, 1]) / f32(3)))
                s = f32(f32(_dist(p, nose, eye) + _dist(p, nose, ear)) + _dist(p, neck, nose))
                size = f32(size + f32(f32(0.85) * s))
            else:
                tx = f32(tx + f32(f32(p[neck, 0] + p[nose, 0]) / f32(2)))
                ty = f32(ty + f32(f32(p[neck, 1] + p[nose, 1]) / f32(2)))
                size = f32(size + f32(f32(2) * _dist(p, neck, nose)))
            counter += 1
        if above[leye] and above[reye]:
            tx = f32(tx + f32(f32(p[leye, 0] + p[reye, 0]) / f32(2)))
            ty = f32(ty + f32(f32(p[leye, 1] + p[reye, 1]) / f32(2)))
            size = f32(size + f32(f32(3) * _dist(p, leye, reye)))
            counter += 1
        if above[lear] and above[rear]:
            tx = f32(tx + f32(f32(p[lear, 0] + p[rear, 0]) / f32(2)))
            ty = f32(ty + f32(f32(p[lear, 1] + p[rear, 1]) / f32(2)))
            size = f32(size + f32(f32(2) * _dist(p, lear, rear)))
            counter += 1
        if counter > 0:
            tx = f32(tx / f32(counter))
            ty = f32(ty / f32(counter))
            size = f32(size / f32(counter))
    half = f32(size / f32(2))
    return np.array([f32(tx - half), f32(ty - half), size, size], f32)


def detect_faces(kp, keys):
    kp = np.asarray(kp, f32)
    return np.array([face_rect(kp[i], keys) for i in range(kp.shape[0])], f32).reshape(-1, 4)


def hand_rect(p, wrist, elbow, shoulder, threshold=f32(0.03)):
    x = y = w = f32(0)
    if p[wrist, 2] > threshold and p[elbow, 2] > threshold and p[shoulder, 2] > threshold:
        r = f32(0.33)
        x = f32(p[wrist, 0] + f32(r * f32(p[wrist, 0] - p[elbow, 0])))
        y = f32(p[wrist, 1] + f32(r * f32(p[wrist, 1] - p[elbow, 1])))
        dwe = _dist(p, wrist, elbow)
        des = f32(f32(0.9) * _dist(p, elbow, shoulder))
        w = f32(f32(1.5) * (dwe if dwe > des else des))
    h = w
    x = f32(x - f32(w / f32(2)))
    y = f32(y - f32(h / f32(2)))
    return np.array([x, y, w, h], f32)


def detect_hands(kp, keys):
    """-> [people, 2 (left, right), 4]"""
    kp = np.asarray(kp, f32)
    out = np.zeros((kp.shape[0], 2, 4), f32)
    for i in range(kp.shape[0]):
        out[i, 0] = hand_rect(kp[i], keys[LWRIST], keys[LELBOW], keys[LSHOULDER])
        out[i, 1] = hand_rect(kp[i], keys[RWRIST], keys[RELBOW], keys[RSHOULDER])
    return out


def face_affine(rect, net_side):
    """faceExtractorCaffe.cpp:225-232 -> 2x3 float64, or None below the minimum size."""
    x, y, w, h = (f32(v) for v in rect)
    if not (min(w, h) > 40):
        return None
    s = float(max(w, h)) / float(net_side)
    return np.array([[s, 0, float(x)], [0, s, float(y)]], np.float64)


def hand_affine(rect, net_side, mirror):
    """cropFrame (handExtractorCaffe.cpp:44-62)."""
    x, y, w, h = (f32(v) for v in rect)
    s = float(f32(w / f32(net_side)))
    return np.array([[-s if mirror else s, 0, float(f32(x + w)) if mirror else float(x)],
                     [0, s, float(y)]], np.float64)


def hand_valid(rect):
    w, h = f32(rect[2]), f32(rect[3])
    return min(w, h) > 1 and f32(w * h) > 10


def recenter(rect, nw, nh):   # op::recenter (rectangle.cpp:216-233) in float
    x, y, w, h = (f32(v) for v in rect)
    cx = f32(x + f32(w / f32(2)))
    cy = f32(y + f32(h / f32(2)))
    return np.array([f32(cx - f32(f32(nw) / f32(2))), f32(cy - f32(f32(nh) / f32(2))), nw, nh], f32)


def hand_scale_rects(rect, number, rng):
    """Multi-scale rectangles (handExtractorCaffe.cpp:392-407)."""
    if number == 1:
        return [np.asarray(rect, f32)]
    init = f32(f32(1) - f32(rng) / f32(2))
    out = []
    for i in range(number):
        s = f32(init + f32(f32(f32(rng) * f32(i)) / f32(f32(number) - f32(1))))
        nw = f32(int(f32(f32(rect[2]) * s) + f32(0.5)) // 2 * 2)
        nh = f32(int(f32(f32(rect[3]) * s) + f32(0.5)) // 2 * 2)
        out.append(recenter(rect, nw, nh))
    return out


def maximum(heat, parts):
    """MaximumCaffe: per channel (x, y, max) of the first maximum in raster order."""
    c, h, w = heat.shape
    out = np.zeros((parts, 3), f32)
    for p in range(parts):
        i = int(np.argmax(heat[p].ravel()))
        out[p] = (i % w, i // w, heat[p].ravel()[i])
    return out


def keypoints_from_output(net_out, M, parts):
    """net output [C, h, w] of one crop -> [parts, 3] keypoints in frame coordinates."""
    c, h, w = net_out.shape
    heat = oracle.resize_merge([net_out], h * 8, w * 8)
    return map_peaks(maximum(heat, parts), M)


def map_peaks(peaks, M):
    out = np.zeros_like(peaks, dtype=f32)
    for p in range(peaks.shape[0]):
        x, y = float(peaks[p, 0]), float(peaks[p, 1])
        out[p, 0] = f32(M[0, 0] * x + M[0, 1] * y + M[0, 2])
        out[p, 1] = f32(M[1, 0] * x + M[1, 1] * y + M[1, 2])
        out[p, 2] = peaks[p, 2]
    return out


def average_score(kp):   # getAverageScore (float accumulation)
    s = f32(0)
    for v in np.asarray(kp, f32)[:, 2]:
        s = f32(s + v)
    return f32(s / f32(kp.shape[0]))


def crop_heatmaps(net_out, parts, scale_mode):
    """updateFaceHeatMapsForPerson / updateHandHeatMapsForPerson (faceExtractorCaffe.cpp:42-75,
    handExtractorCaffe.cpp:126-160) on one crop's net output [C, h, w]: the first `parts`
    channels of the x8 resize, fastTruncate to [0, 1], then *2-1 (PlusMinusOne, 5 / 6),
    (float)positiveIntRound(* 255) (UnsignedChar, 7) or as is (any other ScaleMode), in float."""
    c, h, w = net_out.shape
    heat = oracle.resize_merge([net_out], h * 8, w * 8)[:parts]
    m = np.where(f32(0) > heat, f32(0), heat).astype(f32)       # fastMax(0, v)
    t = np.where(f32(1) < m, f32(1), m).astype(f32)             # fastMin(1, .)
    if scale_mode in (5, 6):
        return (t * f32(2) - f32(1)).astype(f32)
    if scale_mode == 7:
        return np.trunc((t * f32(255)).astype(f32) + f32(0.5)).astype(f32)
    return t
