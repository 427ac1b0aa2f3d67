"""CPU oracle for the output contract (TEST INFRASTRUCTURE ONLY; see oracle/oracle.h).

numpy restatements, in float32 arithmetic, of:
  PoseExtractorNet::getHeatMapsCopy     src/openpose/pose/poseExtractorNet.cpp:106-244
  PoseExtractorNet::getCandidatesCopy   src/openpose/pose/poseExtractorNet.cpp:246-282
  KeypointScaler::scale                 src/openpose/core/keypointScaler.cpp:6-95
  KeepTopNPeople::keepTopPeople         src/openpose/core/keepTopNPeople.cpp:16-86
  getKeypointsRectangle / Area          src/openpose/utilities/keypoint.cpp:289-389
  savePeopleJson (+ addKeypointsToJson,  src/openpose/filestream/fileStream.cpp:20-130,306-344,
    addCandidatesToJson, JsonOfstream)   src/openpose/filestream/jsonOfstream.cpp
Parity unpinned for keypoint.cpp-based code (it includes OpenCV, absent here); the others are
plain float code restated line by line.
"""
import numpy as np

f32 = np.float32
# op::ScaleMode (include/openpose/core/enumClasses.hpp:6-17)
INPUT_RESOLUTION, NET_OUTPUT_RESOLUTION, OUTPUT_RESOLUTION, ZERO_TO_ONE, ZERO_TO_ONE_FIXED, \
    PLUS_MINUS_ONE, PLUS_MINUS_ONE_FIXED, UNSIGNED_CHAR, NO_SCALE = range(9)


def _trunc(v, lo):   # fastTruncate(v, lo, 1) = fastMin(1, fastMax(lo, v))
    m = np.where(f32(lo) > v, f32(lo), v)
    return np.where(f32(1) < m, f32(1), m).astype(f32)


def heatmaps_copy(heat, parts, bkg, npaf, types=7, scale_mode=NO_SCALE):
    """heat [C, H, W] (parts, [bkg], PAFs) -> the copied/scaled [C', H, W] of getHeatMapsCopy."""
    heat = heat.astype(f32)
    out = []
    if types & 1:
        out.append(_scale_parts(heat[:parts], scale_mode))
    if types & 2:
        if not bkg:
            raise ValueError("model has no background channel")
        out.append(_scale_parts(heat[parts:parts + 1], scale_mode))
    if types & 4:
        p0 = parts + (1 if bkg else 0)
        out.append(_scale_pafs(heat[p0:p0 + npaf], scale_mode))
    return np.concatenate(out, 0)


def _scale_parts(v, mode):
    if mode == NO_SCALE:
        return v
    t = _trunc(v, 0.0)
    if mode in (PLUS_MINUS_ONE, PLUS_MINUS_ONE_FIXED):
        return (t * f32(2) - f32(1)).astype(f32)
    if mode == UNSIGNED_CHAR:   # (float)positiveIntRound(t * 255.f)
        return np.trunc(t * f32(255) + f32(0.5)).astype(f32)
    return t


def _scale_pafs(v, mode):
    if mode == NO_SCALE:
        return v
    t = _trunc(v, -1.0)
    if mode in (ZERO_TO_ONE, ZERO_TO_ONE_FIXED):
        return (t * f32(0.5) + f32(0.5)).astype(f32)
    if mode == UNSIGNED_CHAR:
        return np.trunc((t * f32(128.5) + f32(128.5)) + f32(0.5)).astype(f32)
    return t


def candidates(peaks, scale_net_to_output):
    """peaks [parts][128][3] -> list of [count, 3] (x, y * scaleNetToOutput, score)."""
    s = f32(scale_net_to_output)
    out = []
    for p in range(peaks.shape[0]):
        n = int(np.round(peaks[p, 0, 0]))
        c = peaks[p, 1:n + 1].astype(f32).copy()
        c[:, 0] *= s
        c[:, 1] *= s
        out.append(c)
    return out


def scale_keypoints(kp, mode, scale_input_to_output=1.0, scale_net_to_output=1.0,
                    producer_size=(1, 1)):
    kp = np.asarray(kp, f32).copy()
    if mode == INPUT_RESOLUTION:
        return kp
    pw, ph = f32(producer_size[0]), f32(producer_size[1])
    ox = oy = f32(0)
    if mode == OUTPUT_RESOLUTION:
        sx = sy = f32(scale_input_to_output)
    elif mode == NET_OUTPUT_RESOLUTION:
        sx = sy = f32(1.0 / scale_net_to_output)
    elif mode == ZERO_TO_ONE:
        sx, sy = f32(1) / (pw - f32(1)), f32(1) / (ph - f32(1))
    elif mode == ZERO_TO_ONE_FIXED:
        sx = sy = f32(1) / (max(pw, ph) - f32(1))
    elif mode == PLUS_MINUS_ONE:
        ox = oy = f32(-1)
        sx, sy = f32(2) / (pw - f32(1)), f32(2) / (ph - f32(1))
    elif mode == PLUS_MINUS_ONE_FIXED:
        ox = oy = f32(-1)
        sx = sy = f32(2) / (max(pw, ph) - f32(1))
    else:
        raise ValueError("Unknown ScaleMode selected.")
    if ox == 0 and oy == 0:
        if sx != 1 or sy != 1:
            kp[..., 0] *= sx
            kp[..., 1] *= sy
    else:
        kp[..., 0] = kp[..., 0] * sx + ox
        kp[..., 1] = kp[..., 1] * sy + oy
    return kp


def keypoints_area(person, threshold=0.05):
    big = np.finfo(np.float32).max
    minx, maxx, miny, maxy = f32(big), f32(-big), f32(big), f32(-big)
    for x, y, s in person.astype(f32):
        if s > f32(threshold):
            if maxx < x:
                maxx = x
            if minx > x:
                minx = x
            if maxy < y:
                maxy = y
            if miny > y:
                miny = y
    if maxx >= minx and maxy >= miny:
        return f32(maxx - minx) * f32(maxy - miny)
    return f32(0)


def keep_top_n_people(kp, scores, max_people):
    kp = np.asarray(kp, f32)
    n = kp.shape[0]
    if not (n > max_people > 0):
        return kp.copy(), np.arange(n)
    fin = np.array([f32(scores[p]) * np.sqrt(keypoints_area(kp[p])) for p in range(n)], f32)
    th = np.sort(fin)[::-1][max_people - 1]
    above = int((fin > th).sum())
    add = max_people - above
    out = np.zeros((max_people,) + kp.shape[1:], f32)
    idx = []
    on_th = 0
    for p in range(n):
        if fin[p] >= th:
            if fin[p] == th:
                on_th += 1
            if fin[p] > th or on_th <= add:
                out[len(idx)] = kp[p]
                idx.append(p)
    return out, np.array(idx)


# ---- savePeopleJson ------------------------------------------------------------------------
def _fmt(v):
    """std::ostream << float with the default format (precision 6, %g) -- jsonOfstream.hpp:40-44."""
    return "%g" % float(f32(v))


def people_json(keypoint_vector, candidates=None, human_readable=False):
    """op::savePeopleJson's file text.  keypoint_vector: [(array or None, name)], arrays of 1 or
    3 dimensions; op::Array::getSize (array.cpp:421-437): missing dimensions count 1, empty 0."""
    out = []
    braces = brackets = 0

    def enter():
        if human_readable:
            out.append("\n" + "\t" * (braces + brackets))

    def size(a, i):
        if a is None or np.asarray(a).size == 0:
            return 0
        a = np.asarray(a)
        return a.shape[i] if i < a.ndim else 1

    braces += 1
    out.append("{")                                    # objectOpen
    enter()
    out.append('"version":')                           # version("1.3")
    out.append("1.3")
    out.append(",")
    enter()
    out.append('"people":')                            # addKeypointsToJson
    brackets += 1
    out.append("[")
    enter()
    people = max([size(a, 0) for a, _ in keypoint_vector] + [0])
    for p in range(people):
        braces += 1
        out.append("{")
        for v, (a, name) in enumerate(keypoint_vector):
            per_row = size(a, 1) * size(a, 2)
            enter()
            out.append('"%s":' % name)
            brackets += 1
            out.append("[")
            enter()
            if per_row > 0:
                row = np.asarray(a, f32).reshape(-1)[p * per_row:(p + 1) * per_row]
                out.append(",".join(_fmt(x) for x in row))
            brackets -= 1
            enter()
            out.append("]")
            if v < len(keypoint_vector) - 1:
                out.append(",")
        braces -= 1
        enter()
        out.append("}")
        if p < people - 1:
            out.append(",")
            enter()
    brackets -= 1
    enter()
    out.append("]")
    if candidates:                                      # addCandidatesToJson
        out.append(",")
        enter()
        out.append('"part_candidates":')
        brackets += 1
        out.append("[")
        enter()
        braces += 1
        out.append("{")
        for part, cl in enumerate(candidates):
            enter()
            out.append('"%d":' % part)
            brackets += 1
            out.append("[")
            enter()
            out.append(",".join(_fmt(x) for c in cl for x in c[:3]))
            brackets -= 1
            enter()
            out.append("]")
            if part < len(candidates) - 1:
                out.append(",")
        braces -= 1
        enter()
        out.append("}")
        brackets -= 1
        enter()
        out.append("]")
    braces -= 1
    enter()
    out.append("}")
    enter()                                             # ~JsonOfstream
    return "".join(out)
