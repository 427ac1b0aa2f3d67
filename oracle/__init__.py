"""CPU oracle for the OpenPose BODY_25 hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and
only as the checker or the timed CPU baseline.  The product (libopk_hip.so / openpose_amd) never
imports it.  See oracle/oracle.h for what each function restates and its pinning status:
the connector is pinned against the reference's own compiled code (oracle/_ref); NMS, the OpenCV
bicubic resize and the Caffe layers are "parity unpinned" restatements (their reference code needs
OpenCV / Caffe, which this image does not have).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i = ctypes.c_int
_f = ctypes.c_float


def build(ref=True):
    """Compile liboracle.so (and oracle/_ref when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", _HERE, "all"], check=True)
    if ref and os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", _HERE, "ref"], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build(ref=False)
        L = ctypes.CDLL(path)
        L.orc_nms.argtypes = [_f32p, _f32p, _f, _i, _i, _i, _i, _f, _f]
        L.orc_nms_cuda.argtypes = [_f32p, _f32p, _f, _i, _i, _i, _i, _f, _f]
        L.orc_resize_merge_cuda.argtypes = [_f32p, ctypes.POINTER(ctypes.c_void_p), _i, _i, _i32p,
                                            _i, _i, ctypes.c_void_p]
        L.orc_resize_cubic.argtypes = [_f32p, _f32p, _i, _i, _i, _i]
        L.orc_resize_merge.argtypes = [_f32p, ctypes.POINTER(ctypes.c_void_p), _i, _i, _i32p, _i, _i]
        L.orc_cubic_tables.argtypes = [_i, _i, _i32p, _f32p]
        L.orc_set_resize_simd.argtypes = [_i]
        L.orc_resize_simd.restype = _i
        L.orc_paf_score.restype = _f
        L.orc_paf_score.argtypes = [_f32p, _f32p, _f32p, _f32p, _i, _i, _f, _f, _f]
        L.orc_connect_body_parts.argtypes = [_f32p, _f32p, _i, _f32p, _f32p, _i, _i, _i, _i, _f,
                                             _f, _i, _f, _f, _f, _i]
        L.orc_connect_from_scores.argtypes = [_f32p, _f32p, _i, _f32p, _f32p, _i, _i, _i, _f, _f, _i]
        L.orc_connect_gpu_semantics.argtypes = [_f32p, _f32p, _i, _f32p, _f32p, _i, _i, _i, _f, _f,
                                                _i]
        _u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
        L.orc_connect_gpu_tables.argtypes = [_f32p, _f32p, _i, _f32p, _f32p, _i, _i, _u32p, _i, _i,
                                             _f, _f, _i]
        L.orc_pair_scores.argtypes = [_f32p, _f32p, _f32p, _i, _u32p, _u32p, _u32p, _i, _i, _i, _f,
                                      _f, _f]
        L.orc_conv2d.argtypes = [_f32p, _f32p, _f32p, _f32p, _i, _i, _i, _i, _i, _i, _i, _i]
        L.orc_prelu.argtypes = [_f32p, _f32p, _i, _i, _i]
        L.orc_relu.argtypes = [_f32p, ctypes.c_long]
        L.orc_maxpool.argtypes = [_f32p, _f32p, _i, _i, _i, _i, _i, _i, _i, _i]
        _u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        L.orc_scale_and_size.argtypes = [_i, _i, _i, _i, _f, _i, ctypes.c_double,
                                         np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS"),
                                         _i32p]
        L.orc_cvmat_to_input.argtypes = [_f32p, _u8p, _i, _i, ctypes.c_double, _i, _i, _i]
        _i16p = np.ctypeslib.ndpointer(np.int16, flags="C_CONTIGUOUS")
        L.orc_warp_tab.argtypes = [_i, _i16p]
        L.orc_warp_affine_inv.argtypes = [_f32p, _u8p, _i, _i,
                                          np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS"),
                                          _i, _i, _i]
        L.orc_render_keypoints.argtypes = [_f32p, _i, _i, _f32p, _i, _i, _u32p, _i, _f32p, _i,
                                           _f32p, _i, _f, _f, _f, _f, _i, _i, _i, _u8p]
        L.orc_render_heat_map.argtypes = [_f32p, _i, _i, _f32p, _i, _i, _f, _i, _f, _i]
        L.orc_render_heat_maps.argtypes = [_f32p, _i, _i, _f32p, _i, _i, _f, _i, _f32p, _i, _f]
        L.orc_render_pafs.argtypes = [_f32p, _i, _i, _f32p, _i, _i, _f, _i, _i, _f]
        _LIB = L
    return _LIB


def ref_lib():
    """The reference's own connector (compiled from /root/reference), or None if unavailable.

    Only where the reference tree itself is present (this container): a copy of oracle/_ref that
    travelled with the repository to the GPU box is never loaded there -- the GPU tests check
    against the committed fixtures (tests/golden/) that this build produced."""
    global _REF
    if _REF is None:
        if not os.path.isdir("/root/reference"):
            return None
        path = os.path.join(_HERE, "_ref", "libref_connector.so")
        if not os.path.exists(path):
            build(ref=True)
        R = ctypes.CDLL(path, mode=os.RTLD_LAZY)  # OpenCV-only symbols stay unresolved
        R.ref_connect_cpu.argtypes = [_f32p, _f32p, _i, _f32p, _f32p, _i, _i, _i, _i, _f, _f, _i,
                                      _f, _f, _f, _i]
        R.ref_connect_gpu_assembly.argtypes = [_f32p, _f32p, _i, _f32p, _f32p, _i, _i, _i, _f, _f,
                                               _i]
        R.ref_gpu_face_merge_reached.argtypes = [_f32p, _f32p, _i, _i, _i, _f, _i]
        _REF = R
    return _REF


# ---- numpy front ends -------------------------------------------------------------------------
def nms(heat, threshold, max_peaks1=128, offset=(0.0, 0.0), channels=25, cuda=False):
    """nmsCpu (or, cuda=True, nmsGpu's rules) on one frame's heat maps [C, H, W]."""
    heat = np.ascontiguousarray(heat, np.float32)
    c, h, w = heat.shape
    channels = min(channels, c)
    out = np.zeros((channels, max_peaks1, 3), np.float32)
    fn = lib().orc_nms_cuda if cuda else lib().orc_nms
    fn(out, heat, threshold, channels, max_peaks1, h, w, offset[0], offset[1])
    return out


def resize_cubic(src, dh, dw):
    src = np.ascontiguousarray(src, np.float32)
    out = np.empty((dh, dw), np.float32)
    lib().orc_resize_cubic(out, src, src.shape[0], src.shape[1], dh, dw)
    return out


def resize_merge(srcs, dh, dw):
    """srcs: list of [C, h_i, w_i] arrays -> [C, dh, dw] (resizeAndMergeCpu semantics)."""
    srcs = [np.ascontiguousarray(s, np.float32) for s in srcs]
    c = srcs[0].shape[0]
    out = np.empty((c, dh, dw), np.float32)
    ptrs = (ctypes.c_void_p * len(srcs))(*[s.ctypes.data for s in srcs])
    hw = np.array([[s.shape[1], s.shape[2]] for s in srcs], np.int32).ravel()
    lib().orc_resize_merge(out, ptrs, len(srcs), c, hw, dh, dw)
    return out


def resize_merge_cuda(srcs, dh, dw, scale_ratios=None):
    """resizeAndMergeGpu (CUDA build) of one frame: srcs list of [C, h_i, w_i] -> [C, dh, dw];
    None where the reference raises (non-x8 single source, > 8 sources)."""
    srcs = [np.ascontiguousarray(s, np.float32) for s in srcs]
    c = srcs[0].shape[0]
    out = np.empty((c, dh, dw), np.float32)
    ptrs = (ctypes.c_void_p * len(srcs))(*[s.ctypes.data for s in srcs])
    hw = np.array([[s.shape[1], s.shape[2]] for s in srcs], np.int32).ravel()
    r = None if scale_ratios is None else np.ascontiguousarray(scale_ratios, np.float32)
    rc = r.ctypes.data if r is not None else None
    if lib().orc_resize_merge_cuda(out, ptrs, len(srcs), c, hw, dh, dw, rc) != 0:
        return None
    return out


class resize_order:
    """Context manager: the OpenCV version whose vertical summation order the resize restatement
    follows ("4.x": SIMD body of 4 lanes, the default; "3.x": left to right; see resize.c)."""

    def __init__(self, version):
        self.lanes = {"4.x": 4, "3.x": 0}[version]

    def __enter__(self):
        self.prev = lib().orc_resize_simd()
        lib().orc_set_resize_simd(self.lanes)
        return self

    def __exit__(self, *exc):
        lib().orc_set_resize_simd(self.prev)
        return False


def cubic_tables(s, d):
    ofs = np.empty(d, np.int32)
    coef = np.empty((d, 4), np.float32)
    lib().orc_cubic_tables(s, d, ofs, coef)
    return ofs, coef


def _connect_args(params):
    p = dict(inter_min_above=0.95, inter_th=0.05, min_subset_cnt=3, min_subset_score=0.4,
             nms_th=0.05, scale=1.0, maximize_positives=False, pose_model=0, max_people=512)
    p.update(params)
    return p


def connect(heat, peaks, use_reference=False, **params):
    """connectBodyPartsCpu semantics -> (keypoints [P, parts, 3], scores [P])."""
    p = _connect_args(params)
    heat = np.ascontiguousarray(heat, np.float32)
    peaks = np.ascontiguousarray(peaks, np.float32)
    nparts = peaks.shape[0]
    kp = np.zeros((p["max_people"], nparts, 3), np.float32)
    ks = np.zeros(p["max_people"], np.float32)
    fn = ref_lib().ref_connect_cpu if use_reference else lib().orc_connect_body_parts
    n = fn(kp, ks, p["max_people"], heat, peaks, p["pose_model"], heat.shape[2], heat.shape[1],
           peaks.shape[1] - 1, p["inter_min_above"], p["inter_th"], p["min_subset_cnt"],
           p["min_subset_score"], p["nms_th"], p["scale"], int(p["maximize_positives"]))
    if n < 0:
        raise RuntimeError("oracle connector rejected the model")
    n = min(n, p["max_people"])
    return kp[:n].copy(), ks[:n].copy()


def connect_from_scores(pair_scores, peaks, gpu_semantics=False, **params):
    p = _connect_args(params)
    pair_scores = np.ascontiguousarray(pair_scores, np.float32)
    peaks = np.ascontiguousarray(peaks, np.float32)
    nparts = peaks.shape[0]
    kp = np.zeros((p["max_people"], nparts, 3), np.float32)
    ks = np.zeros(p["max_people"], np.float32)
    fn = lib().orc_connect_gpu_semantics if gpu_semantics else lib().orc_connect_from_scores
    n = fn(kp, ks, p["max_people"], pair_scores, peaks, p["pose_model"], peaks.shape[1] - 1,
           p["min_subset_cnt"], p["min_subset_score"], p["scale"], int(p["maximize_positives"]))
    n = min(n, p["max_people"])
    return kp[:n].copy(), ks[:n].copy()


def pose_tables():
    """Pose tables of every PoseModel as the reference computes them (tests/golden/pose_tables.json,
    written by tools/gen_pose_tables.py from the reference's poseParameters.cpp)."""
    import json
    with open(os.path.join(_HERE, "..", "tests", "golden", "pose_tables.json")) as f:
        return json.load(f)


def face_merge_reached(pair_scores, peaks, table, **params):
    """Whether the reference's removePeopleBelowThresholdsAndFillFaces runs its BODY_135
    face-fragment merge on this input (oracle/_ref)."""
    p = _connect_args(params)
    return bool(ref_lib().ref_gpu_face_merge_reached(
        np.ascontiguousarray(pair_scores, np.float32), np.ascontiguousarray(peaks, np.float32),
        table["id"], peaks.shape[1] - 1, p["min_subset_cnt"], p["min_subset_score"],
        int(p["maximize_positives"])))


def connect_gpu_semantics(pair_scores, peaks, table, use_reference=False, **params):
    """connectBodyPartsGpu host assembly for any model (table: a pose_tables() entry).  With
    use_reference the reference's own pafVectorIntoPeopleVector / removePeople... run (its
    face-fragment merge with the restated getKeypointsRoi, oracle/ref_driver.cpp)."""
    p = _connect_args(params)
    pair_scores = np.ascontiguousarray(pair_scores, np.float32)
    peaks = np.ascontiguousarray(peaks, np.float32)
    nparts = peaks.shape[0]
    kp = np.zeros((p["max_people"], nparts, 3), np.float32)
    ks = np.zeros(p["max_people"], np.float32)
    if use_reference:
        n = ref_lib().ref_connect_gpu_assembly(kp, ks, p["max_people"], pair_scores, peaks,
                                               table["id"], peaks.shape[1] - 1, p["min_subset_cnt"],
                                               p["min_subset_score"], p["scale"],
                                               int(p["maximize_positives"]))
        if n == -2:
            return None
    else:
        pairs = np.asarray(table["pairs"], np.uint32)
        n = lib().orc_connect_gpu_tables(kp, ks, p["max_people"], pair_scores, peaks, nparts,
                                         len(pairs) // 2, pairs, peaks.shape[1] - 1,
                                         p["min_subset_cnt"], p["min_subset_score"], p["scale"],
                                         int(p["maximize_positives"]))
    n = min(n, p["max_people"])
    return kp[:n].copy(), ks[:n].copy()


def pair_scores_table(heat, peaks, table, inter_th=0.05, inter_min_above=0.95, nms_th=0.05):
    """Dense [npairs, maxPeaks, maxPeaks] getScoreAB table for any model (PAF channel of pair q:
    parts + bkg + map_idx)."""
    heat = np.ascontiguousarray(heat, np.float32)
    peaks = np.ascontiguousarray(peaks, np.float32)
    pairs = np.asarray(table["pairs"], np.uint32)
    npairs = len(pairs) // 2
    base = table["parts"] + (1 if table["bkg"] else 0)
    mi = np.asarray(table["map_idx"], np.uint32)
    mapx = np.ascontiguousarray(base + mi[0:2 * npairs:2], np.uint32)
    mapy = np.ascontiguousarray(base + mi[1:2 * npairs:2], np.uint32)
    mp = peaks.shape[1] - 1
    out = np.zeros((npairs, mp, mp), np.float32)
    lib().orc_pair_scores(out, heat, peaks, npairs, pairs, mapx, mapy, heat.shape[2],
                          heat.shape[1], mp, inter_th, inter_min_above, nms_th)
    return out


def paf_score(a, b, mapx, mapy, inter_th=0.05, inter_min_above=0.95, nms_th=0.05):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    mapx = np.ascontiguousarray(mapx, np.float32)
    mapy = np.ascontiguousarray(mapy, np.float32)
    return lib().orc_paf_score(a, b, mapx, mapy, mapx.shape[1], mapx.shape[0], inter_th,
                               inter_min_above, nms_th)


def pair_scores(heat, peaks, pairs, map_idx, nparts=25, **kw):
    """Full [npairs, maxPeaks, maxPeaks] score table via getScoreAB (0 for absent peaks)."""
    mp = peaks.shape[1] - 1
    npairs = len(pairs) // 2
    out = np.zeros((npairs, mp, mp), np.float32)
    for q in range(npairs):
        pa, pb = pairs[2 * q], pairs[2 * q + 1]
        na, nb = int(peaks[pa, 0, 0] + 0.5), int(peaks[pb, 0, 0] + 0.5)
        mx = heat[nparts + 1 + map_idx[2 * q]]
        my = heat[nparts + 1 + map_idx[2 * q + 1]]
        for i in range(na):
            for j in range(nb):
                out[q, i, j] = paf_score(peaks[pa, i + 1], peaks[pb, j + 1], mx, my, **kw)
    return out


# ---- Caffe layers -----------------------------------------------------------------------------
def scale_and_size(input_size, net_resolution=(-1, 368), dynamic_behavior=1.0, scale_number=1,
                   scale_gap=0.25):
    """ScaleAndSizeExtractor::extract restated (preprocess.c): (scales, [(w, h)])."""
    scales = np.zeros(scale_number, np.float64)
    sizes = np.zeros(2 * scale_number, np.int32)
    rc = lib().orc_scale_and_size(input_size[0], input_size[1], net_resolution[0],
                                  net_resolution[1], dynamic_behavior, scale_number, scale_gap,
                                  scales, sizes)
    if rc != 0:
        raise ValueError("invalid scale/size configuration")
    return list(scales), [(int(sizes[2 * i]), int(sizes[2 * i + 1])) for i in range(scale_number)]


def cvmat_to_input(frame, scale, net_w, net_h, normalize=1):
    """CvMatToOpInput for one BGR uint8 frame [h, w, 3] -> [3, net_h, net_w] float32."""
    frame = np.ascontiguousarray(frame, np.uint8)
    out = np.empty((3, net_h, net_w), np.float32)
    lib().orc_cvmat_to_input(out, frame, frame.shape[1], frame.shape[0], float(scale), net_w,
                             net_h, normalize)
    return out


def warp_affine_inv(frame, M, net_w, net_h, normalize=1):
    """Face / hand crop: warpAffine(INTER_LINEAR | WARP_INVERSE_MAP) of a BGR uint8 frame [h, w, 3]
    with the 2x3 matrix M -> [3, net_h, net_w] float32."""
    frame = np.ascontiguousarray(frame, np.uint8)
    out = np.empty((3, net_h, net_w), np.float32)
    lib().orc_warp_affine_inv(out, frame, frame.shape[1], frame.shape[0],
                              np.ascontiguousarray(M, np.float64).ravel(), net_w, net_h, normalize)
    return out


def warp_weight_table(cubic):
    k = 4 if cubic else 2
    t = np.zeros(1025 * k * k, np.int16)
    lib().orc_warp_tab(int(cubic), t)
    return t[:1024 * k * k].reshape(32, 32, k, k)


def default_threads():
    """OMP_NUM_THREADS if set (16 on the GPU box: its CPU share), else min(16, cpu_count)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return max(1, min(16, os.cpu_count() or 1))


def conv2d(x, w, b, pad, nthreads=None):
    x = np.ascontiguousarray(x, np.float32)
    w = np.ascontiguousarray(w, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    n, ci, h, wd = x.shape
    co, _, k, _ = w.shape
    out = np.empty((n, co, h, wd), np.float32)
    lib().orc_conv2d(out, x, w, b, n, ci, h, wd, co, k, pad, nthreads or default_threads())
    return out


def prelu(x, slope):
    n, c, h, w = x.shape
    lib().orc_prelu(x, np.ascontiguousarray(slope, np.float32), n, c, h * w)
    return x


def relu(x):
    lib().orc_relu(x, x.size)
    return x


def maxpool(x, k=2, s=2):
    n, c, h, w = x.shape
    oh = -(-(h - k) // s) + 1
    ow = -(-(w - k) // s) + 1
    out = np.empty((n, c, oh, ow), np.float32)
    lib().orc_maxpool(out, np.ascontiguousarray(x), n, c, h, w, k, s, oh, ow)
    return out


# ---- renderers (render.c) ---------------------------------------------------------------------
# renderPoseKeypointsGpu's model -> (render table, scales table, parts, googly eyes)
# (renderPose.cu:129-417, 639-741); face / hand (renderFace.cu:21-46, renderHand.cu:21-46)
RENDER_POSE = {0: ("BODY_25", "BODY_25", 25, (15, 16)), 7: ("BODY_25", "BODY_25", 25, (15, 16)),
               9: ("BODY_25", "BODY_25", 25, (15, 16)), 1: ("COCO", "COCO", 18, (14, 15)),
               2: ("MPI", "COCO", 15, (-1, -1)), 3: ("MPI", "COCO", 15, (-1, -1)),
               4: ("BODY_19", "BODY_19", 19, (15, 16)), 5: ("BODY_19", "BODY_19", 19, (15, 16)),
               6: ("BODY_19", "BODY_19", 19, (15, 16)), 12: ("BODY_19", "BODY_19", 19, (15, 16)),
               8: ("CAR_12", "CAR_12", 12, (4, 5)), 10: ("BODY_23", "BODY_23", 23, (13, 14)),
               11: ("CAR_22", "CAR_22", 22, (6, 7)), 13: ("BODY_25B", "BODY_25B", 25, (1, 2)),
               14: ("BODY_135", "BODY_135", 135, (1, 2))}


def render_tables():
    """The reference's GPU render tables (tests/golden/render_tables.json, written by
    tools/gen_render_tables.py from its *_RENDER_GPU macros), by name."""
    import json
    with open(os.path.join(_HERE, "..", "tests", "golden", "render_tables.json")) as f:
        return {d["name"]: d for d in json.load(f)}


def render_keypoints(frame, kp, table, scales_table=None, parts=None, radius_div=100.0,
                     line_div=120.0, threshold=0.05, alpha=0.6, blend=True, eyes=(-1, -1)):
    """renderKeypointsOld on a copy of frame (float BGR [h][w][3]); kp [people][parts][3].
    Returns (frame, ambiguous [h][w] uint8)."""
    tabs = render_tables()
    t = tabs[table]
    st = tabs[scales_table or table]
    out = np.ascontiguousarray(frame, np.float32).copy()
    h, w = out.shape[:2]
    kp = np.ascontiguousarray(kp, np.float32).reshape(-1, parts or kp.shape[1], 3)
    amb = np.zeros((h, w), np.uint8)
    m = min(w, h)
    lib().orc_render_keypoints(out, w, h, kp, kp.shape[0], kp.shape[1],
                               np.asarray(t["pairs"], np.uint32), len(t["pairs"]) // 2,
                               np.asarray(t["colors"], np.float32), len(t["colors"]) // 3,
                               np.asarray(st["scales"], np.float32), len(t["scales"]),
                               np.float32(m) / np.float32(radius_div),
                               np.float32(m) / np.float32(line_div), threshold, alpha,
                               1 if blend else 0, eyes[0], eyes[1], amb)
    return out, amb


def render_heat_map(frame, heat, scale, part, alpha=0.7, abs_value=False):
    out = np.ascontiguousarray(frame, np.float32).copy()
    heat = np.ascontiguousarray(heat, np.float32)
    lib().orc_render_heat_map(out, out.shape[1], out.shape[0], heat, heat.shape[-1],
                              heat.shape[-2], scale, part, alpha, 1 if abs_value else 0)
    return out


def render_heat_maps(frame, heat, scale, parts, alpha=0.7):
    colors = np.asarray(render_tables()["COCO"]["colors"], np.float32)
    out = np.ascontiguousarray(frame, np.float32).copy()
    heat = np.ascontiguousarray(heat, np.float32)
    lib().orc_render_heat_maps(out, out.shape[1], out.shape[0], heat, heat.shape[-1],
                               heat.shape[-2], scale, parts, colors, len(colors) // 3, alpha)
    return out


def render_pafs(frame, heat, scale, first, count, alpha=0.7):
    out = np.ascontiguousarray(frame, np.float32).copy()
    heat = np.ascontiguousarray(heat, np.float32)
    lib().orc_render_pafs(out, out.shape[1], out.shape[0], heat, heat.shape[-1], heat.shape[-2],
                          scale, first, count, alpha)
    return out
