"""Python front end over the C-ABI (used by tests and bench.py).

Device memory is handed over as torch CUDA tensors (PyTorch is plumbing here: allocation, streams,
torch.distributed); every computation runs in libopk_hip.so.  The function names mirror the
reference operators they replace (include/opk.h lists the reference file:line of each).
"""
import atexit
import ctypes
import weakref

import numpy as np
import torch

from . import _lib
from ._lib import check, int4
from .pose_tables import (BODY_25, CONNECT_CPU, CONNECT_GPU, CONNECT_INTER_MIN_ABOVE_THRESHOLD,
                          CONNECT_INTER_THRESHOLD,
                          CONNECT_MIN_SUBSET_CNT, CONNECT_MIN_SUBSET_SCORE, NMS_THRESHOLD)

# heat-map semantics (include/opk.h OPK_MAPS_*): the reference's CPU build or its CUDA build
MAPS_CPU, MAPS_CUDA = 0, 1
PRECISION_FP16, PRECISION_SPLIT = 0, 1      # opk_net_set_precision


def _ptr(t):
    if t is None:
        return None
    assert t.is_cuda and t.is_contiguous(), "device tensors must be contiguous CUDA tensors"
    return ctypes.c_void_p(t.data_ptr())


# Handles still open at interpreter exit (e.g. held by a test traceback) are closed before the HIP
# runtime's own teardown: poses, then nets, then contexts.
_LIVE = {"pose": weakref.WeakSet(), "extractor": weakref.WeakSet(), "net": weakref.WeakSet(),
         "ctx": weakref.WeakSet()}


@atexit.register
def _close_live():
    for kind in ("pose", "extractor", "net", "ctx"):
        for obj in list(_LIVE[kind]):
            try:
                obj.close()
            except Exception:
                pass


class dev_switches:
    """Context manager setting kernel-variant switches (opk_dev_set; A/B tests and tuning only),
    e.g. `with dev_switches(CONV3_W16=0): ...`; the product defaults are restored on exit."""

    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        L = _lib.load()
        for k, v in self.kv.items():
            check(L.opk_dev_set(k.encode(), int(v), 0))
        return self

    def __exit__(self, *exc):
        L = _lib.load()
        for k in self.kv:
            L.opk_dev_set(k.encode(), 0, 1)
        return False


class Context:
    """One opk_ctx bound to a device; runs on torch's current stream of that device."""

    def __init__(self, device=0, stream=None):
        self.L = _lib.load()
        self.device = device
        torch.cuda.set_device(device)
        s = stream if stream is not None else torch.cuda.current_stream(device)
        self.torch_stream = s
        h = ctypes.c_void_p()
        check(self.L.opk_ctx_create(device, ctypes.c_void_p(s.cuda_stream), ctypes.byref(h)))
        self.h = h
        _LIVE["ctx"].add(self)

    def close(self):
        if self.h:
            self.L.opk_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(self.L.opk_sync(self.h))

    @classmethod
    def host_only(cls):
        """A device-less context (-1): graph planning and conv listing only."""
        self = cls.__new__(cls)
        self.L = _lib.load()
        self.device = -1
        self.torch_stream = None
        h = ctypes.c_void_p()
        check(self.L.opk_ctx_create(-1, None, ctypes.byref(h)))
        self.h = h
        _LIVE["ctx"].add(self)
        return self

    # ---- operators ---------------------------------------------------------------------------
    def convert(self, dst, src):
        """dst <- src element-wise on the device (float32 <-> float64, opk_convert), same count."""
        kinds = {torch.float32: 0, torch.float64: 1}
        assert dst.numel() == src.numel() and dst.dtype in kinds and src.dtype in kinds
        assert dst.is_contiguous() and src.is_contiguous()
        check(self.L.opk_convert(self.h, _ptr(dst), kinds[dst.dtype], _ptr(src), kinds[src.dtype],
                                 src.numel()))

    def resize_and_merge(self, target, sources, semantics=MAPS_CPU, scale_ratios=None):
        """target [N,C,H,W] fp32 CUDA; sources list of [N,C,h,w] (resizeAndMergeGpu).  semantics
        MAPS_CPU: resizeAndMergeCpu's arithmetic; MAPS_CUDA: the CUDA build's (scale_ratios =
        scaleInputToNetInputs, needed with several sources)."""
        n = len(sources)
        ptrs = (ctypes.c_void_p * n)(*[s.data_ptr() for s in sources])
        sizes = (ctypes.c_int * (4 * n))(*[int(v) for s in sources for v in s.shape])
        ratios = None if scale_ratios is None else (ctypes.c_float * n)(*[float(r) for r in scale_ratios])
        check(self.L.opk_resize_and_merge_semantics(self.h, _ptr(target), ptrs, n,
                                                    int4(target.shape), sizes, ratios, semantics))

    def cvmat_to_input(self, net_input, frames, scale, normalize=1):
        """op::CvMatToOpInput for one scale: frames [n, h, w, 3] uint8 BGR (CUDA) ->
        net_input [n, 3, net_h, net_w] float32 (CUDA)."""
        n, h, w, c = frames.shape
        assert c == 3 and frames.dtype == torch.uint8
        assert net_input.shape[0] == n and net_input.shape[1] == 3
        check(self.L.opk_cvmat_to_input(self.h, _ptr(net_input), _ptr(frames), n, w, h, w * 3,
                                        float(scale), net_input.shape[3], net_input.shape[2],
                                        normalize))

    def nms(self, peaks, heat, threshold=NMS_THRESHOLD, offset=(0.0, 0.0), semantics=MAPS_CPU):
        """peaks [N,parts,maxPeaks+1,3]; heat [N,C,H,W] (nmsGpu; semantics MAPS_CPU: nmsCpu's
        rules, MAPS_CUDA: nmsGpu's)."""
        check(self.L.opk_nms_semantics(self.h, _ptr(peaks), None, _ptr(heat), threshold,
                                       int4(peaks.shape), int4(heat.shape), offset[0], offset[1],
                                       semantics))

    def probe_peaks(self):
        """Measured ceilings on this device (opk_probe_peaks): dense fp16 MFMA TFLOP/s on random
        and on zero operands, streaming HBM read GB/s."""
        r, z, h = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        check(self.L.opk_probe_peaks(self.h, ctypes.byref(r), ctypes.byref(z), ctypes.byref(h)))
        return {"mfma_fp16_random_tflops": round(r.value, 1), "mfma_fp16_zero_tflops": round(z.value, 1),
                "hbm_read_gbs": round(h.value, 1)}

    # ---- renderers (renderPose.cu / renderFace.cu / renderHand.cu) ---------------------------
    # frame: float32 CUDA [h, w, 3] BGR, drawn in place; keypoints float32 CUDA [people, parts, 3]
    def render_pose_keypoints(self, frame, pose, pose_model=BODY_25, threshold=0.05,
                              googly_eyes=False, blend_original=True, alpha=0.6):
        """op::renderPoseKeypointsGpu (POSE_DEFAULT_ALPHA_KEYPOINT 0.6)."""
        h, w = frame.shape[:2]
        people = 0 if pose is None else pose.shape[0]
        check(self.L.opk_render_pose_keypoints(self.h, _ptr(frame), pose_model, people, w, h,
                                               None if pose is None else _ptr(pose), threshold,
                                               int(googly_eyes), int(blend_original), alpha))

    def render_face_keypoints(self, frame, face, threshold=0.4, alpha=0.6):
        """op::renderFaceKeypointsGpu; face [people, 70, 3]."""
        h, w = frame.shape[:2]
        check(self.L.opk_render_face_keypoints(self.h, _ptr(frame), w, h, _ptr(face), face.shape[0],
                                               threshold, alpha))

    def render_hand_keypoints(self, frame, hands, threshold=0.2, alpha=0.6):
        """op::renderHandKeypointsGpu; hands [n, 21, 3]."""
        h, w = frame.shape[:2]
        check(self.L.opk_render_hand_keypoints(self.h, _ptr(frame), w, h, _ptr(hands),
                                               hands.shape[0], threshold, alpha))

    def render_heat_map(self, frame, heat, scale, part, alpha=0.7, distance=False):
        """op::renderPoseHeatMapGpu (distance: op::renderPoseDistanceGpu); heat [C, hh, hw]."""
        h, w = frame.shape[:2]
        fn = self.L.opk_render_pose_distance if distance else self.L.opk_render_pose_heat_map
        check(fn(self.h, _ptr(frame), w, h, _ptr(heat), heat.shape[-1], heat.shape[-2], scale,
                 part, alpha))

    def render_heat_maps(self, frame, heat, scale, pose_model=BODY_25, alpha=0.7):
        """op::renderPoseHeatMapsGpu."""
        h, w = frame.shape[:2]
        check(self.L.opk_render_pose_heat_maps(self.h, _ptr(frame), pose_model, w, h, _ptr(heat),
                                               heat.shape[-1], heat.shape[-2], scale, alpha))

    def render_pafs(self, frame, heat, scale, part=None, pose_model=BODY_25, alpha=0.7):
        """op::renderPosePAFGpu (part = its x channel) or, part None, op::renderPosePAFsGpu."""
        h, w = frame.shape[:2]
        if part is None:
            check(self.L.opk_render_pose_pafs(self.h, _ptr(frame), pose_model, w, h, _ptr(heat),
                                              heat.shape[-1], heat.shape[-2], scale, alpha))
        else:
            check(self.L.opk_render_pose_paf(self.h, _ptr(frame), pose_model, w, h, _ptr(heat),
                                             heat.shape[-1], heat.shape[-2], scale, part, alpha))

    def paf_scores(self, scores, heat, peaks, pose_model=BODY_25, inter_th=CONNECT_INTER_THRESHOLD,
                   inter_min_above=CONNECT_INTER_MIN_ABOVE_THRESHOLD, nms_th=NMS_THRESHOLD):
        n, c, h, w = heat.shape
        check(self.L.opk_paf_scores(self.h, _ptr(scores), _ptr(heat), _ptr(peaks), n, pose_model, c,
                                    h, w, peaks.shape[2] - 1, inter_th, inter_min_above, nms_th))

    def connect_body_parts(self, heat, peaks, pose_model=BODY_25, scale=1.0, max_people=512,
                           inter_min_above=CONNECT_INTER_MIN_ABOVE_THRESHOLD,
                           inter_th=CONNECT_INTER_THRESHOLD, min_subset_cnt=CONNECT_MIN_SUBSET_CNT,
                           min_subset_score=CONNECT_MIN_SUBSET_SCORE, nms_th=NMS_THRESHOLD,
                           maximize_positives=False, semantics=CONNECT_CPU):
        """One frame: heat [C,H,W] / [1,C,H,W], peaks [parts,maxPeaks+1,3] (connectBodyPartsGpu
        replacement; semantics CONNECT_CPU / CONNECT_GPU picks the people assembly)."""
        c, h, w = heat.shape[-3:]
        parts = peaks.shape[-3]
        kp = np.zeros((max_people, parts, 3), np.float32)
        ks = np.zeros(max_people, np.float32)
        n = ctypes.c_int()
        check(self.L.opk_connect_body_parts_semantics(
            self.h, kp.ctypes.data_as(ctypes.c_void_p), ks.ctypes.data_as(ctypes.c_void_p),
            max_people, ctypes.byref(n), _ptr(heat), _ptr(peaks), pose_model, c, h, w,
            peaks.shape[-2] - 1, inter_min_above, inter_th, min_subset_cnt, min_subset_score,
            nms_th, scale, int(maximize_positives), semantics))
        k = min(n.value, max_people)
        return kp[:k].copy(), ks[:k].copy()


def scale_and_size(input_size, net_resolution=(-1, 368), dynamic_behavior=1.0, scale_number=1,
                   scale_gap=0.25):
    """op::ScaleAndSizeExtractor::extract: ([scaleInputToNetInputs], [(net_w, net_h)])."""
    L = _lib.load()
    scales = (ctypes.c_double * scale_number)()
    sizes = (ctypes.c_int * (2 * scale_number))()
    check(L.opk_scale_and_size(input_size[0], input_size[1], net_resolution[0], net_resolution[1],
                               float(dynamic_behavior), scale_number, float(scale_gap), scales,
                               sizes))
    return list(scales), [(sizes[2 * i], sizes[2 * i + 1]) for i in range(scale_number)]


def scale_keypoints(keypoints, scale_mode, scale_input_to_output=1.0, scale_net_to_output=1.0,
                    producer_size=(1, 1)):
    """op::KeypointScaler::scale on a copy of keypoints [people, parts, 3]."""
    kp = np.ascontiguousarray(keypoints, np.float32).copy()
    check(_lib.load().opk_scale_keypoints(kp.ctypes.data_as(ctypes.c_void_p), kp.shape[0],
                                          kp.shape[1], scale_mode, float(scale_input_to_output),
                                          float(scale_net_to_output), producer_size[0],
                                          producer_size[1]))
    return kp


def keep_top_n_people(keypoints, scores, max_people):
    """op::KeepTopNPeople::keepTopPeople: (kept keypoints, source index of each kept row)."""
    kp = np.ascontiguousarray(keypoints, np.float32)
    sc = np.ascontiguousarray(scores, np.float32)
    rows = max(kp.shape[0], max_people, 1)
    out = np.zeros((rows,) + kp.shape[1:], np.float32)
    idx = np.full(rows, -1, np.int32)
    n = ctypes.c_int()
    check(_lib.load().opk_keep_top_n_people(kp.ctypes.data_as(ctypes.c_void_p), kp.shape[0],
                                            kp.shape[1], sc.ctypes.data_as(ctypes.c_void_p),
                                            max_people, out.ctypes.data_as(ctypes.c_void_p),
                                            idx.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)))
    return out[:n.value], idx[:n.value]


class _JsonKeypoints(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("data", ctypes.c_void_p), ("ndims", ctypes.c_int),
                ("people", ctypes.c_int), ("parts", ctypes.c_int), ("dims", ctypes.c_int)]


def _json_args(keypoint_vector, candidates):
    keep = []
    arr = (_JsonKeypoints * max(len(keypoint_vector), 1))()
    for i, (a, name) in enumerate(keypoint_vector):
        a = np.ascontiguousarray(a if a is not None else np.zeros(0), np.float32)
        keep.append(a)
        shape = a.shape if a.size else ()
        if len(shape) not in (0, 1, 3):
            shape = (None,) * 2   # rejected by the library like the reference
        dims = list(shape) + [0] * (3 - len(shape))
        arr[i] = _JsonKeypoints(name.encode(), a.ctypes.data if a.size else None, len(shape),
                                dims[0] or 0, dims[1] or 0, dims[2] or 0)
    cands = candidates or []
    counts = np.array([len(c) for c in cands], np.int32)
    flat = np.ascontiguousarray(
        np.concatenate([np.asarray(c, np.float32).reshape(-1, 3) for c in cands])
        if cands and counts.sum() else np.zeros((0, 3)), np.float32)
    keep += [counts, flat]
    return arr, keep, (flat.ctypes.data if flat.size else None,
                       counts.ctypes.data if counts.size else None, len(cands))


def people_json(keypoint_vector, candidates=None, human_readable=False):
    """op::savePeopleJson's file text (fileStream.cpp:306-344) for keypoint_vector = [(array, name)]
    (arrays [people][parts][3], [people] or empty) and candidates = per-part lists of [x, y, score]."""
    L = _lib.load()
    arr, keep, (cp, cc, nparts) = _json_args(keypoint_vector, candidates)
    n = ctypes.c_size_t()
    check(L.opk_people_json(arr, len(keypoint_vector), cp, cc, nparts, int(human_readable), None,
                            0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(n.value + 1)
    check(L.opk_people_json(arr, len(keypoint_vector), cp, cc, nparts, int(human_readable), buf,
                            n.value + 1, ctypes.byref(n)))
    del keep
    return buf.raw[:n.value].decode()


def save_people_json(path, keypoint_vector, candidates=None, human_readable=False):
    """PeopleJsonSaver::save (peopleJsonSaver.cpp:15-30): the same text written to path."""
    L = _lib.load()
    arr, keep, (cp, cc, nparts) = _json_args(keypoint_vector, candidates)
    check(L.opk_save_people_json(path.encode(), arr, len(keypoint_vector), cp, cc, nparts,
                                 int(human_readable)))
    del keep


def datum_keypoint_vector(pose_keypoints, face_keypoints=None, hand_keypoints=(None, None)):
    """The keypointVector WPeopleJsonSaver builds from a Datum (wPeopleJsonSaver.hpp:75-88):
    person ids (-1 each without a person-id extractor, PoseExtractor::extractIds,
    poseExtractor.cpp:136-151), the 2-D body / face / hand arrays and the (empty) 3-D ones."""
    pk = np.asarray(pose_keypoints, np.float32)
    ids = np.full(pk.shape[0], -1, np.float32) if pk.size else None
    return [(ids, "person_id"), (pk, "pose_keypoints_2d"), (face_keypoints, "face_keypoints_2d"),
            (hand_keypoints[0], "hand_left_keypoints_2d"),
            (hand_keypoints[1], "hand_right_keypoints_2d"), (None, "pose_keypoints_3d"),
            (None, "face_keypoints_3d"), (None, "hand_left_keypoints_3d"),
            (None, "hand_right_keypoints_3d")]


def caffemodel_blob(path, layer, index):
    """Host utility: (shape, float32 data) of a blob in a .caffemodel (opk_caffemodel_blob)."""
    L = _lib.load()
    shape = (ctypes.c_int64 * 8)()
    nd = ctypes.c_int()
    check(L.opk_caffemodel_blob(path.encode(), layer.encode(), index, None, 0, shape,
                                ctypes.byref(nd)))
    dims = tuple(shape[i] for i in range(nd.value))
    out = np.empty(int(np.prod(dims)) if dims else 0, np.float32)
    check(L.opk_caffemodel_blob(path.encode(), layer.encode(), index,
                                out.ctypes.data_as(ctypes.c_void_p), out.size, shape,
                                ctypes.byref(nd)))
    return dims, out.reshape(dims)


def pose_model_info(pose_model):
    """Tables of a PoseModel from libopk_hip: dict(parts, bkg, pairs, map_idx, heat_channels,
    nms_threshold, inter_threshold)."""
    L = _lib.load()
    parts, bkg, npairs, hc = (ctypes.c_int() for _ in range(4))
    check(L.opk_pose_model_info(pose_model, ctypes.byref(parts), ctypes.byref(bkg),
                                ctypes.byref(npairs), ctypes.byref(hc), None, None))
    pairs = np.zeros(2 * npairs.value, np.int32)
    nmap = hc.value - parts.value - bkg.value
    mi = np.zeros(max(nmap, 1), np.int32)
    check(L.opk_pose_model_info(pose_model, None, None, None, None,
                                pairs.ctypes.data_as(ctypes.c_void_p),
                                mi.ctypes.data_as(ctypes.c_void_p)))
    nms, inter = ctypes.c_float(), ctypes.c_float()
    check(L.opk_pose_default_thresholds(pose_model, 0, ctypes.byref(nms), ctypes.byref(inter)))
    return dict(id=pose_model, parts=parts.value, bkg=bool(bkg.value), pairs=pairs.tolist(),
                map_idx=mi[:nmap].tolist(), heat_channels=hc.value, nms_threshold=nms.value,
                inter_threshold=inter.value)


def assemble_people(pair_scores, peaks, pose_model=BODY_25, scale=1.0, max_people=512,
                    min_subset_cnt=CONNECT_MIN_SUBSET_CNT, min_subset_score=CONNECT_MIN_SUBSET_SCORE,
                    maximize_positives=False, semantics=CONNECT_CPU):
    """Host-only assembly from numpy pair scores [npairs,mp,mp] + peaks [parts,mp+1,3]."""
    L = _lib.load()
    pair_scores = np.ascontiguousarray(pair_scores, np.float32)
    peaks = np.ascontiguousarray(peaks, np.float32)
    parts = peaks.shape[0]
    kp = np.zeros((max_people, parts, 3), np.float32)
    ks = np.zeros(max_people, np.float32)
    n = ctypes.c_int()
    check(L.opk_assemble_people_semantics(kp.ctypes.data_as(ctypes.c_void_p),
                                          ks.ctypes.data_as(ctypes.c_void_p), max_people,
                                          ctypes.byref(n),
                                          pair_scores.ctypes.data_as(ctypes.c_void_p),
                                          peaks.ctypes.data_as(ctypes.c_void_p), pose_model,
                                          peaks.shape[1] - 1, min_subset_cnt, min_subset_score,
                                          scale, int(maximize_positives), semantics))
    k = min(n.value, max_people)
    return kp[:k].copy(), ks[:k].copy()


class Net:
    """op::NetCaffe replacement (NetHip): prototxt path or "builtin:BODY_25"."""

    def __init__(self, ctx, prototxt="builtin:BODY_25", caffemodel=None):
        self.ctx = ctx
        self.L = ctx.L
        h = ctypes.c_void_p()
        check(self.L.opk_net_create(ctx.h, prototxt.encode(),
                                    caffemodel.encode() if caffemodel else None, ctypes.byref(h)))
        self.h = h
        _LIVE["net"].add(self)

    def close(self):
        if self.h:
            self.L.opk_net_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def convs(self):
        """[{name, cin, num_output, kernel_size, act}] in execution order."""
        out = []
        name = ctypes.create_string_buffer(64)
        cin, cout, k, act = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        for i in range(self.L.opk_net_num_convs(self.h)):
            check(self.L.opk_net_conv_info(self.h, i, name, ctypes.byref(cin), ctypes.byref(cout),
                                           ctypes.byref(k), ctypes.byref(act)))
            out.append(dict(name=name.value.decode(), cin=cin.value, num_output=cout.value,
                            kernel_size=k.value, act=act.value))
        return out

    def set_params(self, params):
        """params: {conv name: (w [co,ci,k,k], bias [co], slope [co] | None)} fp32 numpy."""
        for c in self.convs():
            w, b, s = params[c["name"]]
            w = np.ascontiguousarray(w, np.float32)
            b = np.ascontiguousarray(b, np.float32)
            sp = None
            if s is not None:
                s = np.ascontiguousarray(s, np.float32)
                sp = s.ctypes.data_as(ctypes.c_void_p)
            check(self.L.opk_net_set_conv(self.h, c["name"].encode(),
                                          w.ctypes.data_as(ctypes.c_void_p),
                                          b.ctypes.data_as(ctypes.c_void_p), sp))

    def forward(self, x):
        """x: [n, 3, h, w] fp32 CUDA tensor. Returns (device pointer, shape) of net_output."""
        n, c, h, w = x.shape
        check(self.L.opk_net_forward(self.h, _ptr(x), n, h, w))
        return self.output()

    def load_caffemodel(self, path):
        """Trained weights (CopyTrainedLayersFrom semantics); returns the convs loaded."""
        n = ctypes.c_int()
        check(self.L.opk_net_load_caffemodel(self.h, path.encode(), ctypes.byref(n)))
        return n.value

    def set_precision(self, precision):
        """PRECISION_FP16 (default) or PRECISION_SPLIT (fp16 hi/lo pairs, ~fp32 results at ~3x
        the MFMA work; opk_net_set_precision)."""
        check(self.L.opk_net_set_precision(self.h, int(precision)))

    def set_timing(self, on=True):
        check(self.L.opk_net_set_timing(self.h, int(on)))

    def read_timing(self):
        """(forwards, summed device ms) since the last read (HIP events on the context stream)."""
        n, ms = ctypes.c_int(), ctypes.c_double()
        check(self.L.opk_net_read_timing(self.h, ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value

    def flops_per_frame(self, h, w):
        f = ctypes.c_double()
        check(self.L.opk_net_flops_per_frame(self.h, h, w, ctypes.byref(f)))
        return f.value

    def output(self):
        p = ctypes.c_void_p()
        shape = (ctypes.c_int * 4)()
        check(self.L.opk_net_output(self.h, ctypes.byref(p), shape))
        return p.value, tuple(shape)

    def output_numpy(self):
        p, shape = self.output()
        out = np.empty(shape, np.float32)
        check(self.L.opk_memcpy_d2h(self.ctx.h, out.ctypes.data_as(ctypes.c_void_p),
                                    ctypes.c_void_p(p), out.nbytes))
        return out

    def blob(self, name, frames=None):
        """Named top of the last forward (opk_net_blob) as fp32 NCHW numpy: frames = (first, count),
        default all.  Values are the fp16 activations the kernels stored (net_output: fp32)."""
        shape = (ctypes.c_int * 4)()
        f0, nf = frames if frames is not None else (0, self.output()[1][0])
        check(self.L.opk_net_blob(self.h, name.encode(), f0, nf, None, shape))
        out = np.empty(tuple(shape), np.float32)
        check(self.L.opk_net_blob(self.h, name.encode(), f0, nf,
                                  out.ctypes.data_as(ctypes.c_void_p), shape))
        return out

    def launch_log(self):
        """[(layer, kernel instantiation)] of the last forward run under dev_switches(LAUNCH_LOG=1)."""
        need = ctypes.c_size_t()
        check(self.L.opk_net_launch_log(self.h, None, 0, ctypes.byref(need)))
        buf = ctypes.create_string_buffer(need.value)
        check(self.L.opk_net_launch_log(self.h, buf, need.value, ctypes.byref(need)))
        return [tuple(line.split("\t", 1)) for line in buf.value.decode().splitlines()]


class PoseExtractor:
    """op::PoseExtractorCaffe replacement for batches of frames (PoseHip)."""

    def __init__(self, ctx, net=None, maximize_positives=False, pose_model=BODY_25,
                 semantics=CONNECT_CPU):
        self.ctx = ctx
        self.L = ctx.L
        h = ctypes.c_void_p()
        check(self.L.opk_pose_create_model(ctx.h, net.h if net is not None else None, pose_model,
                                           int(maximize_positives), semantics, ctypes.byref(h)))
        self.h = h
        _LIVE["pose"].add(self)
        self.net = net
        self.parts = pose_model_info(pose_model)["parts"]

    def close(self):
        if self.h:
            self.L.opk_pose_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_property(self, prop, value):
        check(self.L.opk_pose_set_property(self.h, prop, float(value)))

    def set_map_semantics(self, semantics):
        """MAPS_CPU (default) or MAPS_CUDA: the resize + NMS arithmetic of the reference's CPU or
        CUDA build (opk_pose_set_map_semantics)."""
        check(self.L.opk_pose_set_map_semantics(self.h, semantics))

    def set_upsampling_ratio(self, ratio):
        """--upsampling_ratio (PoseExtractorCaffe's upsamplingRatio): heat maps at
        round(out * ratio - 1) + 1 instead of the net input size; <= 0 restores the default."""
        check(self.L.opk_pose_set_upsampling_ratio(self.h, float(ratio)))

    def set_overlay(self, overlay):
        self._overlay = overlay   # keep the tensor alive
        check(self.L.opk_pose_set_overlay(self.h, _ptr(overlay) if overlay is not None else None))

    def forward(self, frames, producer_size):
        n, _, h, w = frames.shape
        check(self.L.opk_pose_forward(self.h, _ptr(frames), n, h, w, producer_size[0],
                                      producer_size[1]))

    def _multi(self, fn, frames, producer_size):
        n = frames[0].shape[0]
        ptrs = (ctypes.c_void_p * len(frames))(*[f.data_ptr() for f in frames])
        for f in frames:
            assert f.is_cuda and f.is_contiguous() and f.shape[0] == n
        hw = (ctypes.c_int * (2 * len(frames)))(*[v for f in frames for v in f.shape[2:]])
        check(fn(self.h, ptrs, hw, len(frames), n, producer_size[0], producer_size[1]))

    def forward_multi(self, frames, producer_size):
        """Multi-scale: frames = list of [n,3,h_i,w_i] net inputs, scale 0 first."""
        self._multi(self.L.opk_pose_forward_multi, frames, producer_size)

    def submit_multi(self, frames, producer_size):
        self._multi(self.L.opk_pose_submit_multi, frames, producer_size)

    def set_input(self, net_resolution=(-1, 368), dynamic_behavior=1.0, scale_number=1,
                  scale_gap=0.25):
        """--net_resolution, --net_resolution_dynamic, --scale_number, --scale_gap."""
        check(self.L.opk_pose_set_input(self.h, net_resolution[0], net_resolution[1],
                                        float(dynamic_behavior), scale_number, float(scale_gap)))

    def _frames(self, fn, frames):
        n, h, w, c = frames.shape
        assert c == 3 and frames.dtype == torch.uint8
        check(fn(self.h, _ptr(frames), n, w, h, w * 3))
        self._frames_n = n

    def forward_frames(self, frames):
        """Raw BGR uint8 frames [n, h, w, 3] (CUDA): GPU preprocessing + net + post-processing."""
        self._frames(self.L.opk_pose_forward_frames, frames)

    def submit_frames(self, frames):
        self._frames(self.L.opk_pose_submit_frames, frames)

    def net_input_numpy(self, scale=0):
        p = ctypes.c_void_p()
        w, h = ctypes.c_int(), ctypes.c_int()
        check(self.L.opk_pose_net_input(self.h, scale, ctypes.byref(p), ctypes.byref(w),
                                        ctypes.byref(h)))
        n = self._frames_n
        out = np.empty((n, 3, h.value, w.value), np.float32)
        check(self.L.opk_memcpy_d2h(self.ctx.h, out.ctypes.data_as(ctypes.c_void_p), p, out.nbytes))
        return out

    def forward_net_output(self, net_output, net_size, producer_size):
        """net_output: [n, heat_channels, h, w] CUDA tensor (or (ptr, shape)); net_size = (w, h)."""
        if isinstance(net_output, tuple):
            ptr, shape = net_output
            ptr = ctypes.c_void_p(ptr)
        else:
            ptr, shape = _ptr(net_output), net_output.shape
        check(self.L.opk_pose_forward_net_output(self.h, ptr, shape[0], shape[2], shape[3],
                                                 net_size[1], net_size[0], producer_size[0],
                                                 producer_size[1]))

    def submit(self, frames, producer_size):
        """Enqueue a batch's device work and return (pipelined use; see opk_pose_submit)."""
        n, _, h, w = frames.shape
        check(self.L.opk_pose_submit(self.h, _ptr(frames), n, h, w, producer_size[0],
                                     producer_size[1]))

    def submit_net_output(self, net_output, net_size, producer_size):
        if isinstance(net_output, tuple):
            ptr, shape = net_output
            ptr = ctypes.c_void_p(ptr)
        else:
            ptr, shape = _ptr(net_output), net_output.shape
        check(self.L.opk_pose_submit_net_output(self.h, ptr, shape[0], shape[2], shape[3],
                                                net_size[1], net_size[0], producer_size[0],
                                                producer_size[1]))

    def collect(self):
        """Wait for the oldest submitted batch, assemble its people; returns its frame count."""
        n = ctypes.c_int(0)
        check(self.L.opk_pose_collect(self.h, ctypes.byref(n)))
        return n.value

    def pending(self):
        return self.L.opk_pose_pending(self.h)

    def num_people(self, frame):
        return self.L.opk_pose_num_people(self.h, frame)

    def keypoints(self, frame):
        n = self.num_people(frame)
        kp = np.zeros((max(n, 1), self.parts, 3), np.float32)
        ks = np.zeros(max(n, 1), np.float32)
        check(self.L.opk_pose_keypoints(self.h, frame, kp.ctypes.data_as(ctypes.c_void_p),
                                        ks.ctypes.data_as(ctypes.c_void_p), n))
        return kp[:n], ks[:n]

    def set_timing(self, on=True):
        check(self.L.opk_pose_set_timing(self.h, int(on)))

    def read_timing(self):
        """(batches, summed post-processing device ms) since the last read."""
        n, ms = ctypes.c_int(0), ctypes.c_double(0)
        check(self.L.opk_pose_read_timing(self.h, ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value

    def read_collect_times(self):
        """{collects, wait_ms, assembly_ms, workers} of the collects since the last read (host
        time waiting for the device results vs assembling people; opk_pose_read_collect_times)."""
        n, w, a, k = ctypes.c_int(0), ctypes.c_double(0), ctypes.c_double(0), ctypes.c_int(0)
        check(self.L.opk_pose_read_collect_times(self.h, ctypes.byref(n), ctypes.byref(w),
                                                 ctypes.byref(a), ctypes.byref(k)))
        return {"collects": n.value, "wait_ms": w.value, "assembly_ms": a.value, "workers": k.value}

    def records(self, out=None):
        """Packed results of every frame of the last collected batch (opk_pose_records):
        per frame [people, keypoints (people x parts x 3), scores (people)], float32.  With `out`
        (a float32 numpy buffer) the records are written there; returns the filled view."""
        used = ctypes.c_size_t(0)
        check(self.L.opk_pose_records(self.h, None, 0, ctypes.byref(used)))
        if out is None:
            out = np.empty(used.value, np.float32)
        if out.size < used.value:
            raise ValueError("records buffer holds %d floats, %d needed" % (out.size, used.value))
        check(self.L.opk_pose_records(self.h, out.ctypes.data_as(ctypes.c_void_p), out.size,
                                      ctypes.byref(used)))
        return out[:used.value]

    def scale_net_to_output(self):
        return self.L.opk_pose_scale_net_to_output(self.h)

    def _dev_array(self, fn):
        p = ctypes.c_void_p()
        shape = (ctypes.c_int * 4)()
        check(fn(self.h, ctypes.byref(p), shape))
        out = np.empty(tuple(shape), np.float32)
        check(self.L.opk_memcpy_d2h(self.ctx.h, out.ctypes.data_as(ctypes.c_void_p), p, out.nbytes))
        return out

    def heatmaps_numpy(self):
        return self._dev_array(self.L.opk_pose_heatmaps)

    def heatmaps_copy(self, types=7, scale_mode=8):
        """getHeatMapsCopy for every frame of the last batch: [n, channels, H, W] float32 numpy
        (types bits: 1 parts, 2 background, 4 PAFs; scale_mode: op::ScaleMode value)."""
        shape = (ctypes.c_int * 4)()
        check(self.L.opk_pose_heatmaps_copy(self.h, types, scale_mode, None, shape))
        dev = torch.empty(tuple(shape), dtype=torch.float32, device="cuda")
        check(self.L.opk_pose_heatmaps_copy(self.h, types, scale_mode, _ptr(dev), shape))
        return dev.cpu().numpy()

    def candidates(self, frame):
        """getCandidatesCopy: list over parts of [count, 3] arrays (x, y output pixels, score)."""
        out = np.zeros((self.parts, 127, 3), np.float32)
        counts = np.zeros(self.parts, np.int32)
        check(self.L.opk_pose_candidates(self.h, frame, out.ctypes.data_as(ctypes.c_void_p),
                                         counts.ctypes.data_as(ctypes.POINTER(ctypes.c_int))))
        return [out[p, :counts[p]].copy() for p in range(self.parts)]

    def peaks_numpy(self):
        return self._dev_array(self.L.opk_pose_peaks)


# ---- face / hand keypoints ---------------------------------------------------------------------
FACE, HAND = 0, 1


def _detect(fn, pose_model, keypoints, per_person):
    kp = np.ascontiguousarray(keypoints, np.float32)
    people, parts = kp.shape[0], (kp.shape[1] if kp.ndim == 3 else 0)
    out = np.zeros((people, per_person, 4), np.float32)
    check(fn(pose_model, kp.ctypes.data_as(ctypes.c_void_p), people, parts,
             out.ctypes.data_as(ctypes.c_void_p)))
    return out


def detect_faces(pose_keypoints, pose_model=BODY_25):
    """op::FaceDetector(poseModel).detectFaces: [people, 4] (x, y, width, height)."""
    return _detect(_lib.load().opk_face_detect, pose_model, pose_keypoints, 1)[:, 0]


def detect_hands(pose_keypoints, pose_model=BODY_25):
    """op::HandDetector(poseModel).detectHands: [people, 2 (left, right), 4]."""
    return _detect(_lib.load().opk_hand_detect, pose_model, pose_keypoints, 2)


class KeypointExtractor:
    """op::FaceExtractorCaffe / op::HandExtractorCaffe over every rectangle of a set of frames:
    kind FACE (net builtin:FACE) or HAND (builtin:HAND); net_resolution = (w, h)."""

    def __init__(self, ctx, net, kind, net_resolution=(368, 368)):
        self.ctx = ctx
        self.L = ctx.L
        self.net = net
        self.kind = kind
        self.net_resolution = tuple(net_resolution)
        h = ctypes.c_void_p()
        check(self.L.opk_extractor_create(ctx.h, net.h, kind, net_resolution[0],
                                          net_resolution[1], ctypes.byref(h)))
        self.h = h
        _LIVE["extractor"].add(self)

    def close(self):
        if self.h:
            self.L.opk_extractor_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def parts(self):
        return self.L.opk_extractor_parts(self.h)

    def set_scales(self, number, rng=0.4):
        """--hand_scale_number / --hand_scale_range."""
        check(self.L.opk_extractor_set_scales(self.h, number, float(rng)))

    def set_max_batch(self, b):
        check(self.L.opk_extractor_set_max_batch(self.h, b))

    def set_heatmaps(self, scale_mode):
        """Per-person heat maps with op::ScaleMode scale_mode (-1 off; opk_extractor_set_heatmaps)."""
        check(self.L.opk_extractor_set_heatmaps(self.h, scale_mode))

    def heatmaps_numpy(self):
        """The last forward's heat maps: face [people, parts, H, W], hand [2, people, parts, H, W]."""
        p = ctypes.c_void_p()
        shape = (ctypes.c_int * 5)()
        check(self.L.opk_extractor_heatmaps(self.h, ctypes.byref(p), shape))
        dims = tuple(shape)
        out = np.zeros(dims, np.float32)
        if out.size:
            check(self.L.opk_memcpy_d2h(self.ctx.h, out.ctypes.data_as(ctypes.c_void_p), p,
                                        out.nbytes))
        return out[0] if self.kind == FACE else out

    def forward(self, frames, rectangles, frame_of=None):
        """frames: BGR uint8 [n, h, w, 3] CUDA tensor; rectangles [people, 4] (face) or
        [people, 2, 4] (hand); frame_of [people] or None.  Returns face [people, parts, 3] or
        hand [2, people, parts, 3] keypoints (numpy)."""
        n, h, w, c = frames.shape
        assert c == 3 and frames.dtype == torch.uint8
        r = np.ascontiguousarray(rectangles, np.float32)
        people = r.shape[0]
        hands = 2 if self.kind == HAND else 1
        out = np.zeros((hands, people, self.parts, 3), np.float32)
        fo = None
        if frame_of is not None:
            fo = np.ascontiguousarray(frame_of, np.int32)
            assert fo.shape == (people,)
        check(self.L.opk_extractor_forward(
            self.h, _ptr(frames), n, w, h, w * 3, r.ctypes.data_as(ctypes.c_void_p),
            fo.ctypes.data_as(ctypes.c_void_p) if fo is not None else None, people,
            out.ctypes.data_as(ctypes.c_void_p)))
        return out[0] if self.kind == FACE else out

    def crops(self):
        """[(2x3 inverse map, net input [3, h, w] numpy)] of the last forward's crops."""
        out = []
        w, h = self.net_resolution
        for i in range(self.L.opk_extractor_crop_count(self.h)):
            m = np.zeros(6, np.float64)
            p = ctypes.c_void_p()
            check(self.L.opk_extractor_crop(self.h, i, m.ctypes.data_as(ctypes.c_void_p),
                                            ctypes.byref(p)))
            x = np.empty((3, h, w), np.float32)
            check(self.L.opk_memcpy_d2h(self.ctx.h, x.ctypes.data_as(ctypes.c_void_p), p,
                                        x.nbytes))
            out.append((m.reshape(2, 3), x))
        return out
