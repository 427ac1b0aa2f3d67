"""ctypes binding of libopk_hip.so (C-ABI: include/opk.h).

The library is REQUIRED: importing the product API without it raises -- there is no CPU or
PyTorch fallback anywhere in the product path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libopk_hip.so")
if os.environ.get("OPK_LIB_PATH"):   # dev A/B of two builds in one process tree
    LIB_PATH = os.environ["OPK_LIB_PATH"]

_c = ctypes
_p = _c.c_void_p
_i = _c.c_int
_f = _c.c_float
_d = _c.c_double
_ip = _c.POINTER(_c.c_int)
_fp = _c.POINTER(_c.c_float)

# name: (restype, argtypes)
_SIGS = {
    "opk_last_error": (_c.c_char_p, []),
    "opk_version": (_i, []),
    "opk_dev_set": (_i, [_c.c_char_p, _i, _i]),
    "opk_ctx_create": (_i, [_i, _p, _c.POINTER(_p)]),
    "opk_ctx_create_private_stream": (_i, [_i, _c.POINTER(_p)]),
    "opk_ctx_destroy": (_i, [_p]),
    "opk_ctx_stream": (_i, [_p, _c.POINTER(_p)]),
    "opk_sync": (_i, [_p]),
    "opk_malloc": (_i, [_p, _c.POINTER(_p), _c.c_size_t]),
    "opk_free": (_i, [_p, _p]),
    "opk_memset": (_i, [_p, _p, _i, _c.c_size_t]),
    "opk_convert": (_i, [_p, _p, _i, _p, _i, _c.c_size_t]),
    "opk_memcpy_h2d": (_i, [_p, _p, _p, _c.c_size_t]),
    "opk_memcpy_d2h": (_i, [_p, _p, _p, _c.c_size_t]),
    "opk_probe_peaks": (_i, [_p, _c.POINTER(_d), _c.POINTER(_d), _c.POINTER(_d)]),
    "opk_render_pose_keypoints": (_i, [_p, _p, _i, _i, _c.c_uint, _c.c_uint, _p, _f, _i, _i, _f]),
    "opk_render_face_keypoints": (_i, [_p, _p, _c.c_uint, _c.c_uint, _p, _i, _f, _f]),
    "opk_render_hand_keypoints": (_i, [_p, _p, _c.c_uint, _c.c_uint, _p, _i, _f, _f]),
    "opk_render_pose_heat_map": (_i, [_p, _p, _c.c_uint, _c.c_uint, _p, _i, _i, _f, _c.c_uint, _f]),
    "opk_render_pose_heat_maps": (_i, [_p, _p, _i, _c.c_uint, _c.c_uint, _p, _i, _i, _f, _f]),
    "opk_render_pose_paf": (_i, [_p, _p, _i, _c.c_uint, _c.c_uint, _p, _i, _i, _f, _i, _f]),
    "opk_render_pose_pafs": (_i, [_p, _p, _i, _c.c_uint, _c.c_uint, _p, _i, _i, _f, _f]),
    "opk_render_pose_distance": (_i, [_p, _p, _c.c_uint, _c.c_uint, _p, _i, _i, _f, _c.c_uint, _f]),
    "opk_resize_and_merge": (_i, [_p, _p, _c.POINTER(_p), _i, _ip, _ip, _fp]),
    "opk_nms": (_i, [_p, _p, _p, _p, _f, _ip, _ip, _f, _f]),
    "opk_nms_semantics": (_i, [_p, _p, _p, _p, _f, _ip, _ip, _f, _f, _i]),
    "opk_pose_set_map_semantics": (_i, [_p, _i]),
    "opk_resize_and_merge_semantics": (_i, [_p, _p, _c.POINTER(_p), _i, _ip, _ip, _fp, _i]),
    "opk_paf_scores": (_i, [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _f, _f, _f]),
    "opk_connect_body_parts": (_i, [_p, _p, _p, _i, _ip, _p, _p, _i, _i, _i, _i, _i, _f, _f, _i,
                                    _f, _f, _f, _i]),
    "opk_assemble_people": (_i, [_p, _p, _i, _ip, _p, _p, _i, _i, _i, _f, _f, _i]),
    "opk_connect_body_parts_semantics": (_i, [_p, _p, _p, _i, _ip, _p, _p, _i, _i, _i, _i, _i, _f,
                                              _f, _i, _f, _f, _f, _i, _i]),
    "opk_assemble_people_semantics": (_i, [_p, _p, _i, _ip, _p, _p, _i, _i, _i, _f, _f, _i, _i]),
    "opk_pose_model_info": (_i, [_i, _ip, _ip, _ip, _ip, _p, _p]),
    "opk_pose_default_thresholds": (_i, [_i, _i, _fp, _fp]),
    "opk_net_create": (_i, [_p, _c.c_char_p, _c.c_char_p, _c.POINTER(_p)]),
    "opk_net_destroy": (_i, [_p]),
    "opk_net_num_convs": (_i, [_p]),
    "opk_net_conv_info": (_i, [_p, _i, _c.c_char_p, _ip, _ip, _ip, _ip]),
    "opk_net_set_conv": (_i, [_p, _c.c_char_p, _p, _p, _p]),
    "opk_net_forward": (_i, [_p, _p, _i, _i, _i]),
    "opk_net_flops_per_frame": (_i, [_p, _i, _i, _c.POINTER(_d)]),
    "opk_net_output": (_i, [_p, _c.POINTER(_p), _ip]),
    "opk_net_blob": (_i, [_p, _c.c_char_p, _i, _i, _p, _ip]),
    "opk_net_launch_log": (_i, [_p, _c.c_char_p, _c.c_size_t, _c.POINTER(_c.c_size_t)]),
    "opk_pose_create": (_i, [_p, _p, _i, _c.POINTER(_p)]),
    "opk_pose_create_model": (_i, [_p, _p, _i, _i, _i, _c.POINTER(_p)]),
    "opk_pose_destroy": (_i, [_p]),
    "opk_pose_set_property": (_i, [_p, _i, _d]),
    "opk_pose_forward": (_i, [_p, _p, _i, _i, _i, _i, _i]),
    "opk_pose_forward_net_output": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _i]),
    "opk_pose_set_upsampling_ratio": (_i, [_p, _f]),
    "opk_pose_heatmap_size": (_i, [_p, _ip]),
    "opk_pose_set_overlay": (_i, [_p, _p]),
    "opk_pose_submit": (_i, [_p, _p, _i, _i, _i, _i, _i]),
    "opk_pose_submit_net_output": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _i]),
    "opk_pose_collect": (_i, [_p, _ip]),
    "opk_pose_submit_multi": (_i, [_p, _c.POINTER(_p), _ip, _i, _i, _i, _i]),
    "opk_pose_forward_multi": (_i, [_p, _c.POINTER(_p), _ip, _i, _i, _i, _i]),
    "opk_pose_pending": (_i, [_p]),
    "opk_pose_num_people": (_i, [_p, _i]),
    "opk_pose_keypoints": (_i, [_p, _i, _p, _p, _i]),
    "opk_pose_set_timing": (_i, [_p, _i]),
    "opk_pose_read_timing": (_i, [_p, _ip, _c.POINTER(_d)]),
    "opk_pose_read_collect_times": (_i, [_p, _ip, _c.POINTER(_d), _c.POINTER(_d), _ip]),
    "opk_net_set_precision": (_i, [_p, _i]),
    "opk_pose_records": (_i, [_p, _p, _c.c_size_t, _c.POINTER(_c.c_size_t)]),
    "opk_pose_heatmaps": (_i, [_p, _c.POINTER(_p), _ip]),
    "opk_pose_peaks": (_i, [_p, _c.POINTER(_p), _ip]),
    "opk_pose_scale_net_to_output": (_f, [_p]),
    "opk_net_load_caffemodel": (_i, [_p, _c.c_char_p, _ip]),
    "opk_caffemodel_blob": (_i, [_c.c_char_p, _c.c_char_p, _i, _p, _c.c_size_t, _p, _ip]),
    "opk_net_set_timing": (_i, [_p, _i]),
    "opk_net_read_timing": (_i, [_p, _ip, _c.POINTER(_d)]),
    "opk_pose_heatmaps_copy": (_i, [_p, _i, _i, _p, _ip]),
    "opk_pose_candidates": (_i, [_p, _i, _p, _ip]),
    "opk_scale_keypoints": (_i, [_p, _i, _i, _i, _d, _d, _i, _i]),
    "opk_keep_top_n_people": (_i, [_p, _i, _i, _p, _i, _p, _p, _ip]),
    "opk_people_json": (_i, [_p, _i, _p, _p, _i, _i, _p, ctypes.c_size_t, _p]),
    "opk_save_people_json": (_i, [ctypes.c_char_p, _p, _i, _p, _p, _i, _i]),
    "opk_face_detect": (_i, [_i, _p, _i, _i, _p]),
    "opk_hand_detect": (_i, [_i, _p, _i, _i, _p]),
    "opk_extractor_create": (_i, [_p, _p, _i, _i, _i, _c.POINTER(_p)]),
    "opk_extractor_destroy": (_i, [_p]),
    "opk_extractor_set_scales": (_i, [_p, _i, _f]),
    "opk_extractor_set_max_batch": (_i, [_p, _i]),
    "opk_extractor_set_heatmaps": (_i, [_p, _i]),
    "opk_extractor_heatmaps": (_i, [_p, _p, _ip]),
    "opk_extractor_parts": (_i, [_p]),
    "opk_extractor_forward": (_i, [_p, _p, _i, _i, _i, _c.c_size_t, _p, _p, _i, _p]),
    "opk_extractor_crop_count": (_i, [_p]),
    "opk_extractor_crop": (_i, [_p, _i, _p, _c.POINTER(_p)]),
    "opk_scale_and_size": (_i, [_i, _i, _i, _i, _f, _i, _d, _c.POINTER(_d), _ip]),
    "opk_cvmat_to_input": (_i, [_p, _p, _p, _i, _i, _i, _c.c_size_t, _d, _i, _i, _i]),
    "opk_pose_set_input": (_i, [_p, _i, _i, _f, _i, _d]),
    "opk_pose_submit_frames": (_i, [_p, _p, _i, _i, _i, _c.c_size_t]),
    "opk_pose_forward_frames": (_i, [_p, _p, _i, _i, _i, _c.c_size_t]),
    "opk_pose_net_input": (_i, [_p, _i, _c.POINTER(_p), _ip, _ip]),
}

_LIB = None


class OpkError(RuntimeError):
    pass


def load():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise OpkError("libopk_hip.so not built (run `python -m openpose_amd.build`); the "
                           "product has no fallback path")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name, None)
            if fn is None:       # reported by tests/test_abi.py::test_exports_every_symbol
                continue
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def exported_symbols():
    return list(_SIGS)


def check(rc):
    if rc != 0:
        raise OpkError("opk error %d: %s" % (rc, load().opk_last_error().decode()))
    return rc


def int4(v):
    return (ctypes.c_int * 4)(*[int(x) for x in v])
