"""openpose_amd -- MI355X-native OpenPose BODY_25 hot path (CNN forward, resizeAndMerge, NMS,
bodyPartConnector) behind the reference's plugin surface.

The product is ``libopk_hip.so`` (HIP kernels for gfx950 + C++ host, C-ABI in include/opk.h).
This Python package is a thin ctypes front end used by the tests and bench.py.
"""
from .pose_tables import *  # noqa: F401,F403
