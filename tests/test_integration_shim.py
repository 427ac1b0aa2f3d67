"""CPU: the drop-in shim (integration/openpose_hip_shim.cpp) compiles against the reference's own
headers -- i.e. it defines resizeAndMergeGpu / nmsGpu / connectBodyPartsGpu with the exact
reference signatures and an op::Net subclass.  Skipped where /root/reference is absent."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.isdir("/root/reference/include"), reason="no reference tree")
@pytest.mark.parametrize("maps", ["", "-DOPK_SHIM_MAPS=OPK_MAPS_CPU"])
def test_shim_compiles_against_reference_headers(maps):
    """Default: the replaced *Gpu symbols keep the CUDA build's map semantics; -DOPK_SHIM_MAPS=
    OPK_MAPS_CPU selects the CPU path's."""
    r = subprocess.run(["g++", "-std=c++14", "-fsyntax-only", "-Wall", "-Wextra", "-Werror"] +
                       ([maps] if maps else []) +
                       ["-I/root/reference/include", "-I" + os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "integration", "openpose_hip_shim.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
