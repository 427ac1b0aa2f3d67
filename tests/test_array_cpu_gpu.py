"""op::ArrayCpuGpu on HIP memory (integration/arrayCpuGpuHip.cpp, replacing the Caffe-only
src/openpose/core/arrayCpuGpu.cpp): a driver built against the reference's own header
(include/openpose/core/arrayCpuGpu.hpp) checks the Blob / SyncedMemory contract -- host side here,
device transitions through libopk_hip on the GPU.  The driver is built where /root/reference exists
(build_array_driver(), also run by __graft_entry__.build()) and travels with the tree."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "_bin", "array_driver")


def build_array_driver():
    """Compile tests/_bin/array_driver (needs the reference headers and libopk_hip.so)."""
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    cmd = ["g++", "-std=c++14", "-O1", "-Wall", "-Wextra", "-Werror",
           "-I/root/reference/include", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "integration"),
           os.path.join(ROOT, "integration", "arrayCpuGpuHip.cpp"),
           os.path.join(ROOT, "tests", "array_driver.cpp"),
           "-L" + os.path.join(ROOT, "openpose_amd"), "-lopk_hip",
           "-Wl,-rpath,$ORIGIN/../../openpose_amd",
           # op::Array's members (core/array.cpp, OpenCV) back one constructor the driver never calls
           "-Wl,--unresolved-symbols=ignore-all", "-o", BIN]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return BIN


@pytest.mark.skipif(not os.path.isdir("/root/reference/include"), reason="no reference tree")
def test_array_cpu_gpu_host_contract():
    build_array_driver()
    r = subprocess.run([BIN, "cpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "cpu ok" in r.stdout, r.stderr + r.stdout


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(BIN), reason="driver not built (needs the reference headers)")
def test_array_cpu_gpu_device_contract():
    r = subprocess.run([BIN, "gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "gpu ok" in r.stdout, r.stderr + r.stdout
    r = subprocess.run([BIN, "cpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
