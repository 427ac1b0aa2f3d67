"""CPU: the C-ABI library (loads, exports every symbol of include/opk.h, host-only entry points) and
the BODY_25 graph (product builtin == oracle restatement == the reference prototxt when present)."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

from oracle import body25
from openpose_amd import _lib
from openpose_amd.api import Context, Net
from tests import prototxt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_PROTO = "/root/reference/models/pose/body_25/pose_deploy.prototxt"


def header_functions():
    text = open(os.path.join(ROOT, "include", "opk.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(opk_\w+)\s*\(", text, re.M)))


def test_library_exports_every_header_symbol():
    fns = header_functions()
    assert len(fns) > 30
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (opk_\w+)", out))
    missing = [f for f in fns if f not in exported]
    assert not missing, missing
    assert set(_lib.exported_symbols()) == set(fns), "ctypes table out of sync with opk.h"


def test_library_loads_and_reports_errors():
    L = _lib.load()
    assert L.opk_version() == 1
    h = ctypes.c_void_p()
    rc = L.opk_net_create(None, b"builtin:BODY_25", None, ctypes.byref(h))
    assert rc == 1 and b"NULL" in L.opk_last_error()


def test_gpu_kernels_are_gfx950_code_objects(tmp_path):
    # llvm-objdump --offloading extracts the bundles next to its input: run it on a copy
    lib = tmp_path / "libopk_hip.so"
    shutil.copy(_lib.LIB_PATH, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True)
    text = out.stdout + out.stderr
    assert "gfx950" in text


def _convs_of(layers):
    return [(l["name"], l["cin"], l["num_output"], l["kernel_size"]) for l in layers
            if l["type"] == "Convolution"]


def test_builtin_graph_matches_oracle_restatement():
    ctx = Context.host_only()
    net = Net(ctx, "builtin:BODY_25")
    got = [(c["name"], c["cin"], c["num_output"], c["kernel_size"]) for c in net.convs()]
    assert got == _convs_of(body25.layers())
    assert len(got) == 114
    assert abs(net.flops_per_frame(368, 656) / 1e9 - 287.26) < 0.01
    assert abs(net.flops_per_frame(368, 368) / 1e9 - 161.15) < 0.01


@pytest.mark.skipif(not os.path.exists(REF_PROTO), reason="no reference tree")
def test_builtin_graph_matches_reference_prototxt():
    ref = prototxt.parse(open(REF_PROTO).read())
    mine = body25.layers()
    assert len(ref) == len(mine) == 261
    for a, b in zip(ref, mine):
        for k in ("name", "type", "bottom", "top", "num_output", "kernel_size", "pad", "stride",
                  "cin"):
            if k in a or k in b:
                assert a.get(k) == b.get(k), (a["name"], k, a.get(k), b.get(k))
    # and the product's own prototxt reader agrees with its builtin graph
    ctx = Context.host_only()
    assert Net(ctx, REF_PROTO).convs() == Net(ctx, "builtin:BODY_25").convs()


def test_unsupported_layers_are_rejected():
    ctx = Context.host_only()
    bad = prototxt.emit([dict(name="c", type="Convolution", bottom=["image"], top=["c"],
                              num_output=8, kernel_size=5, pad=2)]) + \
        'layer { name: "net_output" type: "Concat" bottom: "c" top: "net_output" }\n'
    path = os.path.join(ROOT, "tests", "_bad.prototxt")
    open(path, "w").write(bad)
    try:
        with pytest.raises(_lib.OpkError, match="3x3/pad 1, 7x7/pad 3 and 1x1"):
            Net(ctx, path)
    finally:
        os.unlink(path)


def test_net_output_is_queryable_before_any_forward():
    """NetCaffe::getOutputBlobArray is called once right after initialization, before any forward
    (poseExtractorCaffe.cpp:94-95): opk_net_output answers then, with no device work."""
    ctx = Context.host_only()
    net = Net(ctx, "builtin:BODY_25")
    assert net.output() == (None, (0, 78, 0, 0))
    hand = Net(ctx, "builtin:HAND")
    assert hand.output() == (None, (0, 22, 0, 0))
