"""The reference's other networks: COCO_18, MPI_15 (6 and 4 stages),
face and hand prototxts are read and planned by NetHip -- 7x7/pad 3 refinement stages on a 3-pixel
zero border, ReLU only, and (hand / face) a conv whose top is the output blob.  Host-only context:
no device work.  GPU numerics of the same layer kinds: tests/test_gpu_net.py (7x7 CPM graphs vs
the oracle)."""
import os

import pytest

from openpose_amd.api import Context, Net
from tests import prototxt

MODELS = "/root/reference/models"
CASES = {
    "coco": ("pose/coco/pose_deploy_linevec.prototxt", 57),
    "mpi": ("pose/mpi/pose_deploy_linevec.prototxt", 44),
    "mpi_4": ("pose/mpi/pose_deploy_linevec_faster_4_stages.prototxt", 44),
    "face": ("face/pose_deploy.prototxt", 71),
    "hand": ("hand/pose_deploy.prototxt", 22),
}


def _flops(layers, h, w):
    """2 * MACs of every conv of a parsed prototxt at input h x w (Caffe ceil pooling)."""
    size = {"image": (h, w)}
    chans = {"image": 3}
    total = 0.0
    for l in layers:
        t = l["type"]
        if t == "Convolution":
            hh, ww = size[l["bottom"][0]]
            total += 2.0 * hh * ww * l["num_output"] * chans[l["bottom"][0]] * l["kernel_size"] ** 2
            size[l["top"][0]] = (hh, ww)
            chans[l["top"][0]] = l["num_output"]
        elif t == "Pooling":
            hh, ww = size[l["bottom"][0]]
            size[l["top"][0]] = ((hh - 2 + 1) // 2 + 1, (ww - 2 + 1) // 2 + 1)
            chans[l["top"][0]] = chans[l["bottom"][0]]
        elif t == "Concat":
            size[l["top"][0]] = size[l["bottom"][0]]
            chans[l["top"][0]] = sum(chans[b] for b in l["bottom"])
    return total, chans["net_output"]


@pytest.mark.skipif(not os.path.isdir(MODELS), reason="no reference tree")
@pytest.mark.parametrize("name", sorted(CASES))
def test_reference_prototxt_plans(name):
    rel, out_c = CASES[name]
    path = os.path.join(MODELS, rel)
    layers = prototxt.parse(open(path).read())
    ctx = Context.host_only()
    net = Net(ctx, path)
    convs = net.convs()
    ref_convs = [l for l in layers if l["type"] == "Convolution"]
    assert [c["name"] for c in convs] == [l["name"] for l in ref_convs]
    assert [c["kernel_size"] for c in convs] == [l["kernel_size"] for l in ref_convs]
    assert sorted({c["kernel_size"] for c in convs}) == [1, 3, 7]
    flops, channels = _flops(layers, 368, 368)
    assert channels == out_c
    assert abs(net.flops_per_frame(368, 368) - flops) < 1e-6 * flops
    net.close()


BUILTIN = {"coco": "builtin:COCO_18", "mpi": "builtin:MPI_15", "mpi_4": "builtin:MPI_15_4",
           "face": "builtin:FACE", "hand": "builtin:HAND"}


@pytest.mark.skipif(not os.path.isdir(MODELS), reason="no reference tree")
@pytest.mark.parametrize("name", sorted(BUILTIN))
def test_builtin_graph_matches_reference_prototxt(name):
    """The generated graphs (usable where the reference tree is absent, e.g. on the GPU box) equal
    the reference prototxts conv by conv: name, input channels (hence the wiring of every concat),
    outputs, kernel, activation, and the FLOPs of a 368x368 frame."""
    ctx = Context.host_only()
    a = Net(ctx, BUILTIN[name]).convs()
    b = Net(ctx, os.path.join(MODELS, CASES[name][0])).convs()
    assert a == b
    fa = Net(ctx, BUILTIN[name]).flops_per_frame(368, 368)
    fb = Net(ctx, os.path.join(MODELS, CASES[name][0])).flops_per_frame(368, 368)
    assert fa == fb


def test_builtin_graphs_plan_everywhere():
    ctx = Context.host_only()
    for name, (_, out_c) in CASES.items():
        net = Net(ctx, BUILTIN[name])
        acts = {c["act"] for c in net.convs()}
        assert acts <= {0, 1}                      # ReLU nets (no PReLU)
        assert net.flops_per_frame(368, 368) > 0
    with pytest.raises(Exception):
        Net(ctx, "builtin:NOPE")


@pytest.mark.skipif(not os.path.isdir(MODELS), reason="no reference tree")
@pytest.mark.parametrize("name", sorted(BUILTIN))
def test_python_graph_helper_matches_reference(name):
    """tests/cpm_graphs.py (used by the GPU oracle comparisons) = the reference prototxt."""
    from tests import cpm_graphs
    mine = prototxt.parse(prototxt.emit(cpm_graphs.GRAPHS[BUILTIN[name]]()))
    ref = prototxt.parse(open(os.path.join(MODELS, CASES[name][0])).read())
    strip = lambda L: [(l["name"], l["type"], l["bottom"], l["top"], l.get("num_output"),
                        l.get("kernel_size"), l.get("pad")) for l in L if l["type"] != "ReLU"]
    assert strip(mine) == strip(ref)
    relu_of = lambda L: sorted(l["bottom"][0] for l in L if l["type"] == "ReLU")
    assert relu_of(mine) == relu_of(ref)
