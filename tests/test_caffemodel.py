"""Caffe weight files (.caffemodel): the reader behind opk_net_create(..., caffemodel) (SURVEY.md
§8(f) row 2; the reference loads them with caffe::Net::CopyTrainedLayersFrom, netCaffe.cpp:165).

The trained pose_iter_584000.caffemodel cannot be downloaded here, so files are synthesised with
tests/caffemodel_writer.py in Caffe's wire format: new-style and V1 layers, packed and unpacked
floats, double data, legacy 4-D shapes, unrelated fields.  GPU: a net loaded from a synthetic
BODY_25 caffemodel computes exactly what the same weights set through opk_net_set_conv compute.
"""
import numpy as np
import pytest

from openpose_amd import api
from openpose_amd._lib import OpkError
from tests import caffemodel_writer as cw


def test_reader_formats(tmp_path):
    rng = np.random.default_rng(0)
    w = rng.standard_normal((4, 3, 3, 3)).astype(np.float32)
    b = rng.standard_normal(4).astype(np.float32)
    s = rng.standard_normal(4).astype(np.float32)
    d = rng.standard_normal((2, 5)).astype(np.float64)
    data = cw.net([
        cw.layer("data", "Input", []),                                    # no blobs: skipped
        cw.layer("conv_a", "Convolution", [cw.blob(w), cw.blob(b)]),
        cw.layer("prelu_a", "PReLU", [cw.blob(s, packed=False)]),
        cw.layer("conv_v1", None, [cw.blob(w, legacy=True), cw.blob(b, legacy=True)], v1=True),
        cw.layer("dbl", "InnerProduct", [cw.blob(d, double=True)]),
    ])
    p = tmp_path / "m.caffemodel"
    p.write_bytes(data)
    shape, got = api.caffemodel_blob(str(p), "conv_a", 0)
    assert shape == (4, 3, 3, 3) and np.array_equal(got, w)
    assert np.array_equal(api.caffemodel_blob(str(p), "conv_a", 1)[1], b)
    assert np.array_equal(api.caffemodel_blob(str(p), "prelu_a", 0)[1], s)
    shape, got = api.caffemodel_blob(str(p), "conv_v1", 1)
    assert shape == (1, 1, 1, 4) and np.array_equal(got.reshape(-1), b)   # legacy dims as stored
    assert np.array_equal(api.caffemodel_blob(str(p), "conv_v1", 0)[1].reshape(w.shape), w)
    assert np.array_equal(api.caffemodel_blob(str(p), "dbl", 0)[1], d.astype(np.float32))
    with pytest.raises(OpkError):
        api.caffemodel_blob(str(p), "data", 0)
    with pytest.raises(OpkError):
        api.caffemodel_blob(str(p), "conv_a", 2)


def test_reader_rejects_malformed(tmp_path):
    w = np.ones((2, 2), np.float32)
    good = cw.net([cw.layer("x", "Convolution", [cw.blob(w)])])
    p = tmp_path / "t.caffemodel"
    for bad in (good[:-3], good[:10], good + b"\x0b"):   # truncated; dangling key; bad wire type
        p.write_bytes(bad)
        with pytest.raises(OpkError):
            api.caffemodel_blob(str(p), "x", 0)
    # data count differing from the shape
    p.write_bytes(cw.net([cw.layer("x", "Convolution",
                                   [cw._len(7, cw._len(1, cw._varint(3))) + cw._len(5, b"\0" * 8)])]))
    with pytest.raises(OpkError):
        api.caffemodel_blob(str(p), "x", 0)
    with pytest.raises(OpkError):
        api.caffemodel_blob(str(tmp_path / "missing.caffemodel"), "x", 0)


@pytest.fixture(scope="module")
def body25_model(tmp_path_factory):
    from oracle import body25
    from openpose_amd import synth
    graph = body25.layers()
    params = synth.he_weights(graph, seed=3, out_scale=0.02)
    p = tmp_path_factory.mktemp("cm") / "pose_iter_synthetic.caffemodel"
    p.write_bytes(cw.body25_caffemodel(params, graph))
    return str(p), params, graph


def test_body25_caffemodel_blobs(body25_model):
    path, params, _ = body25_model
    for name in ("conv1_1", "Mconv7_stage1_L2", "Mconv3_stage0_L2_2"):
        w, b, _ = params[name]
        assert np.array_equal(api.caffemodel_blob(path, name, 0)[1], w)
        assert np.array_equal(api.caffemodel_blob(path, name, 1)[1], b)
    assert np.array_equal(api.caffemodel_blob(path, "Mprelu1_stage0_L2_0", 0)[1],
                          params["Mconv1_stage0_L2_0"][2])


@pytest.mark.gpu
def test_gpu_net_from_caffemodel_bitexact(ctx, body25_model, tmp_path):
    import torch
    path, params, graph = body25_model
    x = torch.from_numpy(np.random.default_rng(4).uniform(-0.5, 0.5, (2, 3, 64, 96))
                         .astype(np.float32)).cuda()
    a = api.Net(ctx, "builtin:BODY_25", caffemodel=path)
    a.forward(x)
    got = a.output_numpy()
    b = api.Net(ctx, "builtin:BODY_25")
    b.set_params(params)
    b.forward(x)
    np.testing.assert_array_equal(got, b.output_numpy())
    # a second file overriding one conv: only that layer changes (CopyTrainedLayersFrom by name)
    w, bias, s = params["Mconv7_stage1_L1"]
    p2 = tmp_path / "one.caffemodel"
    p2.write_bytes(cw.net([cw.layer("Mconv7_stage1_L1", "Convolution",
                                    [cw.blob(w * 2), cw.blob(bias)]),
                           cw.layer("not_in_net", "Convolution", [cw.blob(w)])]))
    assert a.load_caffemodel(str(p2)) == 1
    # shape mismatch: Caffe's "Cannot copy param" error
    p2.write_bytes(cw.net([cw.layer("conv1_1", "Convolution",
                                    [cw.blob(np.zeros((64, 3, 3, 2), np.float32)),
                                     cw.blob(np.zeros(64, np.float32))])]))
    with pytest.raises(OpkError, match="shape mismatch"):
        a.load_caffemodel(str(p2))
    # a PReLU conv without its slopes
    w1, b1, _ = params["Mconv1_stage0_L2_0"]
    p2.write_bytes(cw.net([cw.layer("Mconv1_stage0_L2_0", "Convolution", [cw.blob(w1), cw.blob(b1)])]))
    with pytest.raises(OpkError, match="PReLU"):
        a.load_caffemodel(str(p2))
