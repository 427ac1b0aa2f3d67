"""Test helper: writes caffe.NetParameter files in protobuf wire format (no protobuf dependency).

Field numbers are those of Caffe's caffe.proto (NetParameter.layer = 100, .layers (V1) = 2;
LayerParameter.name = 1, .type = 2, .blobs = 7; V1LayerParameter.name = 4, .type = 5 (enum),
.blobs = 6; BlobProto.num/channels/height/width = 1-4, .data = 5, .shape = 7, .double_data = 8;
BlobShape.dim = 1).  Used to build synthetic .caffemodel files for the loader tests -- the
trained pose_iter_584000.caffemodel is not available offline (models/getModels.sh).
"""
import struct

import numpy as np


def _varint(v):
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wire):
    return _varint((field << 3) | wire)


def _len(field, payload):
    return _key(field, 2) + _varint(len(payload)) + payload


def blob(arr, legacy=False, packed=True, double=False):
    a = np.asarray(arr)
    out = b""
    if legacy:   # (num, channels, height, width), right-aligned
        dims = (1,) * (4 - a.ndim) + tuple(a.shape)
        for f, d in zip((1, 2, 3, 4), dims):
            out += _key(f, 0) + _varint(d)
    else:
        out += _len(7, _len(1, b"".join(_varint(d) for d in a.shape)))
    flat = a.reshape(-1)
    if double:
        out += _len(8, flat.astype("<f8").tobytes())
    elif packed:
        out += _len(5, flat.astype("<f4").tobytes())
    else:
        out += b"".join(_key(5, 5) + struct.pack("<f", float(v)) for v in flat)
    return out


def layer(name, type_, blobs, v1=False):
    if v1:   # V1LayerParameter: name 4, type 5 (enum; CONVOLUTION = 4), blobs 6
        body = _len(4, name.encode()) + _key(5, 0) + _varint(4)
        body += b"".join(_len(6, b) for b in blobs)
        return _len(2, body)
    body = _len(1, name.encode()) + _len(2, type_.encode())
    body += _key(10, 0) + _varint(1)                 # an unrelated field (phase-like) to skip
    body += b"".join(_len(7, b) for b in blobs)
    return _len(100, body)


def net(layers, name="synthetic"):
    return _len(1, name.encode()) + b"".join(layers)


def body25_caffemodel(params, graph):
    """A BODY_25 .caffemodel from {conv: (w, b, slope|None)} and the prototxt layer list."""
    act = {}
    for l in graph:
        if l["type"] in ("ReLU", "PReLU"):
            act[l["bottom"][0]] = l["name"]
    parts = []
    for l in graph:
        if l["type"] != "Convolution":
            continue
        w, b, s = params[l["name"]]
        parts.append(layer(l["name"], "Convolution", [blob(w), blob(b)]))
        if s is not None:
            parts.append(layer(act[l["top"][0]], "PReLU", [blob(s)]))
    return net(parts, "BODY_25")
