"""BODY_25 network graph + fp32 CPU forward (TEST INFRASTRUCTURE / CPU baseline; see oracle.h).

``layers()`` restates models/pose/body_25/pose_deploy.prototxt (261 layers) as a list of dicts,
independently of the product's C++ graph builder; tests check both against the prototxt text when
/root/reference is present.  ``forward()`` runs them with the Caffe-semantics C kernels of
oracle/caffe_cpu.c (the CPU restatement of op::NetCaffe::forwardPass, netCaffe.cpp:212-261).
"""
import numpy as np

from . import conv2d, prelu, relu, maxpool


def layers():
    L = []

    def conv(name, bottom, cout, k, act=None):
        L.append(dict(name=name, type="Convolution", bottom=[bottom], top=[name], num_output=cout,
                      kernel_size=k, pad=1 if k == 3 else 0))
        if act == "relu":
            L.append(dict(name="relu" + name[4:], type="ReLU", bottom=[name], top=[name]))
        elif act is not None:
            L.append(dict(name=act, type="PReLU", bottom=[name], top=[name]))

    def pool(name, bottom):
        L.append(dict(name=name, type="Pooling", bottom=[bottom], top=[name], kernel_size=2,
                      stride=2))

    def concat(name, bottoms):
        L.append(dict(name=name, type="Concat", bottom=list(bottoms), top=[name]))

    conv("conv1_1", "image", 64, 3, "relu")
    conv("conv1_2", "conv1_1", 64, 3, "relu")
    pool("pool1_stage1", "conv1_2")
    conv("conv2_1", "pool1_stage1", 128, 3, "relu")
    conv("conv2_2", "conv2_1", 128, 3, "relu")
    pool("pool2_stage1", "conv2_2")
    conv("conv3_1", "pool2_stage1", 256, 3, "relu")
    conv("conv3_2", "conv3_1", 256, 3, "relu")
    conv("conv3_3", "conv3_2", 256, 3, "relu")
    conv("conv3_4", "conv3_3", 256, 3, "relu")
    pool("pool3_stage1", "conv3_4")
    conv("conv4_1", "pool3_stage1", 512, 3, "relu")
    conv("conv4_2", "conv4_1", 512, 3, "prelu4_2")
    conv("conv4_3_CPM", "conv4_2", 256, 3, "prelu4_3_CPM")
    conv("conv4_4_CPM", "conv4_3_CPM", 128, 3, "prelu4_4_CPM")

    def stage(tag, inp, width, ch6, cout):
        x = inp
        for b in range(1, 6):
            names = []
            for j in range(3):
                nm = "Mconv%d_%s_%d" % (b, tag, j)
                conv(nm, x if j == 0 else names[-1], width, 3, "Mprelu%d_%s_%d" % (b, tag, j))
                names.append(nm)
            x = "Mconv%d_%s_concat" % (b, tag)
            concat(x, names)
        conv("Mconv6_%s" % tag, x, ch6, 1, "Mprelu6_%s" % tag)
        conv("Mconv7_%s" % tag, "Mconv6_%s" % tag, cout, 1)
        return "Mconv7_%s" % tag

    paf = stage("stage0_L2", "conv4_4_CPM", 96, 256, 52)
    for s in (1, 2, 3):
        concat("concat_stage%d_L2" % s, ["conv4_4_CPM", paf])
        paf = stage("stage%d_L2" % s, "concat_stage%d_L2" % s, 128, 512, 52)
    concat("concat_stage0_L1", ["conv4_4_CPM", paf])
    hm = stage("stage0_L1", "concat_stage0_L1", 96, 256, 26)
    concat("concat_stage1_L1", ["conv4_4_CPM", hm, paf])
    hm = stage("stage1_L1", "concat_stage1_L1", 128, 512, 26)
    concat("net_output", [hm, paf])
    # input channels of every conv
    chans = {"image": 3}
    for l in L:
        if l["type"] == "Convolution":
            l["cin"] = chans[l["bottom"][0]]
            chans[l["top"][0]] = l["num_output"]
        elif l["type"] == "Pooling":
            chans[l["top"][0]] = chans[l["bottom"][0]]
        elif l["type"] == "Concat":
            chans[l["top"][0]] = sum(chans[b] for b in l["bottom"])
    return L


def forward(x, params, graph=None, nthreads=None, stop_at=None):
    """fp32 CPU forward of the BODY_25 graph. x: [n, 3, h, w] -> net_output [n, 78, h/8, w/8].

    params: {conv name: (w, b, slope|None)}.  Returns the blob dict if ``stop_at`` is "all".
    """
    graph = graph or layers()
    blobs = {"image": np.ascontiguousarray(x, np.float32)}
    for l in graph:
        t = l["type"]
        if t == "Convolution":
            w, b, _ = params[l["name"]]
            blobs[l["top"][0]] = conv2d(blobs[l["bottom"][0]], w, b, l["pad"], nthreads)
        elif t == "ReLU":
            relu(blobs[l["top"][0]])
        elif t == "PReLU":
            conv_name = l["bottom"][0]
            prelu(blobs[l["top"][0]], params[conv_name][2])
        elif t == "Pooling":
            blobs[l["top"][0]] = maxpool(blobs[l["bottom"][0]], l["kernel_size"], l["stride"])
        elif t == "Concat":
            blobs[l["top"][0]] = np.concatenate([blobs[b] for b in l["bottom"]], axis=1)
        if stop_at is not None and l["top"][0] == stop_at:
            return blobs[stop_at]
    if stop_at == "all":
        return blobs
    return blobs["net_output"]
