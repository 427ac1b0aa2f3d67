"""Test helper: the reference's CPM networks (COCO_18, MPI_15, hand, face) as layer dicts, the
structure of models/*/pose_deploy*.prototxt (checked against those files where the reference tree
exists, tests/test_models.py), for oracle comparisons on the GPU box where it does not."""


def _conv(L, name, bottom, cout, k, relu=True, top=None):
    L.append(dict(name=name, type="Convolution", bottom=[bottom], top=[top or name],
                  num_output=cout, kernel_size=k, pad=k // 2))
    if relu:
        L.append(dict(name="relu_" + name, type="ReLU", bottom=[top or name], top=[top or name]))


def _vgg(L, pools):
    _conv(L, "conv1_1", "image", 64, 3)
    _conv(L, "conv1_2", "conv1_1", 64, 3)
    L.append(dict(name=pools[0], type="Pooling", bottom=["conv1_2"], top=[pools[0]], pool="MAX",
                  kernel_size=2, stride=2))
    _conv(L, "conv2_1", pools[0], 128, 3)
    _conv(L, "conv2_2", "conv2_1", 128, 3)
    L.append(dict(name=pools[1], type="Pooling", bottom=["conv2_2"], top=[pools[1]], pool="MAX",
                  kernel_size=2, stride=2))
    _conv(L, "conv3_1", pools[1], 256, 3)
    for j in (2, 3, 4):
        _conv(L, "conv3_%d" % j, "conv3_%d" % (j - 1), 256, 3)
    L.append(dict(name=pools[2], type="Pooling", bottom=["conv3_4"], top=[pools[2]], pool="MAX",
                  kernel_size=2, stride=2))
    _conv(L, "conv4_1", pools[2], 512, 3)
    _conv(L, "conv4_2", "conv4_1", 512, 3)


def pose_graph(pafs, heat, stages):
    L = []
    _vgg(L, ("pool1_stage1", "pool2_stage1", "pool3_stage1"))
    _conv(L, "conv4_3_CPM", "conv4_2", 256, 3)
    _conv(L, "conv4_4_CPM", "conv4_3_CPM", 128, 3)
    for j in range(1, 6):
        for b in ("L1", "L2"):
            src = "conv4_4_CPM" if j == 1 else "conv5_%d_CPM_%s" % (j - 1, b)
            cout = 128 if j <= 3 else (512 if j == 4 else (pafs if b == "L1" else heat))
            _conv(L, "conv5_%d_CPM_%s" % (j, b), src, cout, 3 if j <= 3 else 1, relu=j < 5)
    l1, l2 = "conv5_5_CPM_L1", "conv5_5_CPM_L2"
    for s in range(2, stages + 1):
        cat = "concat_stage%d" % s
        L.append(dict(name=cat, type="Concat", bottom=[l1, l2, "conv4_4_CPM"], top=[cat]))
        for j in range(1, 8):
            for b in ("L1", "L2"):
                src = cat if j == 1 else "Mconv%d_stage%d_%s" % (j - 1, s, b)
                cout = 128 if j <= 6 else (pafs if b == "L1" else heat)
                _conv(L, "Mconv%d_stage%d_%s" % (j, s, b), src, cout, 7 if j <= 5 else 1, relu=j < 7)
        l1, l2 = "Mconv7_stage%d_L1" % s, "Mconv7_stage%d_L2" % s
    L.append(dict(name="concat_stage7", type="Concat", bottom=[l2, l1], top=["net_output"]))
    return L


def single_graph(outputs, face):
    L = []
    _vgg(L, ("pool1", "pool2", "pool3") if face else ("pool1_stage1", "pool2_stage1", "pool3_stage1"))
    _conv(L, "conv4_3", "conv4_2", 512, 3)
    _conv(L, "conv4_4", "conv4_3", 512, 3)
    _conv(L, "conv5_1", "conv4_4", 512, 3)
    _conv(L, "conv5_2", "conv5_1", 512, 3)
    _conv(L, "conv5_3_CPM", "conv5_2", 128, 3)
    _conv(L, "conv6_1_CPM", "conv5_3_CPM", 512, 1)
    _conv(L, "conv6_2_CPM", "conv6_1_CPM", outputs, 1, relu=False)
    prev = "conv6_2_CPM"
    for s in range(2, 7):
        cat = ("features_in_stage_%d" % s) if face else ("concat_stage%d" % s)
        L.append(dict(name=cat, type="Concat", bottom=[prev, "conv5_3_CPM"], top=[cat]))
        for j in range(1, 8):
            src = cat if j == 1 else "Mconv%d_stage%d" % (j - 1, s)
            last = j == 7
            _conv(L, "Mconv%d_stage%d" % (j, s), src, 128 if j <= 6 else outputs,
                  7 if j <= 5 else 1, relu=not last, top="net_output" if last and s == 6 else None)
        prev = "Mconv7_stage%d" % s
    return L


GRAPHS = {
    "builtin:COCO_18": lambda: pose_graph(38, 19, 6),
    "builtin:MPI_15": lambda: pose_graph(28, 16, 6),
    "builtin:MPI_15_4": lambda: pose_graph(28, 16, 4),
    "builtin:HAND": lambda: single_graph(22, False),
    "builtin:FACE": lambda: single_graph(71, True),
}
