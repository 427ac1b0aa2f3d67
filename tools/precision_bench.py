"""dev: CNN forward time of BODY_25 at the bench geometry in fp16 and split precision (HIP events
around each forward, opk_net_set_timing), and the net output's distance between the two.

    python tools/precision_bench.py [frames]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from openpose_amd import synth
    from openpose_amd.api import PRECISION_FP16, PRECISION_SPLIT, Context, Net
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 130
    ctx = Context(0)
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(synth.he_weights(net.convs(), seed=0, out_scale=1.0))
    x = torch.from_numpy(np.random.default_rng(1).uniform(-0.5, 0.5, (n, 3, 368, 656)).astype(np.float32)).cuda()
    res = {"frames": n}
    outs = {}
    for name, prec in (("fp16", PRECISION_FP16), ("split", PRECISION_SPLIT)):
        net.set_precision(prec)
        for _ in range(2):
            net.forward(x)
        torch.cuda.synchronize()
        net.set_timing(True)
        for _ in range(5):
            net.forward(x)
        k, ms = net.read_timing()
        net.set_timing(False)
        res[name + "_ms_per_forward"] = round(ms / k, 3)
        res[name + "_tflops"] = round(net.flops_per_frame(368, 656) * n / (ms / k * 1e-3) / 1e12, 1)
        outs[name] = net.output_numpy()[:2]
    res["split_over_fp16_time"] = round(res["split_ms_per_forward"] / res["fp16_ms_per_forward"], 3)
    a, b = outs["fp16"], outs["split"]
    res["fp16_vs_split_rel_l2"] = float(np.linalg.norm(a - b) / np.linalg.norm(b))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
