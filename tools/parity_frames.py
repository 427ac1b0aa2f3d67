"""Keypoint parity of the GPU pipeline (fp16 and split precision) against the fp32 CPU path on N
frames of the bench geometry -- the bench's `parity` block (bench.gpu_parity_run / cpu_parity) on
a larger sample than its 3 frames:

    python tools/parity_frames.py [N] > parity_N.json
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    from openpose_amd.api import PRECISION_FP16, PRECISION_SPLIT, Context, Net, PoseExtractor
    bench.PARITY_FRAMES = n
    ctx = Context(0)
    net = Net(ctx, "builtin:BODY_25")
    convs = net.convs()
    pose = PoseExtractor(ctx, net)
    pose.set_input((-1, bench.NET_H))
    gen = torch.Generator(device="cuda").manual_seed(4321)
    frames = torch.randint(0, 256, (n, 720, 1280, 3), generator=gen, device="cuda", dtype=torch.uint8)
    g16 = bench.gpu_parity_run(net, pose, convs, frames, PRECISION_FP16)
    gsp = bench.gpu_parity_run(net, pose, convs, frames, PRECISION_SPLIT)
    threads = bench.cpu_share()[0]
    p16, psp = bench.cpu_parity([g16, gsp], threads)
    for p in (p16, psp):
        p.pop("per_frame", None)
    print(json.dumps({"frames": n, "cpu_threads": threads, "fp16": p16, "split": psp}, indent=1))


if __name__ == "__main__":
    main()
