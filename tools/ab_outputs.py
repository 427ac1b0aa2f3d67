"""dev: BODY_25 net output of the library OPK_LIB_PATH points at (default: the in-tree build) on a
fixed synthetic batch, saved for a bit-for-bit comparison between two builds.

    OPK_LIB_PATH=... python tools/ab_outputs.py OUT.npy [frames]
    python tools/ab_outputs.py --compare A.npy B.npy
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    if sys.argv[1] == "--compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        diff = int((a.view(np.uint32) != b.view(np.uint32)).sum())
        print("outputs %s: %d of %d values differ (max |d| %.3g)"
              % (a.shape, diff, a.size, float(np.abs(a - b).max())))
        sys.exit(1 if diff else 0)
    import torch
    from openpose_amd import synth
    from openpose_amd.api import Context, Net, dev_switches
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    # OPK_AB_DEV="KEY=VAL,KEY=VAL": dev switches for both builds (e.g. HEAD_FUSE=0 to bisect)
    sw = dict(kv.split("=") for kv in os.environ.get("OPK_AB_DEV", "").split(",") if kv)
    dev_switches(**{k: int(v) for k, v in sw.items()}).__enter__()
    ctx = Context(0)
    net = Net(ctx, "builtin:BODY_25")
    net.set_params(synth.he_weights(net.convs(), seed=0, out_scale=0.02))
    x = np.random.default_rng(3).uniform(-0.5, 0.5, (n, 3, 368, 656)).astype(np.float32)
    net.forward(torch.from_numpy(x).cuda())
    np.save(sys.argv[1], net.output_numpy())
    net.close()


if __name__ == "__main__":
    main()
