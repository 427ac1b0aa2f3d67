"""Rank body for tests/test_distributed.py::test_launcher_ordered_gather_gloo: started by
openpose_amd.parallel.launch_ranks (the launcher bench.py --gpus N uses), runs bench.py's
per-step record flow on CPU over gloo with synthetic per-frame records, and rank 0 writes the
ordered result.  Usage: rank_stub.py OUT.npz STEPS BATCH PARTS"""
import os
import sys

import numpy as np
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openpose_amd import parallel  # noqa: E402


def frame_result(fid, parts):
    """Deterministic synthetic (keypoints, scores) of frame fid: fid % 4 people."""
    rng = np.random.default_rng(fid)
    people = fid % 4
    return (rng.random((people, parts, 3), dtype=np.float32), rng.random(people, dtype=np.float32))


def main():
    out, steps, batch, parts = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    cap = batch * (1 + 4 * (parts * 3 + 1))
    g = parallel.RecordGather(world, rank, cap, steps, "cpu")
    for i in range(steps):
        first = (i * world + rank) * batch
        recs = parallel.pack_records([frame_result(f, parts) for f in range(first, first + batch)],
                                     parts)
        g.push(i, first, batch, recs)
    res = g.finish(parts)
    if rank == 0:
        np.savez(out, n=len(res), **{"kp%d" % i: r[0] for i, r in enumerate(res)},
                 **{"ks%d" % i: r[1] for i, r in enumerate(res)})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
