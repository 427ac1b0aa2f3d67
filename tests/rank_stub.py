"""Rank body for tests/test_distributed.py::test_launcher_ordered_gather_gloo: started by
openpose_amd.parallel.launch_ranks (the launcher bench.py --gpus N uses), runs bench.py's
per-step record flow on CPU over gloo with synthetic per-frame records, and rank 0 writes the
ordered result.  Usage: rank_stub.py OUT.npz STEPS BATCH PARTS [INTERVAL [RANK:STEP:SECONDS]]
INTERVAL: RecordGather's gather interval (default 1); RANK:STEP:SECONDS: that rank sleeps before
pushing that step (a rank falling behind); every rank writes OUT.rank<r>.json with the seconds its
step loop took (its pushes, before finish())."""
import json
import os
import sys
import time

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
    interval = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    delay = tuple(float(v) for v in sys.argv[6].split(":")) if len(sys.argv) > 6 else (-1, -1, 0)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    cap = batch * (1 + 4 * (parts * 3 + 1))
    g = parallel.RecordGather(world, rank, cap, steps, "cpu", interval=interval)
    recs = []
    for i in range(steps):
        first = (i * world + rank) * batch
        recs.append(parallel.pack_records([frame_result(f, parts) for f in range(first, first + batch)],
                                          parts))
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        if rank == int(delay[0]) and i == int(delay[1]):
            time.sleep(delay[2])
        g.push(i, (i * world + rank) * batch, batch, recs[i])
    loop_s = time.perf_counter() - t0
    res = g.finish(parts)
    with open("%s.rank%d.json" % (out, rank), "w") as f:
        json.dump({"loop_s": loop_s, "interval": g.interval}, f)
    if rank == 0:
        np.savez(out, n=len(res), **{"kp%d" % i: r[0] for i, r in enumerate(res)},
                 **{"ks%d" % i: r[1] for i, r in enumerate(res)})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
