"""GPU: the frame-sharded path of BASELINE.json configs 3 and 5 (frames split across GPUs, one
process per GPU, per-frame records gathered to rank 0 in frame order inside the timed loop;
openpose_amd/parallel.py) run on the real pipelines.  The box has one GPU, so
bench.py runs in its rehearsal mode (OPK_BENCH_REHEARSE=1): the parent spawns the ranks before any
GPU call, every rank puts its pipeline on GPU 0 and the gather runs over gloo -- the code path of
an N-GPU run except the RCCL transport.  The N-rank throughput of such a run means nothing."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["body25", "body135"])
def test_sharded_bench_two_ranks(config):
    env = dict(os.environ, OPK_BENCH_REHEARSE="1", MASTER_ADDR="127.0.0.1")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    batch, steps = 8, 3
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", str(steps),
                        "--warmup", "1", "--batch", str(batch), "--no-cpu-baseline",
                        "--config", config],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["steps"] == steps
    # rank 0 received every frame of both ranks exactly once, in frame order (RecordGather
    # raises on a missing or duplicated frame)
    assert line["config"]["frames_gathered_in_order"] == 2 * batch * steps
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert "REHEARSAL" in line["config"]["parallelism"]
