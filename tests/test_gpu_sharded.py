"""GPU: the frame-sharded path of BASELINE.json configs 3 and 5 (frames split across GPUs, one
process per GPU, per-frame records gathered to rank 0 in frame order inside the timed loop;
openpose_amd/parallel.py) run on the real pipelines.  The box has one GPU, so
bench.py runs in its rehearsal mode (OPK_BENCH_REHEARSE=1): the parent spawns the ranks before any
GPU call, every rank puts its pipeline on GPU 0 and the gather runs over gloo -- the code path of
an N-GPU run except the RCCL transport.  The N-rank throughput of such a run means nothing.

Results, not just plumbing: a frame's synthetic input depends only on its global frame id
(bench.contents_of_rank), so rank 0's gathered records of a 2-rank run must equal, frame for frame
and bit for bit, those of a 1-rank run over the same frame ids (the reference's WQueueOrderer
contract: the sharded pipeline's output is the single pipeline's, in order --
include/openpose/thread/wQueueOrderer.hpp:62-141, wrapperAuxiliary.hpp:1050-1067)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(config, gpus, steps, batch, dump):
    env = dict(os.environ, OPK_BENCH_REHEARSE="1", MASTER_ADDR="127.0.0.1")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(gpus), "--steps", str(steps),
                        "--warmup", "1", "--batch", str(batch), "--no-cpu-baseline",
                        "--config", config, "--dump-records", dump],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["body25", "body135"])
def test_sharded_bench_two_ranks(config, tmp_path):
    batch, steps = 8, 2
    d2, d1 = str(tmp_path / "r2.npz"), str(tmp_path / "r1.npz")
    line = _run(config, 2, steps, batch, d2)
    assert line["n_gpus"] == 2 and line["steps"] == steps
    # rank 0 received every frame of both ranks exactly once, in frame order (RecordGather
    # raises on a missing or duplicated frame)
    assert line["config"]["frames_gathered_in_order"] == 2 * batch * steps
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert "REHEARSAL" in line["config"]["parallelism"]
    # the same frame ids through one rank: identical records, frame for frame
    one = _run(config, 1, 2 * steps, batch, d1)
    assert one["config"]["frames_gathered_in_order"] == 2 * batch * steps
    a, b = np.load(d2), np.load(d1)
    assert len(a["counts"]) == 2 * batch * steps
    np.testing.assert_array_equal(a["counts"], b["counts"])
    np.testing.assert_array_equal(a["keypoints"], b["keypoints"])
    np.testing.assert_array_equal(a["scores"], b["scores"])
    assert a["counts"].sum() >= batch   # people were found


@pytest.mark.gpu
def test_alternating_net_outputs_same_records(tmp_path):
    """Batch i+1's nets write the other of two net-output buffers while batch i's post-processing
    still reads the first (PoseHip::next_output, NET_OUT_ALT): every frame's records equal those of
    the single-buffer pipeline, whose nets wait for the previous post-processing.  The frame
    contents change every step, so a net overwriting an output before its reader ran would show."""
    def run(alt, dump):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1")
        r = subprocess.run([sys.executable, "bench.py", "--steps", "6", "--warmup", "1", "--batch", "32",
                            "--no-cpu-baseline", "--dev", "NET_OUT_ALT=%d" % alt, "--dump-records", dump],
                           cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
    d0, d1 = str(tmp_path / "alt0.npz"), str(tmp_path / "alt1.npz")
    run(0, d0)
    run(1, d1)
    a, b = np.load(d0), np.load(d1)
    assert len(a["counts"]) == 6 * 32
    np.testing.assert_array_equal(a["counts"], b["counts"])
    np.testing.assert_array_equal(a["keypoints"], b["keypoints"])
    np.testing.assert_array_equal(a["scores"], b["scores"])
    assert a["counts"].sum() >= 32


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["body25", "body135"])
def test_rccl_gather_one_rank(config, tmp_path):
    """The RCCL transport of an N-GPU run, executed on the 1-GPU box: bench.py
    --collective-gather creates an nccl process group of one rank and forces RecordGather through
    its collective branch -- pinned host staging, events, dist.gather of CUDA tensors, the
    device-side unpack (_unpack_device) -- and the max-over-ranks all-gather on the device.  The
    gathered records must equal the host path's (world size 1, no process group) bit for bit."""
    batch, steps = 8, 3

    def run(extra, dump):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1")
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "OPK_BENCH_REHEARSE"):
            env.pop(k, None)
        r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--steps", str(steps),
                            "--warmup", "1", "--batch", str(batch), "--no-cpu-baseline",
                            "--config", config, "--dump-records", dump] + extra,
                           cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    dc, dh = str(tmp_path / "coll.npz"), str(tmp_path / "host.npz")
    line = run(["--collective-gather"], dc)
    assert line["n_gpus"] == 1 and "RCCL" in line["config"]["parallelism"]
    assert line["config"]["frames_gathered_in_order"] == batch * steps
    run([], dh)
    a, b = np.load(dc), np.load(dh)
    assert len(a["counts"]) == batch * steps
    np.testing.assert_array_equal(a["counts"], b["counts"])
    np.testing.assert_array_equal(a["keypoints"], b["keypoints"])
    np.testing.assert_array_equal(a["scores"], b["scores"])
    assert a["counts"].sum() >= batch
