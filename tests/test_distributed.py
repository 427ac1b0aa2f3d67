"""CPU, world_size 2 over gloo: the frame-parallel runtime (openpose_amd/parallel.py) gives every
frame exactly once, in frame order, identical to a single-process run.  Per-frame work is the
product's host people assembly (libopk_hip.so, no GPU needed) on synthetic people fields."""
import os
import sys
import tempfile

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from openpose_amd import api, parallel
from openpose_amd import pose_tables as pt
from tests.fields import people_field

N_FRAMES = 7


def frame_record(fid):
    f = people_field(2 + fid % 3, 92, 164, seed=500 + fid)
    pk = oracle.nms(f, 0.05, 128, (0.25, 0.25))
    scores = oracle.pair_scores(f, pk, pt.BODY25_PAIRS, pt.BODY25_MAP_IDX)
    kp, ks = api.assemble_people(scores, pk, scale=1.5)
    return (fid, kp, ks)


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    local = parallel.run_sharded(lambda ids: {i: frame_record(i) for i in ids}, N_FRAMES, 2, rank,
                                 world)
    res = parallel.gather_in_order(local, world, rank)
    if rank == 0:
        np.save(out_path, np.array([r[0] for r in res]))
        np.savez(out_path + ".npz", *[r[1] for r in res])
    dist.barrier()
    dist.destroy_process_group()


def test_shard_covers_all_frames():
    for n in (0, 1, 7, 16, 33):
        for w in (1, 2, 3, 8):
            ids = [i for r in range(w) for i in parallel.shard(n, r, w)]
            assert ids == list(range(n))


def test_frame_parallel_gloo_world2():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res.npy")
        port = 29500 + os.getpid() % 1000
        mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
        order = np.load(out)
        assert order.tolist() == list(range(N_FRAMES))
        got = np.load(out + ".npz")
        for i in range(N_FRAMES):
            _, kp, _ = frame_record(i)
            np.testing.assert_array_equal(got["arr_%d" % i], kp)


def _queue_worker(rank, world, port, out_path, delay):
    """dispatch="queue" with rank 1 slowed down per batch: every frame once, in order, and the
    fast rank takes more batches than its static share."""
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    def work(ids):
        if rank == 1:
            time.sleep(delay)
        return {i: (i, rank) + frame_record(i)[1:] for i in ids}
    local = parallel.run_sharded(work, N_Q, 1, rank, world, dispatch="queue")
    # a second queue in the same group starts from batch 0 again (its own store key)
    again = parallel.run_sharded(lambda ids: {i: i for i in ids}, 4, 1, rank, world, dispatch="queue")
    res = parallel.gather_in_order(local, world, rank)
    res2 = parallel.gather_in_order(again, world, rank)
    if rank == 0:
        np.save(out_path, np.array([[r[0], r[1]] for r in res]))
        np.savez(out_path + ".npz", *[r[2] for r in res])
        np.save(out_path + ".again.npy", np.array(res2))
    dist.barrier()
    dist.destroy_process_group()


N_Q = 12


def test_queue_dispatch_balances_uneven_ranks_gloo():
    """run_sharded(dispatch="queue"): batches pulled from one queue in the process group's store
    (the reference's shared worker queue, wrapperAuxiliary.hpp:1050-1058).  With rank 1 0.25 s
    slower per batch, rank 0 takes most of the 12 one-frame batches (the static split: 6 each);
    the ordered gather still returns every frame once, in frame order, with the single-process
    records; a second queue in the same group is independent of the first."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "q.npy")
        port = 29500 + (os.getpid() + 7) % 1000
        mp.spawn(_queue_worker, args=(2, port, out, 0.25), nprocs=2, join=True)
        rows = np.load(out)
        assert rows[:, 0].tolist() == list(range(N_Q))
        by_rank0 = int((rows[:, 1] == 0).sum())
        assert by_rank0 > N_Q // 2 + 1, rows[:, 1].tolist()
        got = np.load(out + ".npz")
        for i in range(N_Q):
            np.testing.assert_array_equal(got["arr_%d" % i], frame_record(i)[1])
        assert np.load(out + ".again.npy").tolist() == [0, 1, 2, 3]


def test_batch_queue_local():
    q = parallel.BatchQueue(7, 3)
    assert [q.claim(), q.claim(), q.claim(), q.claim()] == [[0, 1, 2], [3, 4, 5], [6], None]
    assert q.taken == 3
    with pytest.raises(ValueError):
        parallel.run_sharded(lambda ids: {}, 4, 1, 0, 1, dispatch="random")


def test_gather_detects_missing_frames():
    with pytest.raises(RuntimeError, match="missing"):
        parallel.gather_in_order({0: 1, 2: 3}, 1, 0)


def test_launcher_ordered_gather_gloo():
    """bench.py --gpus N's launcher (parallel.launch_ranks: N child processes, RANK/WORLD_SIZE/
    MASTER_* set, parent makes no device call) + the per-step RecordGather: rank 0 receives every
    frame exactly once, in frame order, with its records intact."""
    from tests.rank_stub import frame_result
    steps, batch, parts = 3, 5, 25
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res.npz")
        stub = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rank_stub.py")
        rc = parallel.launch_ranks(2, [stub, out, str(steps), str(batch), str(parts)], timeout=120)
        assert rc == 0
        got = np.load(out)
        n = int(got["n"])
        assert n == 2 * steps * batch
        for f in range(n):
            kp, ks = frame_result(f, parts)
            np.testing.assert_array_equal(got["kp%d" % f], kp)
            np.testing.assert_array_equal(got["ks%d" % f], ks)


@pytest.mark.parametrize("interval", [1, 2, 4, 7, 0])
def test_launcher_ordered_gather_intervals(interval):
    """The same flow with the records gathered once per `interval` steps (the last group partial
    for 2 and 4 of 7 steps; 0 = once, at finish): every frame exactly once, in frame order."""
    from tests.rank_stub import frame_result
    steps, batch, parts = 7, 3, 25
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res.npz")
        stub = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rank_stub.py")
        rc = parallel.launch_ranks(2, [stub, out, str(steps), str(batch), str(parts), str(interval)],
                                   timeout=120)
        assert rc == 0
        got = np.load(out)
        assert int(got["n"]) == 2 * steps * batch
        for f in range(2 * steps * batch):
            kp, ks = frame_result(f, parts)
            np.testing.assert_array_equal(got["kp%d" % f], kp)
            np.testing.assert_array_equal(got["ks%d" % f], ks)


def test_gather_interval_decouples_ranks():
    """rank 0 falls one step behind (sleeps 1.5 s before pushing step 1).  With
    a gather per step (interval 1) rank 1 stalls in that step's gather until rank 0 arrives; with
    the bench's interval (0: one gather, at finish) rank 1's step loop never waits for rank 0 -- the ranks
    meet only at finish(), and the ordered records are the same."""
    import json
    steps, batch, parts, delay = 6, 2, 25, 1.5
    stub = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rank_stub.py")
    loops = {}
    for interval in (1, 0):
        with tempfile.TemporaryDirectory() as d:
            out = os.path.join(d, "res.npz")
            rc = parallel.launch_ranks(2, [stub, out, str(steps), str(batch), str(parts), str(interval),
                                           "0:1:%g" % delay], timeout=120)
            assert rc == 0
            assert int(np.load(out)["n"]) == 2 * steps * batch
            loops[interval] = [json.load(open("%s.rank%d.json" % (out, r)))["loop_s"] for r in (0, 1)]
    print("rank loop seconds, rank 0 delayed %.1f s at step 1: per-step gather %s, gather at "
          "finish %s" % (delay, loops[1], loops[0]))
    assert loops[1][1] >= 0.8 * delay        # coupled: rank 1 waited in step 1's gather
    assert loops[0][1] < 0.3 * delay         # decoupled: rank 1 ran its steps without waiting
    assert loops[0][0] >= delay              # (rank 0 did sleep)


def test_launcher_propagates_failure():
    rc = parallel.launch_ranks(2, ["-c", "import os, sys; sys.exit(3 if os.environ['RANK'] == '1' "
                                         "else 0)"], timeout=60)
    assert rc == 3


def test_record_gather_rejects_duplicates_and_gaps():
    g = parallel.RecordGather(1, 0, 100, 2, "cpu")
    rec = parallel.pack_records([(np.zeros((0, 25, 3)), np.zeros(0))] * 2, 25)
    g.push(0, 0, 2, rec)
    g.push(1, 3, 2, rec)          # frames 3, 4: frame 2 never produced
    with pytest.raises(RuntimeError, match="missing"):
        g.finish(25)
    g = parallel.RecordGather(1, 0, 100, 2, "cpu")
    g.push(0, 0, 2, rec)
    g.push(1, 1, 2, rec)          # frame 1 twice
    with pytest.raises(RuntimeError, match="twice"):
        g.finish(25)
    with pytest.raises(RuntimeError, match="capacity"):
        g.push(0, 0, 2, np.zeros(101, np.float32))


def test_record_gather_single_rank_roundtrip():
    """world 1 keeps the records on the host: every frame back intact and in order, steps pushed
    out of order included; a step never pushed is an error."""
    from tests.rank_stub import frame_result
    steps, batch, parts = 4, 3, 25
    results = [frame_result(f, parts) for f in range(steps * batch)]
    cap = max(parallel.pack_records(results[i * batch:(i + 1) * batch], parts).size
              for i in range(steps))
    g = parallel.RecordGather(1, 0, cap, steps, "cpu")
    for i in (2, 0, 3, 1):
        g.push(i, i * batch, batch, parallel.pack_records(results[i * batch:(i + 1) * batch], parts))
    got = g.finish(parts)
    assert len(got) == steps * batch
    for (kp, ks), (rk, rs) in zip(got, results):
        np.testing.assert_array_equal(kp, np.asarray(rk, np.float32).reshape(-1, parts, 3))
        np.testing.assert_array_equal(ks, rs)
    g = parallel.RecordGather(1, 0, cap, steps, "cpu")
    g.push(0, 0, batch, parallel.pack_records(results[:batch], parts))
    with pytest.raises(RuntimeError, match="header"):
        g.finish(parts)


def test_record_gather_duplicate_and_views():
    """finish(): a frame delivered by two blocks is an error; the ordered result indexes like a
    list (negative indices, slices) with views of the gathered records."""
    from tests.rank_stub import frame_result
    batch, parts = 3, 25
    results = [frame_result(f, parts) for f in range(2 * batch)]
    cap = max(parallel.pack_records(results[i * batch:(i + 1) * batch], parts).size for i in range(2))
    g = parallel.RecordGather(1, 0, cap, 2, "cpu")
    g.push(0, 0, batch, parallel.pack_records(results[:batch], parts))
    g.push(1, 0, batch, parallel.pack_records(results[:batch], parts))   # frames 0..2 again
    with pytest.raises(RuntimeError, match="twice"):
        g.finish(parts)
    g = parallel.RecordGather(1, 0, cap, 2, "cpu")
    for i in range(2):
        g.push(i, i * batch, batch, parallel.pack_records(results[i * batch:(i + 1) * batch], parts))
    got = g.finish(parts)
    assert len(got) == 2 * batch and len(got[1:4]) == 3
    np.testing.assert_array_equal(got[-1][1], results[-1][1])
    np.testing.assert_array_equal(got[2:3][0][0], np.asarray(results[2][0], np.float32).reshape(-1, parts, 3))
    with pytest.raises(IndexError):
        got[2 * batch]


def test_record_gather_forced_collective_single_rank():
    """RecordGather(collective=True) at world size 1 (bench.py --collective-gather): the records
    go through dist.gather and the device-side unpack, here over a one-rank gloo group on CPU;
    the result equals the host path's."""
    import torch.distributed as dist
    from tests.rank_stub import frame_result
    steps, batch, parts = 3, 4, 25
    results = [frame_result(f, parts) for f in range(steps * batch)]
    cap = max(parallel.pack_records(results[i * batch:(i + 1) * batch], parts).size
              for i in range(steps))
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % parallel.free_port(),
                            rank=0, world_size=1)
    try:
        g = parallel.RecordGather(1, 0, cap, steps, "cpu", collective=True)
        assert not g.local
        for i in range(steps):
            g.push(i, i * batch, batch, parallel.pack_records(results[i * batch:(i + 1) * batch], parts))
        got = g.finish(parts)
    finally:
        dist.destroy_process_group()
    assert len(got) == steps * batch
    for (kp, ks), (rk, rs) in zip(got, results):
        np.testing.assert_array_equal(kp, np.asarray(rk, np.float32).reshape(-1, parts, 3))
        np.testing.assert_array_equal(ks, rs)


def test_bench_rejects_world_mismatch():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    bench = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
    r = subprocess.run([sys.executable, bench, "--gpus", "4"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_bench_content_depends_on_global_batch_only():
    """bench.py's synthetic input of a frame depends only on its global batch index (step x world
    + rank, the frame ids RecordGather assigns): every world size sees the same content per global
    batch, and each rank holds exactly the contents its batches use."""
    import bench
    for world in (1, 2, 4, 8):
        for rank in range(world):
            have = set(bench.contents_of_rank(rank, world))
            for step in range(12):
                k = step * world + rank
                assert k % bench.CONTENTS in have
            assert have == {(s * world + rank) % bench.CONTENTS for s in range(12)}


def test_rank_cpus_disjoint_gpu_local_shares(monkeypatch):
    """every rank's people-assembly threads get a disjoint share of its GPU's
    NUMA-local CPUs (parallel.rank_cpus, applied by bench.py before any GPU call); the assembly
    pool is sized from the affinity mask (PoseHip::assembly_threads)."""
    monkeypatch.delenv("OPK_BENCH_REHEARSE", raising=False)
    aff = list(range(256))
    numa = [0, 0, 0, 0, 1, 1, 1, 1]
    node_cpus = {0: range(0, 128), 1: range(128, 256)}
    shares = [parallel.rank_cpus(r, 8, aff, numa, node_cpus) for r in range(8)]
    seen = set()
    for r, s in enumerate(shares):
        assert len(s) == 32 and not seen & set(s)
        seen |= set(s)
        assert set(s) <= set(node_cpus[numa[r]])   # GPU-local
    # the mask restricts the shares; no NUMA information: contiguous split of the mask
    shares = [parallel.rank_cpus(r, 2, list(range(16, 48)), [], None) for r in range(2)]
    assert shares == [list(range(16, 32)), list(range(32, 48))]
    assert parallel.rank_cpus(0, 1, aff, numa, node_cpus) is None   # one rank: mask untouched
    # rehearsal (every rank on GPU 0): the ranks split GPU 0's node
    monkeypatch.setenv("OPK_BENCH_REHEARSE", "1")
    shares = [parallel.rank_cpus(r, 2, aff, numa, node_cpus) for r in range(2)]
    assert shares == [list(range(0, 64)), list(range(64, 128))]
    assert parallel.cpu_ranges([0, 1, 2, 5, 7, 8]) == "0-2,5,7-8"
