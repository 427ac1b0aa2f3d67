"""Frame-parallel multi-GPU runtime: one process per GPU, frames sharded, results re-ordered.

Reference behaviour: one PoseExtractorCaffe + worker thread per GPU pulling
frames from a shared queue (include/openpose/wrapper/wrapperAuxiliary.hpp:328-337,1050-1067) and a
WQueueOrderer that re-sequences results by frame id (include/openpose/thread/wQueueOrderer.hpp:
62-141).  Here: one process per GPU under torch.distributed (RCCL on the GPU box, gloo on CPU),
frames assigned to ranks in contiguous blocks, or pulled batch by batch from one queue shared
through the process group's store (run_sharded(dispatch="queue"), BatchQueue) -- no data-path
collective either way: every rank runs the whole hot path on its own frames -- and the per-frame
keypoint records gathered to rank 0 in frame order (the only collective; a few KB per frame).
"""
import os
import socket
import subprocess
import sys
import time

from collections.abc import Sequence

import numpy as np
import torch
import torch.distributed as dist


def shard(n_frames, rank, world):
    """Contiguous frame ids of this rank (sizes differ by at most one)."""
    base, extra = divmod(n_frames, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def gather_in_order(local, world, rank, dst=0, group=None):
    """local: {frame_id: record}. Returns [record, ...] ordered by frame id on `dst`, else None.

    Frames missing from every rank raise (the WQueueOrderer would wait forever for them)."""
    if world == 1:
        parts = [local]
    else:
        parts = [None] * world if rank == dst else None
        dist.gather_object(local, parts, dst=dst, group=group)
        if rank != dst:
            return None
    merged = {}
    for p in parts:
        for k, v in p.items():
            if k in merged:
                raise RuntimeError("frame %d produced twice" % k)
            merged[k] = v
    ids = sorted(merged)
    if ids and ids != list(range(ids[0], ids[0] + len(ids))):
        raise RuntimeError("frames missing from the gather: %s" % sorted(set(range(ids[0], ids[-1] + 1)) - set(ids)))
    return [merged[i] for i in ids]


_QUEUE_SEQ = [0]   # queues made so far (every rank makes them in the same order: same keys)


class BatchQueue:
    """One work queue of frame batches shared by every rank -- the reference's per-GPU workers
    pulling datums from one queue (include/openpose/wrapper/wrapperAuxiliary.hpp:1050-1058) --
    over the process group's key-value store: batch k (frames k*batch .. min((k+1)*batch, n) - 1)
    goes to the rank whose atomic store.add on the queue's counter returned k, so a rank that
    finishes its batches sooner takes more of them and no rank waits for a slower one's share.
    World size 1 (or no process group): a local counter.  claim() returns the next batch's frame
    ids, or None once every batch is taken; the caller's ordered gather (gather_in_order /
    RecordGather.finish) re-sequences the frames, as the reference's WQueueOrderer does."""

    def __init__(self, n_frames, batch, store=None):
        self.n, self.batch = int(n_frames), max(1, int(batch))
        self.batches = (self.n + self.batch - 1) // self.batch
        if store is None and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            store = dist.distributed_c10d._get_default_store()
        self.store = store
        self.key = "opk_batch_queue_%d" % _QUEUE_SEQ[0]
        _QUEUE_SEQ[0] += 1
        self.next_local = 0
        self.taken = 0   # batches this rank claimed

    def claim(self):
        if self.store is None:
            k = self.next_local
            self.next_local += 1
        else:
            k = int(self.store.add(self.key, 1)) - 1
        if k >= self.batches:
            return None
        self.taken += 1
        return list(range(k * self.batch, min((k + 1) * self.batch, self.n)))


def run_sharded(process_batch, n_frames, batch, rank, world, dispatch="static"):
    """Run process_batch(list_of_frame_ids) -> {frame_id: record} over this rank's frames.
    dispatch "static": the contiguous block of shard(); "queue": batches claimed from a BatchQueue
    shared by all ranks (uneven per-frame cost: no rank idles while another still holds work)."""
    out = {}
    if dispatch == "queue":
        q = BatchQueue(n_frames, batch)
        while True:
            ids = q.claim()
            if ids is None:
                return out
            out.update(process_batch(ids))
    if dispatch != "static":
        raise ValueError("dispatch: static or queue")
    mine = list(shard(n_frames, rank, world))
    for i in range(0, len(mine), batch):
        out.update(process_batch(mine[i:i + batch]))
    return out


# ---- per-rank host CPUs ---------------------------------------------------------------------------
def _cpulist(text):
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def gpu_numa_nodes(root="/sys/class/kfd/kfd/topology/nodes"):
    """NUMA node of every GPU in KFD topology order (the HIP device order when no *_VISIBLE_DEVICES
    remaps it): a GPU node (simd_count > 0) links to its CPU node through io_links.  [] when the
    topology is not readable."""
    try:
        nodes = sorted(int(n) for n in os.listdir(root) if n.isdigit())
    except OSError:
        return []
    props = {}
    for n in nodes:
        try:
            with open(os.path.join(root, str(n), "properties")) as f:
                props[n] = dict(l.split()[:2] for l in f if len(l.split()) >= 2)
        except OSError:
            return []
    cpu_nodes = [n for n in nodes if int(props[n].get("cpu_cores_count", 0)) > 0]
    out = []
    for n in nodes:
        if int(props[n].get("simd_count", 0)) == 0:
            continue
        numa = None
        links = os.path.join(root, str(n), "io_links")
        for l in sorted(os.listdir(links)) if os.path.isdir(links) else []:
            try:
                with open(os.path.join(links, l, "properties")) as f:
                    to = dict(x.split()[:2] for x in f if len(x.split()) >= 2).get("node_to")
            except OSError:
                continue
            if to is not None and int(to) in cpu_nodes:
                numa = cpu_nodes.index(int(to))
                break
        out.append(numa)
    return out


def rank_cpus(local_rank, local_world, affinity=None, gpu_numa=None, node_cpus=None):
    """Host CPUs for rank `local_rank` of `local_world` ranks on one node (one GPU each): the CPUs of
    its GPU's NUMA node within the process's affinity mask, split into disjoint contiguous shares
    among the ranks on that node -- the reference's per-GPU worker threads
    (wrapperAuxiliary.hpp:328-337, 1050-1067) each with host cores of their own for the people
    assembly.  Without NUMA information (or a node with none of the allowed CPUs) the affinity
    mask is split into local_world contiguous shares.  None: leave the mask alone (one rank)."""
    if local_world <= 1:
        return None
    aff = sorted(affinity if affinity is not None else os.sched_getaffinity(0))
    if gpu_numa is None:
        visible = any(os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                                                  "ROCR_VISIBLE_DEVICES"))
        gpu_numa = [] if visible else gpu_numa_nodes()
    gpu = local_rank if os.environ.get("OPK_BENCH_REHEARSE") != "1" else 0
    group, pool = list(range(local_world)), aff
    if gpu_numa and all(g is not None for g in gpu_numa) and len(gpu_numa) >= local_world:
        def numa_of(r):
            return gpu_numa[r if os.environ.get("OPK_BENCH_REHEARSE") != "1" else 0]
        node = gpu_numa[gpu]
        if node_cpus is None:
            try:
                with open("/sys/devices/system/node/node%d/cpulist" % node) as f:
                    cpus = set(_cpulist(f.read()))
            except OSError:
                cpus = set()
        else:
            cpus = set(node_cpus[node])
        local = [c for c in aff if c in cpus]
        if local:
            group = [r for r in range(local_world) if numa_of(r) == node]
            pool = local
    k, i = len(group), group.index(local_rank)
    share = len(pool) // k
    if share == 0:
        return [pool[i % len(pool)]]
    return pool[i * share:(i + 1) * share]


def pin_rank_cpus(local_rank, local_world):
    """Restrict this process (before it starts any thread or touches a GPU) to rank_cpus(); returns
    the CPU list applied, or None."""
    cpus = rank_cpus(local_rank, local_world)
    if cpus:
        os.sched_setaffinity(0, cpus)
    return cpus


def cpu_ranges(cpus):
    """[0, 1, 2, 5] -> '0-2,5'."""
    out, cpus = [], sorted(cpus)
    i = 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append("%d" % cpus[i] if i == j else "%d-%d" % (cpus[i], cpus[j]))
        i = j + 1
    return ",".join(out)


# ---- launcher: one process per GPU --------------------------------------------------------------
def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, port=None, env=None, timeout=None):
    """Start `python argv...` n times as ranks 0..n-1 of one job (RANK, LOCAL_RANK, WORLD_SIZE,
    MASTER_ADDR=127.0.0.1, MASTER_PORT) and wait for all of them.  The reference starts one worker
    thread per GPU (wrapperAuxiliary.hpp:328-337); here each GPU gets a process, started as a child
    of a parent that itself makes no GPU call.  If a rank fails, the others are terminated (by
    PID).  Returns 0 or the first non-zero exit status."""
    port = port or free_port()
    procs = []
    for r in range(n):
        e = dict(os.environ if env is None else env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
    t0 = time.time()
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in alive:
                    q.terminate()
        if timeout is not None and time.time() - t0 > timeout and alive:
            for q in alive:
                q.kill()
            rc = rc or 124
        time.sleep(0.05)
    return rc


# ---- ordered per-step result gather (WQueueOrderer) ----------------------------------------------
HEAD = 5   # record header: rank, step, first frame id, frames, payload floats


class RecordGather:
    """Gathers every rank's per-frame result records to rank 0, in frame order.

    The reference's WQueueOrderer (include/openpose/thread/wQueueOrderer.hpp:62-141) re-sequences
    the datums that its per-GPU workers finish out of order.  Here the frames of step i are split
    into contiguous per-rank slices (rank r holds frames (i * world + r) * batch ...), each rank
    packs its slice's records (PoseExtractor.records(): per frame [people, keypoints, scores]),
    and the records move to rank 0 (RCCL over xGMI on the GPU box, gloo on CPU) once per
    `interval` steps: one gather of the group's blocks, the last (partial) group at finish();
    interval <= 0: one gather of all steps, at finish().
    A gather is a rendezvous of all ranks, so with interval 1 a rank that falls behind by one step
    stalls every other rank at that step's gather (measured on gloo: tests/test_distributed.py
    test_gather_interval_decouples_ranks); with interval k the ranks meet only every k steps --
    interval 0 (bench.py's default) couples them only at finish(), as the reference's workers are
    coupled only by its ordered output queue.  `finish()` on rank 0 returns the records of every frame in frame
    order and raises if a frame is missing or duplicated.  `capacity` = floats per rank and step
    (records beyond it raise).  `collective`: move the records through the collective even at
    world size 1 (a process group must exist) -- the 1-GPU box's test of the transport an N-GPU
    run uses (pinned staging, events, dist.gather of device tensors, the device-side unpack)."""

    def __init__(self, world, rank, capacity, steps, device, group=None, collective=False,
                 interval=1):
        self.world, self.rank, self.steps, self.group = world, rank, steps, group
        self.device = torch.device(device)
        self.cap = int(capacity)
        # (a group that never fills before the last step is gathered by finish())
        self.interval = int(interval) if int(interval) > 0 else max(1, steps) + 1
        self.local = world == 1 and not collective
        if self.local:
            # nothing to move: the records stay on the host, one block per step (pages touched
            # here, outside any timed region)
            self.blocks = np.zeros((steps, HEAD + self.cap), np.float32)
            self.blocks.fill(-1.0)
            return
        cuda = self.device.type == "cuda"
        g = min(self.interval, max(1, steps))   # staging rows
        self.send = torch.zeros((g, HEAD + self.cap), dtype=torch.float32, device=self.device)
        # two host staging groups: the upload of group k may still be in flight while group k+1
        # packs (cuda: pinned memory + one event per group)
        self.host = [torch.zeros((g, HEAD + self.cap), dtype=torch.float32, pin_memory=cuda)
                     for _ in range(2)]
        self.events = [torch.cuda.Event() if cuda else None for _ in range(2)]
        self.pending = 0          # steps packed into the current group, not yet gathered
        self.gathered = 0         # steps already gathered
        # rank-major, so that each rank's blocks of a group are one contiguous gather target
        self.recv = (torch.zeros((world, steps, HEAD + self.cap), dtype=torch.float32,
                                 device=self.device) if rank == 0 else None)
        if self.recv is not None:
            # the device ops of finish() once here, so that their first-use costs (code object
            # loads on a GPU) fall outside any timed region
            self.recv[:, :, :HEAD].cpu()
            torch.cat([self.recv[r, i, HEAD:HEAD + 1]
                       for i in range(self.steps) for r in range(self.world)]).cpu()

    def push(self, step, first_frame, n_frames, records):
        n = int(records.size)
        if n > self.cap:
            raise RuntimeError("rank %d step %d: %d record floats exceed the gather capacity %d"
                               % (self.rank, step, n, self.cap))
        if self.local:
            blk = self.blocks[step]
            blk[:HEAD] = (self.rank, step, first_frame, n_frames, n)
            blk[HEAD:HEAD + n] = records
            return
        if step != self.gathered + self.pending:
            raise RuntimeError("rank %d: step %d pushed out of order" % (self.rank, step))
        grp = self.gathered // self.interval
        k = grp % 2
        if self.pending == 0 and self.events[k] is not None and grp >= 2:
            self.events[k].synchronize()   # this staging group's previous upload has landed
        h = self.host[k].numpy()[self.pending]
        h[:HEAD] = (self.rank, step, first_frame, n_frames, n)
        h[HEAD:HEAD + n] = records
        self.pending += 1
        if self.pending == self.interval:
            self._gather()

    def _gather(self):
        """One gather of the current group's blocks (all ranks have the same steps, so the same
        groups)."""
        g = self.pending
        if g == 0:
            return
        k = (self.gathered // self.interval) % 2
        self.send[:g].copy_(self.host[k][:g], non_blocking=True)
        if self.events[k] is not None:
            self.events[k].record()
        s0 = self.gathered
        dist.gather(self.send[:g], [self.recv[r, s0:s0 + g] for r in range(self.world)]
                    if self.rank == 0 else None, dst=0, group=self.group)
        self.gathered += g
        self.pending = 0

    def _unpack_device(self):
        """(headers [steps, world, HEAD], the used part of every (step, rank) block, concatenated
        in (step, rank) order): two device-to-host copies, most of each worst-case-sized block
        stays behind."""
        heads = self.recv[:, :, :HEAD].transpose(0, 1).cpu().numpy()
        lens = heads[:, :, 4].astype(np.int64)
        if (lens < 0).any() or (lens > self.cap).any():
            raise RuntimeError("record headers hold impossible lengths: %s" % lens.tolist())
        body = torch.cat([self.recv[r, i, HEAD:HEAD + int(lens[i, r])]
                          for i in range(self.steps) for r in range(self.world)]).cpu().numpy()
        return heads, body

    def finish(self, parts):
        """Rank 0: every frame's record in frame order, as an OrderedRecords sequence of
        (keypoints [people, parts, 3], scores [people]); raises if a frame is missing or produced
        twice, or a block's records do not parse to its header's length."""
        if not self.local:
            self._gather()   # the last (partial) group
        if self.rank != 0:
            return None
        if self.local:   # headers and bodies in place (never-pushed steps: header -1)
            heads = self.blocks[:, None, :HEAD]
            starts = (np.arange(self.steps) * (HEAD + self.cap) + HEAD)[:, None]
            body_all = self.blocks.reshape(-1)
        else:
            heads, body_all = self._unpack_device()
            lens = heads[:, :, 4].astype(np.int64)
            starts = np.concatenate([[0], np.cumsum(lens.reshape(-1))[:-1]]).reshape(lens.shape)
        stride = parts * 3 + 1
        ids, offs, counts = [], [], []
        for i in range(self.steps):
            for r in range(self.world):
                head = heads[i, r]
                rank, step, first, nf, n = (int(v) for v in head)
                if rank != r or step != i:
                    raise RuntimeError("step %d rank %d: record header %s" % (i, r, head.tolist()))
                base = int(starts[i, r])
                o = base
                for f in range(first, first + nf):   # the per-frame walk: one count read each
                    people = int(body_all[o])
                    ids.append(f)
                    offs.append(o)
                    counts.append(people)
                    o += 1 + people * stride
                if o - base != n:
                    raise RuntimeError("step %d rank %d: %d of %d record floats parsed"
                                       % (i, r, o - base, n))
        ids = np.asarray(ids, np.int64)
        order = np.argsort(ids, kind="stable")
        ids = ids[order]
        if len(ids) and (np.any(ids[1:] == ids[:-1])):
            raise RuntimeError("frame %d produced twice" % int(ids[1:][ids[1:] == ids[:-1]][0]))
        if len(ids) and not np.array_equal(ids, np.arange(len(ids))):
            raise RuntimeError("frames missing from the gather: %s"
                               % sorted(set(range(int(ids[-1]) + 1)) - set(ids.tolist())))
        return OrderedRecords(body_all, np.asarray(offs, np.int64)[order],
                              np.asarray(counts, np.int64)[order], parts)


class OrderedRecords(Sequence):
    """The gathered records of frames 0..F-1 in frame order (RecordGather.finish): item f is
    (keypoints [people, parts, 3], scores [people]) as views into the gathered storage, made on
    access -- the parse (every frame's position and people count) and its checks are done."""

    def __init__(self, body, offsets, counts, parts):
        self._body, self._off, self._cnt, self.parts = body, offsets, counts, parts

    def __len__(self):
        return len(self._off)

    def __getitem__(self, f):
        if isinstance(f, slice):
            return [self[i] for i in range(*f.indices(len(self)))]
        if f < 0:
            f += len(self)
        if not 0 <= f < len(self):
            raise IndexError(f)
        o, n = int(self._off[f]) + 1, int(self._cnt[f])
        k = n * self.parts * 3
        return self._body[o:o + k].reshape(n, self.parts, 3), self._body[o + k:o + k + n]


def pack_records(results, parts):
    """Host-side packing of [(keypoints, scores), ...] into the opk_pose_records layout."""
    out = []
    for kp, ks in results:
        kp = np.asarray(kp, np.float32).reshape(-1, parts, 3)
        out.append(np.float32([kp.shape[0]]))
        out.append(kp.reshape(-1))
        out.append(np.asarray(ks, np.float32).reshape(-1))
    return np.concatenate(out) if out else np.zeros(0, np.float32)
