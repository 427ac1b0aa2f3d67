"""Frame-parallel multi-GPU runtime: one process per GPU, frames sharded, results re-ordered.

Reference behaviour: one PoseExtractorCaffe + worker thread per GPU pulling
frames from a shared queue (include/openpose/wrapper/wrapperAuxiliary.hpp:328-337,1050-1067) and a
WQueueOrderer that re-sequences results by frame id (include/openpose/thread/wQueueOrderer.hpp:
62-141).  Here: one process per GPU under torch.distributed (RCCL on the GPU box, gloo on CPU),
frames assigned to ranks in contiguous blocks (no data-path collective: every rank runs the whole
hot path on its own frames), and the per-frame keypoint records gathered to rank 0 in frame order
(the only collective; a few KB per frame).
"""
import os
import socket
import subprocess
import sys
import time

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


def run_sharded(process_batch, n_frames, batch, rank, world):
    """Run process_batch(list_of_frame_ids) -> {frame_id: record} over this rank's frames."""
    mine = list(shard(n_frames, rank, world))
    out = {}
    for i in range(0, len(mine), batch):
        out.update(process_batch(mine[i:i + batch]))
    return out


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
    """Gathers every rank's per-frame result records to rank 0 once per step, in frame order.

    The reference's WQueueOrderer (include/openpose/thread/wQueueOrderer.hpp:62-141) re-sequences
    the datums that its per-GPU workers finish out of order.  Here the frames of step i are split
    into contiguous per-rank slices (rank r holds frames (i * world + r) * batch ...), each rank
    packs its slice's records (PoseExtractor.records(): per frame [people, keypoints, scores]),
    and one gather per step (RCCL over xGMI on the GPU box, gloo on CPU) moves them to rank 0.
    `finish()` on rank 0 returns the records of every frame in frame order and raises if a frame
    is missing or duplicated.  `capacity` = floats per rank and step (records beyond it raise)."""

    def __init__(self, world, rank, capacity, steps, device, group=None):
        self.world, self.rank, self.steps, self.group = world, rank, steps, group
        self.device = torch.device(device)
        self.cap = int(capacity)
        if world == 1:
            # nothing to move: the records stay on the host, one block per step (pages touched
            # here, outside any timed region)
            self.blocks = np.zeros((steps, HEAD + self.cap), np.float32)
            self.blocks.fill(-1.0)
            return
        cuda = self.device.type == "cuda"
        self.send = torch.zeros(HEAD + self.cap, dtype=torch.float32, device=self.device)
        # two host staging buffers: the upload of step i may still be in flight while step i+1
        # packs (cuda: pinned memory + one event per buffer)
        self.host = [torch.zeros(HEAD + self.cap, dtype=torch.float32, pin_memory=cuda)
                     for _ in range(2)]
        self.events = [torch.cuda.Event() if cuda else None for _ in range(2)]
        self.recv = (torch.zeros((steps, world, HEAD + self.cap), dtype=torch.float32,
                                 device=self.device) if rank == 0 else None)
        if self.recv is not None:
            # the device ops of finish() once here, so that their first-use costs (code object
            # loads on a GPU) fall outside any timed region
            self.recv[:, :, :HEAD].cpu()
            torch.cat([self.recv[i, r, HEAD:HEAD + 1]
                       for i in range(self.steps) for r in range(self.world)]).cpu()

    def push(self, step, first_frame, n_frames, records):
        n = int(records.size)
        if n > self.cap:
            raise RuntimeError("rank %d step %d: %d record floats exceed the gather capacity %d"
                               % (self.rank, step, n, self.cap))
        if self.world == 1:
            blk = self.blocks[step]
            blk[:HEAD] = (self.rank, step, first_frame, n_frames, n)
            blk[HEAD:HEAD + n] = records
            return
        k = step % 2
        if self.events[k] is not None and step >= 2:
            self.events[k].synchronize()
        h = self.host[k].numpy()
        h[:HEAD] = (self.rank, step, first_frame, n_frames, n)
        h[HEAD:HEAD + n] = records
        self.send[:HEAD + n].copy_(self.host[k][:HEAD + n], non_blocking=True)
        if self.events[k] is not None:
            self.events[k].record()
        dist.gather(self.send, list(self.recv[step].unbind(0)) if self.rank == 0 else None,
                    dst=0, group=self.group)

    def _unpack_device(self):
        """(headers [steps, world, HEAD], the used part of every (step, rank) block, concatenated
        in (step, rank) order): two device-to-host copies, most of each worst-case-sized block
        stays behind."""
        heads = self.recv[:, :, :HEAD].cpu().numpy()
        lens = heads[:, :, 4].astype(np.int64)
        if (lens < 0).any() or (lens > self.cap).any():
            raise RuntimeError("record headers hold impossible lengths: %s" % lens.tolist())
        body = torch.cat([self.recv[i, r, HEAD:HEAD + int(lens[i, r])]
                          for i in range(self.steps) for r in range(self.world)]).cpu().numpy()
        return heads, body

    def finish(self, parts):
        """Rank 0: [(keypoints [people, parts, 3], scores [people]), ...] for frames 0..F-1."""
        if self.rank != 0:
            return None
        if self.world == 1:   # headers and bodies in place (never-pushed steps: header -1)
            heads = self.blocks[:, None, :HEAD]
            starts = (np.arange(self.steps) * (HEAD + self.cap) + HEAD)[:, None]
            body_all = self.blocks.reshape(-1)
        else:
            heads, body_all = self._unpack_device()
            lens = heads[:, :, 4].astype(np.int64)
            starts = np.concatenate([[0], np.cumsum(lens.reshape(-1))[:-1]]).reshape(lens.shape)
        frames = {}
        for i in range(self.steps):
            for r in range(self.world):
                head = heads[i, r]
                rank, step, first, nf, n = (int(v) for v in head)
                if rank != r or step != i:
                    raise RuntimeError("step %d rank %d: record header %s" % (i, r, head.tolist()))
                base = int(starts[i, r])
                body = body_all[base:base + n]   # views (the result keeps the storage alive)
                o = 0
                for f in range(first, first + nf):
                    people = int(body[o])
                    o += 1
                    kp = body[o:o + people * parts * 3].reshape(people, parts, 3)
                    o += people * parts * 3
                    ks = body[o:o + people]
                    o += people
                    if f in frames:
                        raise RuntimeError("frame %d produced twice" % f)
                    frames[f] = (kp, ks)
                if o != n:
                    raise RuntimeError("step %d rank %d: %d of %d record floats parsed" % (i, r, o, n))
        ids = sorted(frames)
        if ids != list(range(len(ids))):
            raise RuntimeError("frames missing from the gather: %s"
                               % sorted(set(range(ids[-1] + 1)) - set(ids)))
        return [frames[i] for i in ids]


def pack_records(results, parts):
    """Host-side packing of [(keypoints, scores), ...] into the opk_pose_records layout."""
    out = []
    for kp, ks in results:
        kp = np.asarray(kp, np.float32).reshape(-1, parts, 3)
        out.append(np.float32([kp.shape[0]]))
        out.append(kp.reshape(-1))
        out.append(np.asarray(ks, np.float32).reshape(-1))
    return np.concatenate(out) if out else np.zeros(0, np.float32)
