"""Frame-parallel multi-GPU runtime: one process per GPU, frames sharded, results re-ordered.

Reference behaviour: one PoseExtractorCaffe + worker thread per GPU pulling
frames from a shared queue (include/openpose/wrapper/wrapperAuxiliary.hpp:328-337,1050-1067) and a
WQueueOrderer that re-sequences results by frame id (include/openpose/thread/wQueueOrderer.hpp:
62-141).  Here: one process per GPU under torch.distributed (RCCL on the GPU box, gloo on CPU),
frames assigned to ranks in contiguous blocks (no data-path collective: every rank runs the whole
hot path on its own frames), and the per-frame keypoint records gathered to rank 0 in frame order
(the only collective; a few KB per frame).
"""
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
