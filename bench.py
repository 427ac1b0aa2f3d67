#!/usr/bin/env python3
"""bench.py -- OpenPose BODY_25 hot path on MI355X: frames/sec, whole node.

Workload (BASELINE.json configs[1] on one GPU; configs[2] with --gpus N): BODY_25 at
net_resolution -1x368 on synthetic 1280x720 BGR uint8 frames.  One step = one batch of frames per
GPU through the reference's whole per-frame path (ScaleAndSizeExtractor -> CvMatToOpInput ->
PoseExtractorCaffe::forwardPass):
    warpAffine 1280x720 -> 656x368 + normalisation -> CNN forward (114 convs, MFMA fp16 / fp32
    accumulate) -> + people overlay -> resize x8 (78 maps) -> NMS (25 parts) -> PAF line integrals
    -> host people assembly -> per-frame keypoint records -> ordered gather to rank 0.
`--config multiscale` runs BASELINE configs[3] instead (--scale_number 4 --scale_gap 0.25: nets at
656x368, 480x272, 320x176, 160x80 per frame, their x8 resizes averaged).  `--config body135` runs
configs[4]: BODY_135 through the poseNetOutput injection path (the reference has no BODY_135
prototxt): synthetic 439 x 46 x 82 net outputs with 20 people per frame -> resize x8 (439 maps) ->
NMS (135 parts) -> PAF integrals (152 pairs) -> connectBodyPartsGpu's global-sort assembly.
Inputs are resident in HBM before timing: uint8 frames (uniform random pixels) and per-frame
5-person overlays (synthetic weights carry no meaning, so a deterministic people field is added to
the net output -- its cost is counted).

Multi-GPU (--gpus N): one process per GPU.  Started under torch.distributed.run the ranks come
from the environment; started directly, this process spawns N ranks (openpose_amd.parallel.
launch_ranks) before any GPU call and waits for them.  Frames shard across ranks with no
collective in the data path (frame-parallel replicas, weak scaling); each rank's per-frame keypoint
records are gathered to rank 0 in frame order (RCCL gather over xGMI, the reference's
WQueueOrderer) inside the timed region -- once at the end of the timed steps by default
(--gather-interval 0: ranks meet only there), or every --gather-interval steps.
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from openpose_amd import parallel  # noqa: E402  (no GPU call at import)

METRIC = "frames/sec whole-node, BODY_25 -1x368 @1280x720, 1/2/4/8 GPU + CPU ref"
NET_H, NET_W = 368, 656
PRODUCER = (1280, 720)
PARTS = 25
PEAK_FP16_TFLOPS = 2500.0     # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0         # MI355X HBM3E (MI355X_MICROARCH.md)
# resizeAndMerge x8 write + NMS read of the 25 part planes per frame at config 2 (SURVEY.md §8d:
# 1,176,864 + 75,319,296 + 24,140,800 + 38,400 bytes): what the reference's post-processing moves
POST_BYTES_FRAME = 100_675_360


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per step per GPU (throughput mode); 0: tile-aligned (body25 / "
                         "multiscale: tile_aligned_batch, 130 on a 256-CU MI355X), 64 for body135")
    ap.add_argument("--config", choices=["body25", "multiscale", "body135"], default="body25",
                    help="body25: BASELINE configs[1]/[2]; multiscale: configs[3] (4 scales); "
                         "body135: configs[4] (BODY_135 net-output injection, 20 people)")
    ap.add_argument("--people", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads; 0: the CPUs this process may run on "
                         "(sched_getaffinity), capped by OMP_NUM_THREADS when the host sets it")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample")
    ap.add_argument("--dump-records", default=None, metavar="NPZ",
                    help="rank 0: write the gathered per-frame records of the timed steps (tests)")
    ap.add_argument("--collective-gather", action="store_true",
                    help="test: at --gpus 1, create the RCCL process group anyway and move the "
                         "records through the collective gather an N-GPU run uses")
    ap.add_argument("--precision", choices=["fp16", "split"], default="fp16",
                    help="body25 / multiscale: the net's arithmetic (opk_net_set_precision): fp16 "
                         "(the product path, the default) or split (fp16 hi/lo pairs, ~fp32 "
                         "results, three MFMA passes per conv)")
    ap.add_argument("--gather-interval", type=int, default=0,
                    help="steps per gather of the per-frame records to rank 0 (N > 1); 0: one gather "
                         "at the end of the timed steps, so ranks are coupled only there")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="the default run (1 GPU, body25, fp16) also times split precision, "
                         "config 4 (multiscale) and config 5 (body135) in child processes and "
                         "reports them under `configs`; this flag skips those legs")
    ap.add_argument("--dev", action="append", default=[], metavar="KEY=VAL",
                    help="kernel-variant switch for A/B runs (opk_dev_set; include/opk.h)")
    return ap.parse_args()


def cpu_share():
    """(threads for the CPU baseline, affinity CPU count, OMP_NUM_THREADS or None).  The GPU box's
    harness sets OMP_NUM_THREADS to the CPU share of one GPU (16) while os.cpu_count() and even the
    affinity mask may show the whole machine; the baseline uses the affinity set, capped by that
    share."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    omp = int(env) if env and env.isdigit() and int(env) > 0 else None
    return (min(aff, omp) if omp else aff), aff, omp


def cgroup_cpu_quota():
    """CPUs' worth of time the process's cgroup allows (cpu.max quota / period, cgroup v2; v1's
    cfs_quota_us / cfs_period_us), or None when unlimited or unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


# the kernel sources behind each group of PMC-derived figures: the CNN forward (traffic, MFMA
# busy) and the post-processing step (overlay add, NMS, PAF: post_roofline)
KERNEL_GROUPS = {
    "cnn": ("conv.h", "conv1_fused.hip", "conv3.hip", "conv3_dev.h", "conv3w.hip", "conv3w8.hip",
            "conv_head.hip", "conv_image.hip", "pool.hip"),
    "post": ("heat_dev.h", "kernels.h", "misc.hip", "nms.hip", "paf.hip", "resize.hip"),
}


def kernel_src_sha(group=None, read=None):
    """sha256 over the kernel sources (openpose_amd/csrc/kernels/*, or one KERNEL_GROUPS group):
    which kernels a committed PMC summary was collected with (tools/pmc_round.sh records the
    digests).  read(name) -> bytes: the sources of another tree (tools/pmc_stamp.py: a commit)."""
    import hashlib
    d = os.path.join(ROOT, "openpose_amd", "csrc", "kernels")
    if read is None:
        def read(name):
            with open(os.path.join(d, name), "rb") as fh:
                return fh.read()
    names = sorted(os.listdir(d)) if group is None else sorted(KERNEL_GROUPS[group])
    h = hashlib.sha256()
    for f in names:
        h.update(f.encode() + b"\0" + read(f))
    return h.hexdigest()[:16]


def pmc_provenance(path, group=None):
    """Commit + kernel-source digest a PMC summary was collected at, and whether the kernels its
    figures describe (`group` of KERNEL_GROUPS, else every kernel) are still the ones running now."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    sha = d.get("kernel_src_sha")
    out = {"source": os.path.relpath(path, ROOT), "pmc_commit": d.get("commit"),
           "kernel_src_sha": sha, "all_kernels_match_this_tree": sha == kernel_src_sha() if sha else None}
    gsha = d.get("%s_kernel_src_sha" % group) if group else None
    if gsha:
        out["kernel_group"] = group
        out["group_kernel_src_sha"] = gsha
        out["kernels_match_this_tree"] = gsha == kernel_src_sha(group)
    else:
        out["kernels_match_this_tree"] = out["all_kernels_match_this_tree"]
    return out


CONTENTS = 4   # distinct synthetic batches: global batch k carries content k % CONTENTS


def contents_of_rank(rank, world, steps=None):
    """Synthetic contents this rank's batches use (global batch index k = step * world + rank, the
    frame ids the ordered gather assigns), so that a frame's input depends only on its global
    frame id: an N-rank run and a 1-rank run over the same frame ids see the same frames."""
    return sorted({(i * world + rank) % CONTENTS for i in range(CONTENTS)})   # period <= CONTENTS


def dump_records(path, ordered):
    """[(keypoints [people, parts, 3], scores [people])] per frame -> npz (tests)."""
    counts = np.array([len(ks) for _, ks in ordered], np.int64)
    kp = np.concatenate([np.asarray(k, np.float32).reshape(-1) for k, _ in ordered] + [np.zeros(0, np.float32)])
    ks = np.concatenate([np.asarray(s, np.float32).reshape(-1) for _, s in ordered] + [np.zeros(0, np.float32)])
    np.savez(path, counts=counts, keypoints=kp, scores=ks)


def tile_aligned_batch(cus, rounds=4):
    """Frames per step that fill whole rounds of 512-position conv tiles at the 1/8-resolution
    level, where 91 of the 3x3 layers run one persistent workgroup per CU: the padded 48 x 84
    image of 46 x 82 is 4,032 positions per frame, so 4 x 256 x 512 // 4032 = 130 frames make
    1,024 tiles = 4 per CU (64 frames make 504: 8 CUs idle in the second round; 66 make 520:
    a third round for 8 CUs, -12 %).  Measured in one call (profiles/round3/batch/): 3,551 /
    3,591 / 3,139 / 3,612 / 3,625 frames/s at 64 / 65 / 66 / 128 / 130 frames."""
    ppf = (NET_H // 8 + 2) * (NET_W // 8 + 2)
    return max(1, rounds * cus * 512 // ppf)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(args, params, frames_np, overlays_np):
    """fp32 CPU restatement (oracle/) of the same pipeline on the same uint8 frames: warpAffine +
    normalisation, CNN (im2col + SGEMM, OpenMP), OpenCV-semantics cubic resize, nmsCpu,
    connectBodyPartsCpu.  Config 2 for ~cpu_seconds, then config 1 (one 368x368 frame)."""
    import oracle
    from oracle import body25
    graph = body25.layers()
    threads = args.cpu_threads
    t0 = time.perf_counter()
    done = 0
    people = 0
    while True:
        scales, [(nw, nh)] = oracle.scale_and_size(PRODUCER)
        x = oracle.cvmat_to_input(frames_np[done % len(frames_np)], scales[0], nw, nh)[None]
        out = body25.forward(x, params, graph=graph, nthreads=threads)[0]
        out = out + overlays_np[done % len(overlays_np)]
        heat = oracle.resize_merge([out], NET_H, NET_W)
        scale = 1.959128
        peaks = oracle.nms(heat, 0.05, 128, (0.5 / scale, 0.5 / scale))
        kp, _ = oracle.connect(heat, peaks, scale=scale)
        people += len(kp)
        done += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds:
            break
    # the same pipeline on every CPU of the affinity mask (the 1-GPU box's harness sets
    # OMP_NUM_THREADS to a 16-CPU share of the node while the mask may hold all of them), reported
    # beside the share's figure
    _, aff, _ = cpu_share()
    full = None
    quota = cgroup_cpu_quota()
    if aff > threads and quota is not None and quota < aff:
        full = {"skipped": True, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                "note": "the process's CPU quota (cgroup cpu.max) is %.1f CPUs: threads beyond it "
                        "time-share those CPUs (measured once on the 1-GPU box, round 5: 0.046 "
                        "frames/s on 256 threads against 1.54 on 16, profiles/round5/r5d/bench.log)"
                        % quota}
    elif aff > threads:
        tf = time.perf_counter()
        nf = 0
        while True:
            scales, [(nw, nh)] = oracle.scale_and_size(PRODUCER)
            x = oracle.cvmat_to_input(frames_np[nf % len(frames_np)], scales[0], nw, nh)[None]
            out = body25.forward(x, params, graph=graph, nthreads=aff)[0]
            out = out + overlays_np[nf % len(overlays_np)]
            heat = oracle.resize_merge([out], NET_H, NET_W)
            peaks = oracle.nms(heat, 0.05, 128, (0.5 / 1.959128, 0.5 / 1.959128))
            oracle.connect(heat, peaks, scale=1.959128)
            nf += 1
            elf = time.perf_counter() - tf
            if elf >= min(args.cpu_seconds, 8.0):
                break
        full = {"value": nf / elf, "unit": "frames/s", "cores": aff,
                "sample": "%d frame(s) of the same config-2 pipeline, %.1f s on %d threads (every CPU "
                          "of the affinity mask)" % (nf, elf, aff)}
    # config 1: one 368x368 frame (net input 368x368, output 46x46), the same stages
    t1 = time.perf_counter()
    x1 = np.random.default_rng(0).uniform(-0.5, 0.5, (1, 3, 368, 368)).astype(np.float32)
    o1 = body25.forward(x1, params, graph=graph, nthreads=threads)[0]
    h1 = oracle.resize_merge([o1], 368, 368)
    p1 = oracle.nms(h1, 0.05, 128, (0.25, 0.25))
    oracle.connect(h1, p1, scale=1.0)
    el1 = time.perf_counter() - t1
    _, aff, omp = cpu_share()
    return {"value": done / el, "unit": "frames/s", "cores": threads, "kind": "port",
            "full_affinity": full, "cgroup_cpu_quota": quota,
            "affinity_cpus": aff, "omp_num_threads_env": omp, "host_cpus": os.cpu_count(),
            "cpu_model": cpu_model(),
            "cores_note": "threads = the CPUs in this process's affinity mask, capped by "
                          "OMP_NUM_THREADS (the CPU share the GPU box allots per GPU) when set",
            "sample": "%d frame(s) of the full config-2 pipeline on 1280x720 frames (warpAffine + "
                      "CNN fp32 at 656x368 + resize + NMS + connector), oracle/ CPU restatement, "
                      "%.1f s on %d threads, %d people found"
                      % (done, el, threads, people),
            "config1": {"value": 1.0 / el1, "unit": "frames/s",
                        "sample": "1 frame, BODY_25 368x368 net input (161.1 GFLOP) + resize + "
                                  "NMS + connector, %.1f s" % el1},
            "published_reference_cpu": "~0.1 FPS BODY_25 CPU-only (doc/06_maximizing_openpose_"
                                       "speed.md:21), other hardware"}


PARITY_FRAMES = 3


def gpu_parity_run(net, pose, convs, frames_u8, precision=0):
    """GPU half of the parity block (outside every timed region, after the bench): the bench's
    first PARITY_FRAMES frames at the bench geometry through the pipeline with FULL-strength heads
    (out_scale 1: the random net drives the maps, no overlay), so fp16-vs-fp32 CNN differences are
    what the post-processing sees.  precision: opk_net_set_precision.  Returns what the CPU leg
    compares against."""
    from openpose_amd import synth
    params = synth.he_weights(convs, seed=0, out_scale=1.0)
    net.set_params(params)
    net.set_precision(precision)
    pose.set_overlay(None)
    pose.forward_frames(frames_u8[:PARITY_FRAMES])
    return {"params": params, "net_input": pose.net_input_numpy(), "net_output": net.output_numpy(),
            "peaks": pose.peaks_numpy(), "keypoints": [pose.keypoints(f)[0] for f in range(PARITY_FRAMES)],
            "scale": pose.scale_net_to_output()}


def split_precision_cost(net, pose, frames_u8, fp16_ms):
    """CNN time of one bench batch in split precision (HIP events, 3 forwards after a warm one),
    against the fp16 forward of the timed steps."""
    from openpose_amd.api import PRECISION_FP16, PRECISION_SPLIT
    net.set_precision(PRECISION_SPLIT)
    pose.forward_frames(frames_u8)
    torch.cuda.synchronize()
    net.set_timing(True)
    for _ in range(3):
        pose.forward_frames(frames_u8)
    k, ms = net.read_timing()
    net.set_timing(False)
    net.set_precision(PRECISION_FP16)
    return {"cnn_ms_per_step": round(ms / k, 3), "fp16_cnn_ms_per_step": round(fp16_ms, 3),
            "relative_cost": round(ms / k / fp16_ms, 3),
            "note": "split precision (opk_net_set_precision OPK_PRECISION_SPLIT): every weight and "
                    "activation an fp16 hi/lo pair, three MFMA passes per conv on the generic conv "
                    "kernel, no fused kernels"}


def cpu_parity(gs, threads):
    """CPU half (the cpu_baseline leg: the fp32 reference path on the same frames, oracle/ +
    oracle/parity.py as the checker): net rel-L2, NMS peak indices identical / within 1 px, the
    largest refined-peak and keypoint shifts, people counts and people reproduced within 1e-3 --
    for every GPU run in gs (one per precision; the fp32 reference computed once).  North star:
    keypoints within 1e-3 of the CPU reference with peak indices bit-exact; this measures it on a
    CNN-driven field."""
    import oracle
    from oracle import body25, parity
    graph = body25.layers()
    g0 = gs[0]
    s = g0["scale"]
    off = float(np.float32(0.5 / np.float64(s)))
    t0 = time.perf_counter()
    refs = []
    for f in range(PARITY_FRAMES):
        ref = body25.forward(g0["net_input"][f:f + 1], g0["params"], graph=graph, nthreads=threads)[0]
        heat_r = oracle.resize_merge([ref], NET_H, NET_W)
        peaks_r = oracle.nms(heat_r, 0.05, 128, (off, off))
        rk, _ = oracle.connect(heat_r, peaks_r, scale=s)
        refs.append((ref, parity.peak_mask(heat_r, 0.05, PARTS), peaks_r, rk))
    outs = []
    for g in gs:
        out = {"frames": PARITY_FRAMES, "workload": "BODY_25 656x368 net input from 1280x720 uint8 "
               "frames, He-init weights with full-strength heads (out_scale 1), no overlay",
               "per_frame": []}
        tot_peaks = tot_same = tot_near = 0
        worst_peak = worst_kp = 0.0
        num = den = 0.0
        for f in range(PARITY_FRAMES):
            ref, mask_r, peaks_r, rk = refs[f]
            got = g["net_output"][f]
            num += float(np.sum((got.astype(np.float64) - ref) ** 2))
            den += float(np.sum(ref.astype(np.float64) ** 2))
            heat_g = oracle.resize_merge([got], NET_H, NET_W)   # = the GPU's lazy maps (bit-exact)
            total, same, near = parity.compare_peaks(mask_r, parity.peak_mask(heat_g, 0.05, PARTS))
            shift = parity.refined_shift(peaks_r, g["peaks"][f])
            kshift, matched = parity.keypoint_shift(rk, g["keypoints"][f], radius=2.0 * s)
            # north star: keypoints within 1e-3 (net-input pixels; keypoints are in frame pixels)
            exact = parity.people_identical(rk, g["keypoints"][f], 1e-3 * s)
            tot_peaks += total
            tot_same += same * total
            tot_near += near * total
            worst_peak = max(worst_peak, shift)
            worst_kp = max(worst_kp, kshift)
            out["per_frame"].append({
                "net_rel_l2": round(float(np.linalg.norm(got - ref) / np.linalg.norm(ref)), 7),
                "fp32_peaks": total, "peak_index_identical": round(same, 5),
                "peaks_within_1px": round(near, 5), "people_gpu": len(g["keypoints"][f]),
                "people_fp32": len(rk), "people_matched_2px": matched,
                "people_identical_1e-3": exact, "max_keypoint_shift_px": round(kshift, 4)})
        out.update({
            "net_rel_l2": round((num / den) ** 0.5, 7),
            "fp32_peaks": tot_peaks,
            "peak_index_identical": round(tot_same / max(tot_peaks, 1), 5),
            "peaks_within_1px": round(tot_near / max(tot_peaks, 1), 5),
            "max_refined_peak_shift_heatmap_px": round(worst_peak, 4),
            "max_keypoint_shift_px": round(worst_kp, 4),
            "people_delta": sum(p["people_gpu"] - p["people_fp32"] for p in out["per_frame"]),
            "people_identical_1e-3_frac": round(sum(p["people_identical_1e-3"] for p in out["per_frame"]) /
                                                max(sum(p["people_fp32"] for p in out["per_frame"]), 1), 5),
            "note": "integer peak sets by nmsCpu's test on each side's own x8 maps; refined-peak "
                    "shift over peaks matched within 1 heat-map px; keypoint shift over people with "
                    "the same parts matched greedily within a 2 net-px mean distance (frame pixels); "
                    "people identical = same parts, every keypoint within 1e-3 net-input px"})
        outs.append(out)
    outs[0]["cpu_seconds"] = round(time.perf_counter() - t0, 1)
    return outs


def host_breakdown(host, steps, collect_times=None):
    """Rank 0's host time in the timed region: per step, the submit call (enqueue), collect (wait
    for the batch + people assembly) and records (pack + gather push); finish (the ordered gather's
    unpack on rank 0) once for the whole run.  collect_times (PoseExtractor.read_collect_times):
    collect split into the wait for the batch's device results and the people assembly, and the
    assembly threads / CPUs this rank had."""
    out = {k: round(v / steps * 1e3, 3) for k, v in host.items() if k != "finish"}
    out["finish_total"] = round(host.get("finish", 0.0) * 1e3, 3)
    if collect_times:
        n = max(collect_times["collects"], 1)
        out["collect_device_wait"] = round(collect_times["wait_ms"] / n, 3)
        out["collect_assembly"] = round(collect_times["assembly_ms"] / n, 3)
        out["assembly_workers"] = collect_times["workers"]
        out["cpus"] = parallel.cpu_ranges(os.sched_getaffinity(0))
    return out


def rank_host_info(dist, host_ms):
    """Every rank's assembly threads and CPU set (rank 0 prints them: disjoint per rank)."""
    mine = {"assembly_workers": host_ms.get("assembly_workers"), "cpus": host_ms.get("cpus"),
            "collect_device_wait": host_ms.get("collect_device_wait"),
            "collect_assembly": host_ms.get("collect_assembly")}
    if dist is None:
        return [mine]
    allr = [None] * dist.get_world_size()
    dist.all_gather_object(allr, mine)
    return allr


def _first(*rel):
    for r in rel:
        p = os.path.join(ROOT, "profiles", r)
        if os.path.exists(p):
            return p
    return os.path.join(ROOT, "profiles", rel[-1])


# Committed rocprofv3 PMC summaries (tools/pmc_round.sh + pmc_report.py + pmc_summary.py; each
# records the commit and kernel-source digest it was collected at, reported beside the numbers
# read from it): CNN HBM bytes per forward, time-weighted MFMA busy, and the post-processing
# kernels' per-step VALU / HBM counts.  Their "batch" must equal the bench's frames per step.
PMC_TRAFFIC = _first("round6/pmc/pmc_traffic.json", "round5/r5f/pmc/pmc_traffic.json", "round4/pmc/pmc_traffic.json")
POST_PMC = _first("round6/pmc/report.json", "round5/r5f/pmc/report.json", "round4/pmc/report.json")
POST_PMC_B135 = _first("round6/pmc_body135/report.json", "round5/r5f/pmc_body135/report.json", "round4/pmc_body135/report.json")
# split precision's CNN (bench.py --precision split): its own counter passes
PMC_SPLIT_TRAFFIC = _first("round6/pmc_split/pmc_traffic.json")
PMC_SPLIT = _first("round6/pmc_split/report.json")


def pmc_traffic(batch, path=PMC_TRAFFIC):
    """HBM bytes of one CNN forward from the committed PMC summary (FETCH_SIZE x2 on gfx950 +
    WRITE_SIZE over every kernel of one forward), or None when it was taken at another batch."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return d.get("cnn_forward_hbm_bytes") if d.get("batch") == batch else None


def pmc_mfma_busy(batch, path=POST_PMC):
    """Time-weighted MFMA busy of the CNN's conv kernels (SQ_VALU_MFMA_BUSY_CYCLES over 1,024
    SIMDs x the cycles each launch ran) from the committed PMC report, or None at another batch."""
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("batch") != batch:
        return None
    return round(d["cnn"]["time_weighted_mfma_busy"], 4)


VALU_PEAK_GINSTS = 1024 * 0.5 * 2.4   # wave64 VALU instructions: 1 per 2 cycles per SIMD-32, 2.4 GHz


def post_roofline(batch, post_ms, pmc_path=POST_PMC, ref_bytes_frame=POST_BYTES_FRAME):
    """Post-processing against its real bound: the PMC VALU wave-instructions and HBM bytes of
    one step's post kernels (committed summary, same batch) over the live HIP-event time.  The
    lazy heat maps mean these kernels move a few % of what the reference's resize + NMS move, so
    the bound is VALU issue / latency, not HBM; the reference-bytes rate is reported separately as
    work avoided, never as a fraction."""
    ref_rate = ref_bytes_frame * batch / (post_ms * 1e-3) / 1e9
    out = {"kernel": "post-processing per step (overlay add + lazy resize/NMS detect + NMS "
                     "finalize + PAF integrals), HIP events on its stream over three "
                     "batches in the single-buffer order (not beside the next nets)",
           "avg_launch_ms": round(post_ms, 3),
           "work_avoided": {"reference_bytes_per_frame": ref_bytes_frame,
                            "reference_bytes_over_time_gbs": round(ref_rate, 1),
                            "note": "the reference's x8 resize write + NMS read per frame over our "
                                    "time; the lazy heat maps never move these bytes (DESIGN.md "
                                    "§4.2), so this is not a roofline fraction"}}
    try:
        with open(pmc_path) as f:
            pmc = json.load(f)["post_step"]
    except (OSError, ValueError, KeyError):
        pmc = None
    try:
        with open(pmc_path) as f:
            pmc_batch = json.load(f).get("batch", 64)
    except (OSError, ValueError):
        pmc_batch = None
    if pmc is None or batch != pmc_batch:
        out.update({"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None,
                    "note": "no PMC summary for this batch size"})
        return out
    valu = pmc["valu_insts"] / (post_ms * 1e-3) / 1e9
    hbm = pmc["hbm_bytes"] / (post_ms * 1e-3) / 1e9
    vf, hf = valu / VALU_PEAK_GINSTS, hbm / PEAK_HBM_GBS
    if vf >= hf:
        out.update({"bound": "valu", "achieved": round(valu, 1), "peak": VALU_PEAK_GINSTS,
                    "unit": "G VALU wave-instructions/s", "frac": round(vf, 4)})
    else:
        out.update({"bound": "hbm", "achieved": round(hbm, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(hf, 4)})
    out.update({"valu_frac": round(vf, 4), "hbm_frac": round(hf, 4),
                "pmc_per_step": {"valu_wave_insts": pmc["valu_insts"], "hbm_bytes": pmc["hbm_bytes"]},
                "pmc_source": pmc_provenance(pmc_path, "post"),
                "note": "neither bound is near its peak: the NMS walk (the largest post kernel) is "
                        "bound by its scalar instruction stream (row tables, taps), DESIGN.md 4.8"})
    return out


def dist_setup(world, local, collective=False):
    """Device and process group of this rank: its own GPU and RCCL.  OPK_BENCH_REHEARSE=1 (dev, a
    1-GPU box): every rank on GPU 0 with gloo, to run the N-rank launcher, the ordered gather in
    the timed loop and the max-over-ranks timing on real hardware (the ranks share the GPU, so the
    throughput of such a run means nothing).  collective (--collective-gather, tests): an RCCL
    group of one rank, so a 1-GPU box runs the N-GPU transport (device gather, all-gather)."""
    rehearse = os.environ.get("OPK_BENCH_REHEARSE") == "1"
    dev = 0 if rehearse else local
    torch.cuda.set_device(dev)
    dist = None
    if world == 1 and collective:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(parallel.free_port()))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", dev))
    elif world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return dev, dist, "cpu" if rehearse and world > 1 else "cuda"


# the legs the default run adds to its JSON line (`configs`): BASELINE.json's other 1-GPU
# configurations and the parity-meeting precision, each a short bench.py run of its own
EXTRA_LEGS = (
    ("split_precision", ["--precision", "split", "--steps", "10", "--warmup", "2"]),
    ("config4_multiscale", ["--config", "multiscale", "--steps", "10", "--warmup", "2"]),
    ("config5_body135", ["--config", "body135", "--steps", "30", "--warmup", "3"]),
)
_TORCHRUN_ENV = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                 "ROLE_WORLD_SIZE", "GROUP_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                 "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS")


def extra_legs(args, timeout=240):
    """Run each EXTRA_LEGS configuration as a child bench.py process on this GPU (started after
    every measurement of this run, which stays idle meanwhile; a child process, not an exec) and
    return {name: summary of its JSON line} -- the driver's one bench line then carries
    driver-observed config-4, config-5 and split-precision throughput."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in _TORCHRUN_ENV}
    out = {}
    for name, extra in EXTRA_LEGS:
        cmd = [sys.executable, "-u", os.path.abspath(__file__), "--gpus", "1", "--no-cpu-baseline",
               "--no-extra-configs"] + extra + sum((["--dev", d] for d in args.dev), [])
        t0 = time.perf_counter()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
        except subprocess.TimeoutExpired:
            out[name] = {"error": "timed out after %d s" % timeout, "args": extra}
            continue
        wall = time.perf_counter() - t0
        line = next((ln for ln in reversed(r.stdout.splitlines()) if ln.startswith("{")), None)
        if r.returncode != 0 or line is None:
            out[name] = {"error": "exit %d" % r.returncode, "args": extra,
                         "stderr_tail": r.stderr[-600:]}
            continue
        d = json.loads(line)
        rf = d.get("roofline") or {}
        leg = {"args": extra, "value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"],
               "steps": d["steps"], "warmup": d["warmup"], "dtype": d["dtype"],
               "frames_per_step": d["config"].get("frames_per_step_per_gpu"),
               "workload": d["config"]["workload"], "process_wall_s": round(wall, 1),
               "roofline": {k: rf.get(k) for k in ("bound", "kernel", "achieved", "peak", "unit", "frac",
                                                   "avg_launch_ms", "algorithmic_gflop_per_launch",
                                                   "mfma_passes_per_useful_flop", "pass_tflops",
                                                   "frac_of_measured_random_operand_mfma", "mfma_busy",
                                                   "traffic")
                            if k in rf},
               "pmc_mfma_busy_source": (rf.get("pmc") or {}).get("mfma_busy"),
               "host_ms": d.get("host_ms")}
        if d.get("post_roofline"):
            pr = d["post_roofline"]
            leg["post_roofline"] = {k: pr.get(k) for k in ("bound", "achieved", "unit", "frac",
                                                           "avg_launch_ms")}
        out[name] = leg
    return out


def rank_main(args, rank, world, local):
    local, dist, comm_dev = dist_setup(world, local, args.collective_gather)

    from openpose_amd import synth
    from openpose_amd.api import Context, Net, PoseExtractor, dev_switches, scale_and_size

    if args.dev:   # A/B runs only; the product configuration has none
        dev_switches(**{k: int(v) for k, v in (d.split("=", 1) for d in args.dev)}).__enter__()

    ctx = Context(local)
    net = Net(ctx, "builtin:BODY_25")
    convs = net.convs()
    params = synth.he_weights(convs, seed=0, out_scale=0.02)
    net.set_params(params)
    if args.precision == "split":
        from openpose_amd.api import PRECISION_SPLIT
        net.set_precision(PRECISION_SPLIT)
    pose = PoseExtractor(ctx, net)

    B = args.batch or tile_aligned_batch(torch.cuda.get_device_properties(local).multi_processor_count)
    nscales = 4 if args.config == "multiscale" else 1
    W_IN, H_IN = PRODUCER
    frames = {}
    for c in contents_of_rank(rank, world, args.steps):
        gen = torch.Generator(device="cuda").manual_seed(1234 + c)
        frames[c] = torch.randint(0, 256, (B, H_IN, W_IN, 3), generator=gen, device="cuda",
                                  dtype=torch.uint8)
    first_content = min(frames)
    pose.set_input((-1, NET_H), scale_number=nscales, scale_gap=0.25)
    _, net_sizes = scale_and_size(PRODUCER, (-1, NET_H), 1.0, nscales, 0.25)
    assert net_sizes[0] == (NET_W, NET_H)
    flops_frame = sum(net.flops_per_frame(h, w) for (w, h) in net_sizes)

    # net-output statistics before any overlay (the overlay is added in place into it)
    pose.forward_frames(frames[first_content])
    out_std = float(net.output_numpy()[:2].std()) if nscales == 1 else None
    # the people field of a frame depends on its global frame id, like its pixels: frame id
    # k * B + f of global batch k (content c = k % CONTENTS) gets overlay seed c * B + f (= the
    # frame id modulo the contents' period), so every step's post-processing sees new fields
    ov_np = {c: np.stack([synth.overlay(args.people, NET_H // 8, NET_W // 8, seed=c * B + f)
                          for f in range(B)]) for c in frames}
    overlays = {c: torch.from_numpy(v).cuda() for c, v in ov_np.items()}

    # per-step ordered gather of the per-frame records (capacity: 4x the synthetic people + 8)
    cap = B * (1 + (4 * args.people + 8) * (PARTS * 3 + 1))
    gather = parallel.RecordGather(world, rank, cap, args.steps, comm_dev,
                                    collective=dist is not None, interval=args.gather_interval)

    # Two-stage pipeline (opk_pose_submit / opk_pose_collect): the device work of batch i+1 is
    # enqueued before the host assembly of batch i, which then overlaps it.
    rec_buf = np.empty(cap, np.float32)
    collected = [0]

    host = {"submit": 0.0, "collect": 0.0, "records": 0.0}   # host seconds in the timed steps

    def collect(timed):
        c0 = time.perf_counter()
        pose.collect()
        if timed:
            c1 = time.perf_counter()
            i = collected[0]
            gather.push(i, (i * world + rank) * B, B, pose.records(rec_buf))
            collected[0] += 1
            host["collect"] += c1 - c0
            host["records"] += time.perf_counter() - c1

    def step(i, timed):
        c = (i * world + rank) % CONTENTS
        s0 = time.perf_counter()
        pose.set_overlay(overlays[c])   # (read at submit; the buffers are never rewritten)
        pose.submit_frames(frames[c])
        if timed:
            host["submit"] += time.perf_counter() - s0
        if pose.pending() > 1:
            collect(timed)

    def drain(timed):
        while pose.pending() > 0:
            collect(timed)

    for i in range(args.warmup):
        step(i, False)
    drain(False)
    torch.cuda.synchronize()
    people = [pose.num_people(f) for f in range(min(B, 4))]

    # CNN forward and post-processing device times: HIP events recorded by the library around
    # every forward / every batch's post-processing, on the context stream the kernels run on
    net.set_timing(True)
    pose.set_timing(True)
    pose.read_collect_times()   # (reset)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, True)
    drain(True)
    collect_times = pose.read_collect_times()
    f0 = time.perf_counter()
    ordered = gather.finish(PARTS)        # rank 0: every frame's record, in frame order
    host["finish"] = time.perf_counter() - f0
    if rank == 0 and args.dump_records:
        dump_records(args.dump_records, ordered)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    nfw, fw_ms = net.read_timing()
    npost, post_ms = pose.read_timing()
    net.set_timing(False)
    pose.set_timing(False)
    # one timed region per forward, or per batch when the scales run on concurrent streams
    assert nfw in (args.steps, args.steps * nscales), nfw
    assert npost == args.steps, npost
    net_ms = fw_ms / args.steps            # all scales of one step
    post_ms /= npost
    # In the timed loop batch i's post-processing runs beside batch i+1's nets (alternating net
    # outputs, PoseHip::next_output), so its event span there includes time-sharing with them.
    # Its own time, the post_roofline's denominator, comes from three more untimed batches in the
    # single-buffer order (each batch's nets wait for the previous post-processing).
    post_overlap_ms = post_ms
    with dev_switches(NET_OUT_ALT=0):
        pose.set_timing(True)
        for i in range(3):
            step(i, False)
        drain(False)
        npost_s, post_s_ms = pose.read_timing()
        pose.set_timing(False)
    post_ms = post_s_ms / npost_s
    per_rank = [[rank, elapsed, net_ms, post_ms]]
    if dist is not None:
        t = torch.tensor([rank, elapsed, net_ms, post_ms], device=comm_dev, dtype=torch.float64)
        allr = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allr, t)
        per_rank = [x.tolist() for x in allr]
        elapsed = max(r[1] for r in per_rank)
        net_ms = max(r[2] for r in per_rank)
        post_ms = max(r[3] for r in per_rank)

    # measured ceilings of this GPU (outside the timed region): the rate the conv instruction
    # reaches from registers on random operands is the attainable MFMA roof under this clock
    peaks = ctx.probe_peaks()

    host_ms = host_breakdown(host, args.steps, collect_times)
    rank_hosts = rank_host_info(dist, host_ms)
    total_frames = world * B * args.steps
    if rank == 0:
        assert len(ordered) == total_frames, (len(ordered), total_frames)
    fps = total_frames / elapsed
    achieved = flops_frame * B / (net_ms * 1e-3) / 1e12
    workload = ("BODY_25 net_resolution -1x368 (net input 656x368) on synthetic 1280x720 uint8 "
                "frames, %d-person overlay per frame; warpAffine+CNN+resize+NMS+PAF+assembly+"
                "ordered gather" % args.people)
    if nscales > 1:
        workload = ("BODY_25 multi-scale --scale_number 4 --scale_gap 0.25 (nets %s) on synthetic "
                    "1280x720 uint8 frames, %d-person overlay; warpAffine x4 + CNN x4 + merged "
                    "resize + NMS + PAF + assembly + ordered gather"
                    % ("/".join("%dx%d" % s for s in net_sizes), args.people))
    result = {
        "metric": METRIC,
        "value": round(fps, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp16" if args.precision == "fp16" else "fp16 hi/lo split (3 MFMA passes)",
        "precision": args.precision,
        "dev_switches": args.dev or None,
        "data": "synthetic uint8 BGR 1280x720 frames (uniform random), random-init weights",
        "config": {
            "workload": workload,
            "frames_per_step_per_gpu": B,
            "net_input": [NET_H, NET_W],
            "net_inputs_all_scales": [[h, w] for (w, h) in net_sizes],
            "heatmaps": [78, NET_H, NET_W],
            "parallelism": ("frame-parallel replicas x%d (one process per GPU, RCCL ordered "
                            "gather of per-frame records to rank 0)" % world) if comm_dev == "cuda"
                           else "REHEARSAL x%d: every rank on GPU 0, gloo gather" % world,
            "compute": ("warp u8 fixed-point; conv fp16 x fp16 -> fp32 MFMA; resize/NMS/PAF fp32"
                        if args.precision == "fp16" else
                        "warp u8 fixed-point; conv as fp16 hi/lo pairs (x_hi w_hi + x_lo w_hi + "
                        "x_hi w_lo -> fp32 MFMA, stored as hi/lo); resize/NMS/PAF fp32"),
            "people_per_frame_found": people,
            "net_output_std_before_overlay": None if out_std is None else round(out_std, 5),
            "frames_gathered_in_order": total_frames,
            "gather_interval_steps": args.gather_interval or "at the end of the timed steps",
        },
        "per_rank": [{"rank": int(r[0]), "s": round(r[1], 4), "cnn_ms_per_step": round(r[2], 3),
                      "post_ms_per_step": round(r[3], 3)} for r in per_rank],
        "roofline": {
            "bound": "mfma",
            "kernel": "BODY_25 CNN forward (113 halo implicit-GEMM conv launches + fused first "
                      "conv + 3 pools) per step of %d frames%s"
                      % (B, "" if nscales == 1 else " x 4 scales"),
            "achieved": round(achieved, 2),
            "peak": PEAK_FP16_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP16_TFLOPS, 4),
            "traffic": (None if nscales != 1 else pmc_traffic(B) if args.precision == "fp16"
                        else pmc_traffic(B, PMC_SPLIT_TRAFFIC)),
            # time-weighted MFMA busy of the conv kernels (PMC; split: over its three passes)
            "mfma_busy": (None if nscales != 1 else pmc_mfma_busy(B) if args.precision == "fp16"
                          else pmc_mfma_busy(B, PMC_SPLIT)),
            "mfma_passes_per_useful_flop": 1 if args.precision == "fp16" else 3,
            # split: the MFMA work issued (three fp16 passes per useful FLOP)
            "pass_tflops": round(achieved * (1 if args.precision == "fp16" else 3), 2),
            "pmc": ({"traffic": pmc_provenance(PMC_TRAFFIC, "cnn"), "mfma_busy": pmc_provenance(POST_PMC, "cnn")}
                    if args.precision == "fp16" else
                    {"traffic": pmc_provenance(PMC_SPLIT_TRAFFIC, "cnn"), "mfma_busy": pmc_provenance(PMC_SPLIT, "cnn")}),
            "traffic_unit": "bytes per launch (HBM, PMC)",
            "algorithmic_gflop_per_launch": round(flops_frame * B / 1e9, 2),
            "avg_launch_ms": round(net_ms, 3),
            "measured_ceilings": peaks,
            "frac_of_measured_random_operand_mfma": round(achieved / peaks["mfma_fp16_random_tflops"], 4),
        },
        "post_roofline": (dict(post_roofline(B, post_ms), overlapped_event_span_ms=round(post_overlap_ms, 3))
                          if nscales == 1 else None),
        "host_ms": host_ms,
        "per_rank_host": rank_hosts,
    }
    if rank == 0 and world == 1 and nscales == 1 and not args.no_cpu_baseline and args.precision == "fp16":
        frames_np = frames[first_content][:2].cpu().numpy()   # uint8 [2][720][1280][3]
        result["cpu_baseline"] = cpu_baseline(args, params, frames_np, ov_np[first_content][:2])
        # keypoint parity at full strength on the same frames, fp16 and split precision, and the
        # cost of split precision (after every measurement: this replaces the net's weights)
        from openpose_amd.api import PRECISION_FP16, PRECISION_SPLIT
        g16 = gpu_parity_run(net, pose, convs, frames[first_content], PRECISION_FP16)
        gsp = gpu_parity_run(net, pose, convs, frames[first_content], PRECISION_SPLIT)
        net.set_precision(PRECISION_FP16)
        p16, psp = cpu_parity([g16, gsp], args.cpu_threads)
        psp["cost"] = split_precision_cost(net, pose, frames[first_content], net_ms)
        p16["precision"] = "fp16 (the measured product path)"
        psp["precision"] = "split (opk_net_set_precision OPK_PRECISION_SPLIT)"
        result["parity"] = dict(p16, split_precision=psp)
    if (rank == 0 and world == 1 and nscales == 1 and args.precision == "fp16" and not args.no_extra_configs
            and not args.dump_records and not args.collective_gather):
        result["configs"] = extra_legs(args)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def rank_main_body135(args, rank, world, local):
    """BASELINE configs[4]: post-processing stress through the injection path (no CNN: the
    reference has no BODY_135 network); frames/s and the post-processing HBM roofline."""
    local, dist, comm_dev = dist_setup(world, local, args.collective_gather)
    from openpose_amd import synth
    from openpose_amd.api import Context, PoseExtractor, dev_switches, pose_model_info
    from openpose_amd.pose_tables import BODY_135, CONNECT_GPU
    if args.dev:   # A/B runs only; the product configuration has none
        dev_switches(**{k: int(v) for k, v in (d.split("=", 1) for d in args.dev)}).__enter__()

    people = 20 if args.people == 5 else args.people
    t = pose_model_info(BODY_135)   # the library's tables (generated from poseParameters.cpp)
    C = t["parts"] + int(t["bkg"]) + len(t["map_idx"])   # 439
    H8, W8 = NET_H // 8, NET_W // 8
    B = args.batch or 64   # no CNN in this config: no tile alignment
    distinct = 8
    fields = np.stack([synth.overlay(people, H8, W8, seed=7000 + k, table=t) +
                       np.random.default_rng(k).normal(0, 0.01, (C, H8, W8)).astype(np.float32)
                       for k in range(distinct)]).astype(np.float32)
    # content c of a global batch (contents_of_rank): frame f holds field (f + 3c) % distinct
    net_out = {c: torch.from_numpy(fields[(np.arange(B) + 3 * c) % distinct]).cuda()
               for c in contents_of_rank(rank, world, args.steps)}
    ctx = Context(local)
    pose = PoseExtractor(ctx, None, pose_model=BODY_135, semantics=CONNECT_GPU)
    parts = t["parts"]
    cap = B * (1 + (4 * people + 8) * (parts * 3 + 1))
    gather = parallel.RecordGather(world, rank, cap, args.steps, comm_dev,
                                    collective=dist is not None, interval=args.gather_interval)
    rec_buf = np.empty(cap, np.float32)
    collected = [0]

    host = {"submit": 0.0, "collect": 0.0, "records": 0.0}   # host seconds in the timed steps

    def collect(timed):
        c0 = time.perf_counter()
        pose.collect()
        if timed:
            c1 = time.perf_counter()
            i = collected[0]
            gather.push(i, (i * world + rank) * B, B, pose.records(rec_buf))
            collected[0] += 1
            host["collect"] += c1 - c0
            host["records"] += time.perf_counter() - c1

    def step(i, timed):
        s0 = time.perf_counter()
        pose.submit_net_output(net_out[(i * world + rank) % CONTENTS], (NET_W, NET_H), PRODUCER)
        if timed:
            host["submit"] += time.perf_counter() - s0
        if pose.pending() > 1:
            collect(timed)

    def drain(timed):
        while pose.pending() > 0:
            collect(timed)

    for i in range(args.warmup):
        step(i, False)
    drain(False)
    torch.cuda.synchronize()
    found = [pose.num_people(f) for f in range(min(B, 4))]
    pose.set_timing(True)
    pose.read_collect_times()   # (reset)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, True)
    drain(True)
    collect_times = pose.read_collect_times()
    f0 = time.perf_counter()
    ordered = gather.finish(parts)
    host["finish"] = time.perf_counter() - f0
    if rank == 0 and args.dump_records:
        dump_records(args.dump_records, ordered)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    npost, post_ms = pose.read_timing()
    pose.set_timing(False)
    post_ms /= max(npost, 1)
    if dist is not None:
        tt = torch.tensor([elapsed, post_ms], device=comm_dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, post_ms = float(tt[0]), float(tt[1])
    host_ms = host_breakdown(host, args.steps, collect_times)
    rank_hosts = rank_host_info(dist, host_ms)
    total_frames = world * B * args.steps
    if rank == 0:
        assert len(ordered) == total_frames, (len(ordered), total_frames)
    # what the reference's post-processing moves per frame: the x8 resize
    # of all 439 maps (read + write) and the NMS read of the 135 part planes (+ its peaks)
    post_bytes = (4 * C * H8 * W8 + 4 * C * NET_H * NET_W + 4 * parts * NET_H * NET_W +
                  4 * parts * 128 * 3)
    result = {
        "metric": METRIC,
        "value": round(total_frames / elapsed, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic BODY_135 net outputs (%d-person fields + N(0, 0.01) noise), resident "
                "in HBM" % people,
        "config": {
            "workload": "BODY_135 (135 keypoints) poseNetOutput injection, 439x46x82 net output "
                        "per frame for a 1280x720 producer, %d people per frame; resize x8 + NMS "
                        "+ PAF integrals + connectBodyPartsGpu assembly + ordered gather" % people,
            "frames_per_step_per_gpu": B,
            "heatmaps": [C, NET_H, NET_W],
            "parallelism": ("frame-parallel replicas x%d (one process per GPU, RCCL ordered "
                            "gather of per-frame records to rank 0)" % world) if comm_dev == "cuda"
                           else "REHEARSAL x%d: every rank on GPU 0, gloo gather" % world,
            "people_per_frame_found": found,
            "frames_gathered_in_order": total_frames,
            "gather_interval_steps": args.gather_interval or "at the end of the timed steps",
        },
        "roofline": dict(post_roofline(B, post_ms, POST_PMC_B135, post_bytes), traffic=None),
        "host_ms": host_ms,
        "per_rank_host": rank_hosts,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle   # the CPU baseline leg only
        t_orc = oracle.pose_tables()[BODY_135]
        t1 = time.perf_counter()
        done = 0
        while True:
            heat = oracle.resize_merge([fields[done % distinct]], NET_H, NET_W)
            scale = 1.959128
            off = 0.5 / scale
            peaks = oracle.nms(heat, 0.05, 128, (off, off), channels=parts)
            ps = oracle.pair_scores_table(heat, peaks, t_orc)
            oracle.connect_gpu_semantics(ps, peaks, t_orc, scale=scale)
            done += 1
            el = time.perf_counter() - t1
            if el >= min(args.cpu_seconds, 10.0):
                break
        result["cpu_baseline"] = {
            "value": done / el, "unit": "frames/s", "cores": 1, "kind": "port",
            "affinity_cpus": cpu_share()[1], "host_cpus": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": "%d frame(s): oracle/ resize (439 maps) + NMS + pair scores + GPU-path "
                      "assembly, %.1f s, single-threaded" % (done, el)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.cpu_threads <= 0:
        args.cpu_threads = cpu_share()[0]
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # direct start with --gpus N: one child process per GPU, this process touches no GPU
        sys.exit(parallel.launch_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    # several ranks on this node: each keeps to its GPU-local share of the host CPUs (before any
    # thread or GPU call), so the ranks' people-assembly threads never share cores
    parallel.pin_rank_cpus(local, int(os.environ.get("LOCAL_WORLD_SIZE", world)))
    if args.config == "body135":
        rank_main_body135(args, rank, world, local)
    else:
        rank_main(args, rank, world, local)


if __name__ == "__main__":
    main()
