#!/usr/bin/env python3
"""bench.py -- OpenPose BODY_25 hot path on MI355X: frames/sec, whole node.

Workload (BASELINE.json configs[1], one GPU; configs[2] when launched with --gpus N under
torch.distributed.run): BODY_25 at net_resolution -1x368 on synthetic 1280x720 BGR uint8 frames.
One step = one batch of frames per GPU through the reference's whole per-frame path
(ScaleAndSizeExtractor -> CvMatToOpInput -> PoseExtractorCaffe::forwardPass):
    warpAffine 1280x720 -> 656x368 + normalisation -> CNN forward (114 convs, MFMA fp16 / fp32
    accumulate) -> + people overlay -> resize x8 (78 maps) -> NMS (25 parts) -> PAF line integrals
    -> host people assembly -> keypoints per frame.
Inputs are resident in HBM before timing: uint8 frames (uniform random pixels) and per-frame
5-person overlays (synthetic weights carry no meaning, so a deterministic people field is added to
the net output -- its cost is counted).

Frames shard across ranks with no collective in the data path (frame-parallel replicas, weak
scaling); the only cross-rank traffic is the barrier and the max-reduce of the timer.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec whole-node, BODY_25 -1x368 @1280x720, 1/2/4/8 GPU + CPU ref"
NET_H, NET_W = 368, 656
PRODUCER = (1280, 720)
PEAK_FP16_TFLOPS = 2500.0     # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64,
                    help="frames per step per GPU (throughput mode; DESIGN.md §5 lists 16 too)")
    ap.add_argument("--people", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample")
    return ap.parse_args()


def cpu_baseline(args, params, frames_np, overlays_np):
    """fp32 CPU restatement (oracle/) of the same pipeline on the same uint8 frames: warpAffine +
    normalisation, CNN (im2col + SGEMM, OpenMP), OpenCV-semantics cubic resize, nmsCpu,
    connectBodyPartsCpu."""
    import oracle
    from oracle import body25
    graph = body25.layers()
    t0 = time.perf_counter()
    done = 0
    people = 0
    while True:
        scales, [(nw, nh)] = oracle.scale_and_size(PRODUCER)
        x = oracle.cvmat_to_input(frames_np[done % len(frames_np)], scales[0], nw, nh)[None]
        out = body25.forward(x, params, graph=graph, nthreads=args.cpu_threads)[0]
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
    return {"value": done / el, "unit": "frames/s", "cores": args.cpu_threads, "kind": "port",
            "sample": "%d frame(s) of the full pipeline on 1280x720 frames (warpAffine + CNN fp32 "
                      "at 656x368 + resize + NMS + connector), oracle/ CPU restatement, %.1f s, "
                      "%d people found"
                      % (done, el, people)}


def pmc_traffic(batch):
    """HBM bytes of one CNN forward from the committed rocprofv3 PMC summary (FETCH_SIZE x2 on
    gfx950 + WRITE_SIZE over every kernel of one forward; tools/pmc_summary.py), or None when the
    summary was taken at another batch size."""
    path = os.path.join(ROOT, "profiles", "round1", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return d.get("cnn_forward_hbm_bytes") if d.get("batch") == batch else None


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from openpose_amd import synth
    from openpose_amd.api import Context, Net, PoseExtractor

    ctx = Context(local)
    net = Net(ctx, "builtin:BODY_25")
    convs = net.convs()
    params = synth.he_weights(convs, seed=0, out_scale=0.02)
    net.set_params(params)
    pose = PoseExtractor(ctx, net)

    B = args.batch
    gen = torch.Generator(device="cuda").manual_seed(1234 + rank)
    W_IN, H_IN = PRODUCER
    frames = [torch.randint(0, 256, (B, H_IN, W_IN, 3), generator=gen, device="cuda",
                            dtype=torch.uint8) for _ in range(2)]
    pose.set_input((-1, NET_H))   # --net_resolution -1x368 -> 656x368 for 1280x720
    ov_np = np.stack([synth.overlay(args.people, NET_H // 8, NET_W // 8, seed=1000 * rank + f)
                      for f in range(B)])
    overlay = torch.from_numpy(ov_np).cuda()
    pose.set_overlay(overlay)
    flops_frame = net.flops_per_frame(NET_H, NET_W)
    out_shape = (B, 78, NET_H // 8, NET_W // 8)

    # Two-stage pipeline (opk_pose_submit / opk_pose_collect): the device work of batch i+1 is
    # enqueued before the host assembly of batch i, which then overlaps it.
    def step(i):
        pose.submit_frames(frames[i % 2])
        if pose.pending() > 1:
            pose.collect()

    def drain():
        while pose.pending() > 0:
            pose.collect()

    for i in range(args.warmup):
        step(i)
    drain()
    torch.cuda.synchronize()
    people = [pose.num_people(f) for f in range(B)]
    pose.forward_frames(frames[0])
    out_std = float(net.output_numpy()[:2].std())
    net_in = pose.net_input_numpy()
    assert net_in.shape == (B, 3, NET_H, NET_W)

    # CNN forward time: HIP events recorded by the library around every forward, on the
    # context stream the conv kernels run on (opk_net_set_timing)
    net.set_timing(True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    nfw, fw_ms = net.read_timing()
    net.set_timing(False)
    assert nfw == args.steps, nfw
    net_ms = fw_ms / nfw
    if world > 1:
        t = torch.tensor([elapsed, net_ms], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, net_ms = float(t[0]), float(t[1])

    total_frames = world * B * args.steps
    fps = total_frames / elapsed
    achieved = flops_frame * B / (net_ms * 1e-3) / 1e12
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
        "dtype": "fp16",
        "data": "synthetic uint8 BGR 1280x720 frames (uniform random), random-init weights",
        "config": {
            "workload": "BODY_25 net_resolution -1x368 (net input 656x368) on synthetic 1280x720 "
                        "uint8 frames, %d-person overlay per frame; warpAffine+CNN+resize+NMS+PAF+"
                        "assembly" % args.people,
            "frames_per_step_per_gpu": B,
            "net_input": [NET_H, NET_W],
            "heatmaps": [78, NET_H, NET_W],
            "parallelism": "frame-parallel replicas x%d" % world,
            "compute": "warp u8 fixed-point; conv fp16 x fp16 -> fp32 MFMA; resize/NMS/PAF fp32",
            "people_per_frame_found": people[:4],
            "net_output_std_before_overlay": round(out_std, 5),
        },
        "roofline": {
            "bound": "mfma",
            "kernel": "BODY_25 CNN forward (113 halo implicit-GEMM conv launches + fused first "
                      "conv + 3 pools) per step of %d frames" % B,
            "achieved": round(achieved, 2),
            "peak": PEAK_FP16_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP16_TFLOPS, 4),
            "traffic": pmc_traffic(B),
            "traffic_unit": "bytes per launch (HBM, PMC)",
            "algorithmic_gflop_per_launch": round(flops_frame * B / 1e9, 2),
            "avg_launch_ms": round(net_ms, 3),
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        frames_np = frames[0][:2].cpu().numpy()   # uint8 [2][720][1280][3]
        result["cpu_baseline"] = cpu_baseline(args, params, frames_np, ov_np[:2])
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
