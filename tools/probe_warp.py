"""Probe: the frame warp (opk_cvmat_to_input, 130 x 1280x720 uint8 -> 656x368 fp32) with 1, 2 and
4 destination rows per workgroup (WARP_ROWS), event-timed on the context stream, interleaved."""
import torch

from openpose_amd import api
from openpose_amd.api import Context, dev_switches


def main():
    ctx = Context(0)
    n = 130
    g = torch.Generator(device="cuda").manual_seed(5)
    frames = torch.randint(0, 256, (n, 720, 1280, 3), generator=g, device="cuda", dtype=torch.uint8)
    scales, sizes = api.scale_and_size((1280, 720), (-1, 368), 1.0, 1, 0.25)
    w, h = sizes[0]
    out = torch.empty((n, 3, h, w), device="cuda")
    ref = None
    res = {}
    for rep in range(3):
        for rows in (1, 2, 4):
            with dev_switches(WARP_ROWS=rows):
                for _ in range(3):
                    ctx.cvmat_to_input(out, frames, scales[0])
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    ctx.cvmat_to_input(out, frames, scales[0])
                e.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(e) / 20 * 1e3
                if ref is None:
                    ref = out.clone()
                assert torch.equal(out, ref), rows
                res.setdefault(rows, []).append(us)
                print("rows %d: %.1f us per 130-frame warp" % (rows, us), flush=True)
    print({k: round(min(v), 1) for k, v in res.items()})


if __name__ == "__main__":
    main()
