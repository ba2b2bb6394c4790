"""Predicted multi-GPU scaling from one GPU: the per-rank band of the N-GPU bench, rendered alone.

    python tools/band_scaling.py [--precision bf16] [--importance 0] [--steps 5]

bench.py at N GPUs gives rank r the rows D.band(r, N, 600) of each suite view and gathers the
packed tiles to rank 0 (nerf_amd/distributed.py).  This times every rank's band on the one GPU
of this box, one band at a time, with the bench's own frame loop (render_band into the cached
tile, both views of generate_test_poses(2)); the slowest band at N is the compute part of the
N-GPU view time, so t(1 GPU) / t(slowest band) is the scaling the bands allow before the
gather (timed separately at N > 1 in the bench line as exchange_ms_per_frame).  One JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nerf-dbr_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--importance", type=int, default=0, help="128: config 4's 64+128 hierarchical frame")
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()

    import torch

    from nerf_amd import distributed as D
    from nerf_amd import weights as W
    from nerf_amd.benchmark.benchmark_suite import generate_test_poses
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    width, height = 800, 600
    spp = 64 if args.importance else args.spp
    ckpt = W.write_lego_checkpoint(os.path.join(tempfile.mkdtemp(prefix="band_scaling_"), "lego.pth"))
    r = MI355XRenderer(args.precision, n_importance=args.importance, device_index=0)
    r.setup(ckpt)
    poses = generate_test_poses(2)

    def view_ms(r0, r1):
        tile = torch.empty(r1 - r0, width, 4, device="cuda")

        def step():
            for p in poses:
                r.render_band(p, (width, height), spp, r0, r1, tile)

        for _ in range(2):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / (args.steps * len(poses))

    out = {"precision": args.precision, "frame": f"{width}x{height}x{spp}" + (f"+{args.importance}" if args.importance else ""),
           "bands": {}}
    t1 = view_ms(0, height)
    for n in (1, 2, 4, 8):
        ms = [t1] if n == 1 else [view_ms(*D.band(k, n, height)) for k in range(n)]
        out["bands"][str(n)] = {"rank_ms_per_view": [round(m, 3) for m in ms], "slowest_ms": round(max(ms), 3),
                                "speedup_before_gather": round(t1 / max(ms), 3),
                                "efficiency_before_gather": round(t1 / max(ms) / n, 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
