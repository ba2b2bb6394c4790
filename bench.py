"""Benchmark: rays/s of the MI355X NeRF render path at 800x600, 128 samples/ray.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 it
is launched by torch.distributed.run, one process per GPU (RCCL).  A step is one
``render_image`` of the full 800x600 frame at 128 uniform samples per ray on the
fine network (the reference benchmark's semantics, ``benchmark_suite.py:151-235``;
rays/s = W*H / time, ``:216-220``).  With N GPUs each rank renders its row band and
the bands are all-gathered over RCCL (strong scaling: the frame is fixed).

Rank 0 prints one JSON line.  ``roofline`` is the fine-MLP kernel's algorithmic
FLOP rate (W*H_band*S*1,055,744 FLOP per launch, HIP events on the launch stream)
against the dense MFMA peak of the compute dtype.  ``cpu_baseline`` times the
oracle (a PyTorch-CPU restatement of the reference renderer) on a bounded row band
of the same frame, on this node's host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "nerf-dbr_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3, "fp8": 5000.0}   # MI355X dense MFMA peaks (MI355X_MICROARCH.md)
METRIC = "rays/sec at 800x600x128spp (render_image, fine net, uniform samples)"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--precision", choices=["bf16", "fp32", "fp8"], default="bf16")
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=600)
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample length (0: skip)")
    ap.add_argument("--no-error-check", action="store_true", help="skip the bf16-vs-fp32 error band")
    ap.add_argument("--no-extras", action="store_true", help="skip the other BASELINE configs (C2, C3, C5)")
    return ap.parse_args()


def time_frames(render, n_warm, n_steps):
    """Mean seconds per call of render() (device-synchronised)."""
    import torch

    for _ in range(n_warm):
        render()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_steps):
        render()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n_steps


def other_configs(ckpt, pose, local, ref32):
    """The BASELINE configs besides the headline, 1 GPU each:
    C2 400x300x64 fp32 (the parity path), C3 800x600 64+128 hierarchical bf16,
    C5 800x600x128 fp8."""
    from nerf_amd import weights as W
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    out = {}
    dt = time_frames(lambda: ref32.render_rows(pose, (400, 300), 64, 0, 300), 1, 3)
    out["c2_fp32_400x300x64"] = {"rays_per_s": 400 * 300 / dt, "ms_per_frame": 1e3 * dt}

    h = MI355XRenderer("bf16", n_importance=128, device_index=local)
    h.setup(ckpt)
    h.hip.set_profiling(True)
    dt = time_frames(lambda: h.render_rows(pose, (800, 600), 64, 0, 600), 2, 5)
    st = h.hip.stage_ms()
    flop = 800 * 600 * (64 + 192) * W.FLOPS_PER_SAMPLE
    mlp_ms = st["coarse_mlp"] + st["fine_mlp"]
    out["c3_hierarchical_bf16_800x600_64+128"] = {
        "rays_per_s": 800 * 600 / dt, "ms_per_frame": 1e3 * dt, "stage_ms": st,
        "mlp_tflops": flop / (mlp_ms * 1e-3) / 1e12, "mlp_frac_bf16_peak": flop / (mlp_ms * 1e-3) / 1e12 / 2500.0,
        "samples_per_ray": "64 coarse (coarse net) + 192 fine (fine net on the sorted union)"}

    f8 = MI355XRenderer("fp8", device_index=local)
    f8.setup(ckpt)
    f8.hip.set_profiling(True)
    dt = time_frames(lambda: f8.render_rows(pose, (800, 600), 128, 0, 600), 2, 5)
    ms = f8.hip.stage_ms()["fine_mlp"]
    tf = 800 * 600 * 128 * W.FLOPS_PER_SAMPLE / (ms * 1e-3) / 1e12
    rgb8, d8 = f8.render_rows(pose, (800, 600), 128, 292, 308)
    rgb32, d32 = ref32.render_rows(pose, (800, 600), 128, 292, 308)
    out["c5_fp8_800x600x128"] = {
        "rays_per_s": 800 * 600 / dt, "ms_per_frame": 1e3 * dt, "mlp_kernel_ms": ms, "mlp_tflops": tf,
        "mlp_frac_fp8_peak": tf / PEAK_TFLOPS["fp8"],
        "rgb_max_abs_vs_fp32": float((rgb8 - rgb32).abs().max()),
        "rgb_mean_abs_vs_fp32": float((rgb8 - rgb32).abs().mean()),
        "depth_max_abs_vs_fp32": float((d8 - d32).abs().max())}
    return out


def sharded_hierarchical(ckpt, pose, local, rank, world, width, height, n_warm=2, n_steps=5):
    """C4: 64 coarse + 128 importance samples, bf16, each rank its row band, one
    all-gather per frame; rays/s of the whole frame over the slowest rank."""
    import torch
    import torch.distributed as dist

    from nerf_amd import distributed as D
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    h = MI355XRenderer("bf16", n_importance=128, device_index=local)
    h.setup(ckpt)
    r0, r1 = D.band(rank, world, height)
    rgb_b = torch.empty(r1 - r0, width, 3, device="cuda")
    dep_b = torch.empty(r1 - r0, width, device="cuda")

    def step():
        h.render_rows(pose, (width, height), 64, r0, r1, rgb_b, dep_b)
        D.gather_bands(rgb_b, dep_b, width, height)

    for _ in range(n_warm):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(n_steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    dt = D.reduce_max(time.perf_counter() - t0) / n_steps
    return {"rays_per_s": width * height / dt, "ms_per_frame": 1e3 * dt, "n_gpus": world,
            "samples_per_ray": "64 coarse (coarse net) + 192 fine (fine net on the sorted union)",
            "parallelism": f"row-band x{world} + {dist.get_backend()} all-gather"}


def cpu_baseline(pose, width, height, spp, target_s):
    """Oracle (PyTorch CPU) on a band of rows of the same frame; ~target_s seconds of CPU work."""
    import torch

    from nerf_amd import weights as W
    from oracle import nerf_oracle as O

    _, fine = W.synthetic_models(0)
    net = O.Net(fine)
    r0 = height // 2
    t0 = time.time()
    O.render_image(net, pose, (width, height), spp, rows=(r0, r0 + 2))
    per_row = (time.time() - t0) / 2
    rows = max(2, min(height - r0, int(target_s / max(per_row, 1e-6))))
    t0 = time.time()
    O.render_image(net, pose, (width, height), spp, rows=(r0, r0 + rows))
    dt = time.time() - t0
    cpu = "unknown CPU"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": rows * width / dt, "unit": "rays/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle render_image rows [{r0},{r0 + rows}) of {width}x{height}x{spp} "
                      f"({rows * width} rays, {dt:.1f} s, 512-ray chunks, torch {torch.__version__}, "
                      f"{torch.get_num_threads()} threads on {cpu})"}


def main():
    args = parse()
    # stdout carries exactly one JSON line; the renderers' reference-style
    # progress messages go to stderr
    json_out, sys.stdout = sys.stdout, sys.stderr
    import numpy as np
    import torch
    import torch.distributed as dist

    from nerf_amd import distributed as D
    from nerf_amd import weights as W
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    rank, world, local, dev = D.init_from_env()       # RCCL process group when world > 1
    local = dev

    width, height, spp = args.width, args.height, args.spp
    ckpt_dir = tempfile.mkdtemp(prefix=f"nerf_bench_r{rank}_")
    ckpt = W.write_synthetic_checkpoint(os.path.join(ckpt_dir, "synthetic.pth"), seed=0)
    r = MI355XRenderer(args.precision, device_index=local)
    r.setup(ckpt)
    r.hip.set_profiling(True)

    pose = torch.eye(4)            # benchmark_suite.generate_test_poses view 0
    pose[2, 3] = 4.0
    r0, r1 = D.band(rank, world, height)
    band_rays = (r1 - r0) * width
    rgb_b = torch.empty(r1 - r0, width, 3, device="cuda")
    dep_b = torch.empty(r1 - r0, width, device="cuda")

    def step():
        r.render_rows(pose, (width, height), spp, r0, r1, rgb_b, dep_b)
        if world > 1:
            D.gather_bands(rgb_b, dep_b, width, height)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()                                          # queued back to back: no host sync per frame
    barrier()
    elapsed = D.reduce_max(time.perf_counter() - t0)   # max over ranks
    # the fine-MLP kernel's HIP-event times of the timed frames (the library's
    # per-frame event ring, recorded on the launch stream)
    n_hist = min(args.steps, 64)
    mlp_ms = [f["fine_mlp"] for f in r.hip.stage_ms_history(n_hist)]
    ms_step = 1000.0 * elapsed / args.steps
    value = width * height * args.steps / elapsed

    flop_launch = band_rays * spp * W.FLOPS_PER_SAMPLE
    kern_ms = float(np.mean(mlp_ms))
    traffic, traffic_src = None, None
    kname = f"mlp_{args.precision}_kernel"
    pmc = os.path.join(REPO, "profiles", "pmc_latest.json")
    if os.path.exists(pmc) and (width, height, spp, world) == (800, 600, 128, 1):
        # the headline launch's own counters: profiles/collect.sh profiles the
        # headline bench alone, so every dispatch of this kernel there is this launch
        k = json.load(open(pmc)).get("kernels", {}).get(kname, {})
        if "hbm_bytes_per_launch" in k:
            traffic = k["hbm_bytes_per_launch"]
            traffic_src = (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `{k['command']}` "
                           f"({k['source']}); bytes/launch, FETCH_SIZE x2 (gfx950)")
    achieved = flop_launch / (kern_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.precision]

    extra = {}
    if world > 1 and not args.no_extras:
        # BASELINE config 4: the 64+128 hierarchical frame (bf16), sharded in row
        # bands over every rank and all-gathered -- every rank takes part
        extra["c4_hierarchical_sharded"] = sharded_hierarchical(ckpt, pose, local, rank, world, width, height)
        # per-frame breakdown at N GPUs: the slowest rank's MLP kernel
        # and the exchange alone (the step's packing copies + all-gather), 10 frames
        barrier()
        t_x = time.perf_counter()
        for _ in range(10):
            D.gather_bands(rgb_b, dep_b, width, height)
        barrier()
        extra["exchange_ms_per_frame"] = 1e3 * D.reduce_max(time.perf_counter() - t_x) / 10
        extra["mlp_ms_per_frame_rank_max"] = D.reduce_max(kern_ms)
    ref = None
    if rank == 0 and ((args.precision != "fp32" and not args.no_error_check) or (world == 1 and not args.no_extras)):
        ref = MI355XRenderer("fp32", device_index=local)
        ref.setup(ckpt)
    if rank == 0 and args.precision != "fp32" and not args.no_error_check:
        # bf16 / fp8 vs the fp32 path (itself gated at 1e-4 vs the reference in tests/) on a band
        a0, a1 = height // 2 - 8, height // 2 + 8
        rgb32, d32 = ref.render_rows(pose, (width, height), spp, a0, a1)
        rgb_lp, d_lp = r.render_rows(pose, (width, height), spp, a0, a1)
        extra[f"{args.precision}_vs_fp32_rgb_max_abs"] = float((rgb_lp - rgb32).abs().max())
        extra[f"{args.precision}_vs_fp32_rgb_mean_abs"] = float((rgb_lp - rgb32).abs().mean())
        extra[f"{args.precision}_vs_fp32_depth_max_abs"] = float((d_lp - d32).abs().max())
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ref.render_rows(pose, (width, height), spp, 0, height)
        torch.cuda.synchronize()
        extra["fp32_path_rays_per_s_1gpu"] = width * height / (time.perf_counter() - t1)

    if rank == 0 and world == 1 and not args.no_extras:
        extra["other_configs"] = other_configs(ckpt, pose, local, ref)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(pose, width, height, spp, args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic: conditioned random-init NeRFModel weights (numpy seed 0), suite pose view 0",
            "config": {"workload": f"render_image {width}x{height}, {spp} uniform samples/ray, fine net",
                       "resolution": [width, height], "samples_per_ray": spp,
                       "parallelism": (f"row-band x{world} + "
                                       f"{'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()} all-gather"
                                       if world > 1 else "1 GPU")},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": kname, "kernel_ms": kern_ms,
                         "flop_per_launch": flop_launch},
            "cpu_baseline": cpu,
        }
        out.update(extra)
        print(json.dumps(out), file=json_out, flush=True)
    if world > 1:
        dist.barrier()            # rank 0's extras (error band) finish before any rank tears down
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
