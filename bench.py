"""Benchmark: rays/s of the MI355X NeRF render path at 800x600, 128 samples/ray.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 it
runs one process per GPU (RCCL): launched by torch.distributed.run, or, when started
plainly (no WORLD_SIZE in the environment), it starts torch.distributed.run itself as
a child process and relays rank 0's line (``self_launch``).  A step is one
``render_image`` of the full 800x600 frame at 128 uniform samples per ray on the
fine network for each of the suite's two views (``generate_test_poses(2)``; the
reference benchmark's semantics, ``benchmark_suite.py:151-235``; rays/s = W*H / the
mean view time, ``:188-220``).  With N GPUs each rank renders its row band
into a packed [rows, W, 4] tile (``nerf_render_band``) and the tiles are gathered
to rank 0 over RCCL (strong scaling: the frame is fixed).

Rank 0 prints one JSON line.  ``roofline`` is the fine-MLP kernel's algorithmic
FLOP rate (W*H_band*S*1,055,744 FLOP per launch, HIP events on the launch stream)
against the dense MFMA peak of the compute dtype.  ``readme_grid`` times the
reference README's resolution x samples grid for bf16, fp8 and fp32 with the same
step (band + gather at N > 1), each cell with its fractions of the MFMA roofline.
``cpu_baseline`` times the oracle (a PyTorch-CPU restatement of the reference
renderer) on this node's host cores with the suite's protocol (2 views of
``generate_test_poses(2)``), on bounded samples of three cells.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from datetime import timedelta

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "nerf-dbr_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

# MI355X dense MFMA peaks (MI355X_MICROARCH.md).  bf16x3 / f16x3 run three 16-bit MFMAs
# per product (W_hi.X_hi + W_hi.X_lo + W_lo.X_hi), so their algorithmic ceiling is a
# third of the bf16 (= f16) peak.
# fp8 (round 5) is mixed: 393,216 of a sample's 527,872 MACs on the fp8 MFMA (5 PF), the other
# 134,656 (L0, L1, L4's encoding inputs, C0, heads) on the bf16 MFMA (2.5 PF), so its ceiling
# is 527,872 / (134,656 / 2.5 + 393,216 / 5) = 3.98 PFLOP/s (mlp_fp8.hip); the C5 line also
# reports the fraction of the plain fp8 peak.
FP8_MIX_MACS = {"bf16": 134656, "fp8": 393216}
FP8_MIX_CEILING = 527872 / (FP8_MIX_MACS["bf16"] / 2500.0 + FP8_MIX_MACS["fp8"] / 5000.0)
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3, "fp8": FP8_MIX_CEILING, "bf16x3": 2500.0 / 3, "f16x3": 2500.0 / 3}
METRIC = "rays/sec at 800x600x128spp (render_image, fine net, uniform samples)"
GRID_RES = [(200, 150), (400, 300), (800, 600)]                 # reference main.py:134-141
GRID_SPP = [32, 64, 128]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--precision", choices=["bf16", "fp32", "fp8", "bf16x3", "f16x3"], default="bf16")
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=600)
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--cpu-seconds", type=float, default=30.0, help="total CPU-baseline budget (0: skip)")
    ap.add_argument("--no-error-check", action="store_true", help="skip the headline path's whole-frame error vs the reference")
    ap.add_argument("--no-extras", action="store_true", help="skip the other BASELINE configs and the grid")
    ap.add_argument("--no-grid", action="store_true", help="skip the README resolution x spp grid")
    ap.add_argument("--no-train", action="store_true", help="skip the training-step leg")
    ap.add_argument("--train-steps", type=int, default=10)
    ap.add_argument("--launch-check", action="store_true",
                    help="no GPU work: form the process group (gloo), and rank 0 prints the line's "
                         "launch fields (tests the N > 1 launch contract on CPU)")
    return ap.parse_args()


def self_launch(argv, n_gpus):
    """``python bench.py --gpus N ...`` with no torchrun environment: start
    ``torch.distributed.run --nproc-per-node N`` on this same script as a CHILD process
    (never an exec: nothing here has touched the GPU, and the ranks initialise it in
    their own processes), relay rank 0's JSON line to stdout, everything else to
    stderr, and return the child's exit code."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n_gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    print(f"bench.py: WORLD_SIZE unset with --gpus {n_gpus}; launching {' '.join(cmd)}", file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    lines = []
    for line in proc.stdout:
        if line.lstrip().startswith("{"):
            lines.append(line.strip())
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = proc.wait()
    for line in lines:
        print(line, flush=True)
    return rc


def launch_check(args):
    """The launch contract without a GPU: the ranks form a gloo group, count themselves with
    one all-reduce, and rank 0 prints one line with the fields the driver reads."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.ones(1)
        dist.all_reduce(t)
        world = int(t.item())
    # the line's host-side fields at this N: the band-scaled traffic and the CPU baseline (run
    # with the same rank protocol as a real N > 1 bench, at --cpu-seconds)
    from nerf_amd import distributed as D

    r0, r1 = D.band(rank, world, args.height)
    kname = {"bf16x3": "mlp_x3_kernel<OpBf16>", "f16x3": "mlp_x3_kernel<OpF16>"}.get(args.precision,
                                                                                    f"mlp_{args.precision}_kernel")
    traffic, traffic_src = launch_traffic(kname, args.width, args.height, args.spp, world, (r1 - r0) * args.width)
    cpu = ranked_cpu_baseline(rank, world, args.cpu_seconds)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "rays/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "launch_check": True,
                          "launched_by": "self" if os.environ.get("NERF_BENCH_SELF_LAUNCHED") else "external",
                          "roofline": {"kernel": kname, "traffic": traffic, "traffic_source": traffic_src},
                          "cpu_baseline": cpu}),
              flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


# ------------------------------------------------------------------ helpers --
def sync_barrier(world):
    import torch
    import torch.distributed as dist

    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def frame_step(r, poses, width, height, spp, rank, world):
    """One step of renderer r as the benchmark runs it: one frame per pose of ``poses``
    (the suite's protocol, benchmark_suite.py:188-220: both views of
    generate_test_poses(2), rays/s = W*H / the mean view time), each the whole frame at
    N = 1 (render_rows, the plugin's render_image path), else this rank's band rendered
    into the packed tile and gathered to rank 0.  Returns (step, rays in this band per
    frame); a step is len(poses) frames."""
    import torch

    from nerf_amd import distributed as D

    r0, r1 = D.band(rank, world, height)
    if world == 1:
        rgb = torch.empty(height, width, 3, device="cuda")
        dep = torch.empty(height, width, device="cuda")

        def step():
            for pose in poses:
                r.render_rows(pose, (width, height), spp, 0, height, rgb, dep)

        return step, width * height
    tile = D.band_tile(world, height, width, r.torch_device())

    def step():
        for pose in poses:
            r.render_band(pose, (width, height), spp, r0, r1, tile)
            D.gather_tiles_to_root(tile, width, height)

    return step, (r1 - r0) * width


def per_view_ms(r, n_views, n_frames, stage="fine_mlp"):
    """Mean HIP-event time of a stage per view over the last n_frames frames, which
    alternate over the views in order."""
    import numpy as np

    hist = r.hip.stage_ms_history(min(n_frames, 64))
    off = (-len(hist)) % n_views            # align the history's first frame with view 0
    return [float(np.mean([f[stage] for f in hist[v + off::n_views]])) for v in range(n_views)]


def check_gathered(r, pose, width, height, spp, rank, world):
    """Outside any timed region: every rank renders its band into the packed tile, the tiles
    are gathered to rank 0, and rank 0 renders the whole frame alone with the same renderer;
    the two must agree bit for bit (a ray's result does not depend on which band it is in).
    Returns the verdict on rank 0, None elsewhere."""
    import torch

    from nerf_amd import distributed as D

    r0, r1 = D.band(rank, world, height)
    tile = D.band_tile(world, height, width, r.torch_device())
    r.render_band(pose, (width, height), spp, r0, r1, tile)
    frame = D.gather_tiles_to_root(tile, width, height, copy=True)
    if rank != 0:
        return None
    rgb = torch.empty(height, width, 3, device=r.torch_device())
    dep = torch.empty(height, width, device=r.torch_device())
    r.render_rows(pose, (width, height), spp, 0, height, rgb, dep)
    torch.cuda.synchronize()
    return {"gathered_equals_single": bool(torch.equal(frame[..., :3], rgb) and torch.equal(frame[..., 3], dep)),
            "rgb_max_abs": float((frame[..., :3] - rgb).abs().max()),
            "depth_max_abs": float((frame[..., 3] - dep).abs().max()),
            "check": f"rank 0 rendered {width}x{height}x{spp}" + (f"+{r.n_importance}" if r.n_importance else "")
                     + f" ({r.precision}) alone vs the {world} gathered band tiles"}


def dist_record():
    """The process group as it formed: backend, world size and the RCCL version."""
    import torch
    import torch.distributed as dist

    rec = {"backend": dist.get_backend(), "world_size": dist.get_world_size()}
    if rec["backend"] == "nccl":
        try:
            rec["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
        except Exception as e:            # noqa: BLE001 -- informational only
            rec["rccl_version"] = f"unavailable: {e}"
    return rec


class ClockSampler:
    """The GPU's graphics clock, power and hotspot temperature sampled with amdsmi every
    ``period`` seconds in a thread while the timed frames run (so clock drift between runs
    is attributable).  Fails soft: without amdsmi, or without access, ``summary()`` says why."""

    KEYS = ("current_gfxclks", "current_gfxclk", "average_gfxclk_frequency", "current_socket_power",
            "average_socket_power", "temperature_hotspot")

    def __init__(self, device_index, period=0.02):
        import threading

        self.period, self.samples, self.error = period, [], None
        self._stop = threading.Event()
        self._thread = None
        try:
            import amdsmi
            import torch

            amdsmi.amdsmi_init()
            self._smi = amdsmi
            handles = amdsmi.amdsmi_get_processor_handles()
            props = torch.cuda.get_device_properties(device_index)
            want = (getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", None))
            self._h = None
            for h in handles:
                dom, rest = amdsmi.amdsmi_get_gpu_device_bdf(h).split(":", 1)
                if (int(dom, 16), int(rest.split(":")[0], 16)) == want:
                    self._h = h
            if self._h is None and len(handles) == 1:
                self._h = handles[0]
            if self._h is None:
                raise RuntimeError(f"no amdsmi handle matches PCI {want} among {len(handles)}")
            self._thread = threading.Thread(target=self._run, daemon=True)
        except Exception as e:            # noqa: BLE001 -- telemetry is optional
            self.error = f"{type(e).__name__}: {e}"

    def _read(self):
        out = {}
        try:
            m = self._smi.amdsmi_get_gpu_metrics_info(self._h)
            for k in self.KEYS:
                v = m.get(k)
                if isinstance(v, (list, tuple)):
                    v = [x for x in v if isinstance(x, (int, float)) and 0 < x < 65535]
                    v = sum(v) / len(v) if v else None
                if isinstance(v, (int, float)) and 0 < v < 65535:
                    out[k] = float(v)
        except Exception as e:            # noqa: BLE001
            self.error = f"{type(e).__name__}: {e}"
        return out

    def _run(self):
        import time as _t

        while not self._stop.is_set():
            r = self._read()
            if r:
                self.samples.append(r)
            _t.sleep(self.period)

    def __enter__(self):
        if self._thread is not None:
            self._thread.start()
        return self

    def __exit__(self, *exc):
        if self._thread is not None:
            self._stop.set()
            self._thread.join(timeout=5)

    def summary(self):
        out = {"source": "amdsmi_get_gpu_metrics_info", "samples": len(self.samples), "period_s": self.period}
        if self.error:
            out["error"] = self.error
        for k in self.KEYS:
            v = [smp[k] for smp in self.samples if k in smp]
            if v:
                out[k] = {"mean": sum(v) / len(v), "min": min(v), "max": max(v)}
        return out


def time_steps(step, n_warm, n_steps, world):
    """Max over ranks of the mean seconds per step (barrier + synchronize both sides)."""
    from nerf_amd import distributed as D

    for _ in range(n_warm):
        step()
    sync_barrier(world)
    t0 = time.perf_counter()
    for _ in range(n_steps):
        step()
    sync_barrier(world)
    return D.reduce_max(time.perf_counter() - t0) / n_steps


def kernel_ms(r, n, stage="fine_mlp"):
    """Mean HIP-event time of a stage over the last n frames of renderer r."""
    import numpy as np

    return float(np.mean([f[stage] for f in r.hip.stage_ms_history(min(n, 64))]))


# ------------------------------------------------------------ README grid --
def readme_grid(renderers, poses, rank, world):
    """rays/s on {200x150, 400x300, 800x600} x {32, 64, 128} spp for each precision,
    on the suite's two views (rays/s = W*H / mean view time), with the fractions of the
    MFMA roofline: ``frac_frame`` = whole-job FLOP rate / (N x peak), ``frac_kernel`` =
    the slowest rank's fine-MLP kernel rate / peak."""
    from nerf_amd import distributed as D
    from nerf_amd import weights as W

    out = {}
    for prec, r in renderers.items():
        peak = PEAK_TFLOPS[prec]
        rows = {}
        for (w, h) in GRID_RES:
            for spp in GRID_SPP:
                step, band_rays = frame_step(r, poses, w, h, spp, rank, world)
                n = 1 if prec in ("fp32", "bf16x3", "f16x3") and w * h * spp >= 400 * 300 * 128 else 2
                dt = time_steps(step, 1, n, world) / len(poses)
                r.check_range()
                kms = D.reduce_max(kernel_ms(r, n * len(poses)))
                flop = w * h * spp * W.FLOPS_PER_SAMPLE
                rows[f"{w}x{h}x{spp}"] = {
                    "rays_per_s": w * h / dt, "ms_per_frame": 1e3 * dt,
                    "frac_frame": flop / dt / 1e12 / (world * peak),
                    "frac_kernel": band_rays * spp * W.FLOPS_PER_SAMPLE / (kms * 1e-3) / 1e12 / peak,
                    "kernel_ms": kms}
        out[prec] = rows
    return out


GOLDEN = os.path.join(REPO, "tests", "golden")
FIXTURES = {  # whole frames rendered by the reference (tests/golden/make_golden.py)
    "headline": "render_lego_800x600_s128_full.npz",   # PyTorchCPURenderer.render_image, 800x600x128
    "c3": "render_lego_800x600_c3_full.npz",           # reference pieces + fixed-gather sampler, 64+128
}
TRUTH = {"c3": "render_lego_800x600_c3_fp64.npz"}      # the same C3 chain in float64


def truth_error(rgb, dep, t_rgb, t_dep):
    """One frame against the float64 truth: max RGB / depth error, pixels over 1e-4."""
    import numpy as np

    e_rgb = np.abs(np.asarray(rgb, np.float64) - t_rgb).max(-1)
    e_dep = np.abs(np.asarray(dep, np.float64) - t_dep)
    return {"rgb_max_abs": float(e_rgb.max()), "depth_max_abs": float(e_dep.max()),
            "pixels_over_1e-4": int(((e_rgb >= 1e-4) | (e_dep >= 1e-4)).sum())}


def errors_vs_reference(r, which="headline"):
    """Outside any timed region: renderer r renders every pose of the reference's whole-frame
    fixture (``FIXTURES[which]``) into NaN-filled outputs, and each frame is compared with the
    reference's pixels: max and mean RGB error, max depth error, the pixels whose RGB or depth
    error exceeds the 1e-4 gate, and those whose depth moves by more than 1e-2 (the single-pixel
    flips of a last sample with sigma ~ 0, BASELINE.json's "RGB max-abs err" next to rays/s)."""
    import numpy as np
    import torch

    path = os.path.join(GOLDEN, FIXTURES[which])
    if not os.path.exists(path):
        return {"error": f"fixture missing: {os.path.relpath(path, REPO)}"}
    g = np.load(path)
    w, h = int(g["W"]), int(g["H"])
    spp = int(g["S"]) if "S" in g else int(g["S_coarse"])
    out = {"reference": os.path.relpath(path, REPO), "views": []}
    tpath = os.path.join(GOLDEN, TRUTH[which]) if which in TRUTH else None
    t = np.load(tpath) if tpath and os.path.exists(tpath) else None
    if t is not None:
        out["truth"] = os.path.relpath(tpath, REPO)
    for k, pid in enumerate(g["pose_ids"]):
        rgb = torch.full((h, w, 3), float("nan"), device=r.torch_device())
        dep = torch.full((h, w), float("nan"), device=r.torch_device())
        r.render_rows(torch.from_numpy(g["poses"][k]), (w, h), spp, 0, h, rgb, dep)
        r.check_range()
        torch.cuda.synchronize()
        e_rgb = np.abs(rgb.cpu().numpy() - g[f"rgb_{k}"])
        e_dep = np.abs(dep.cpu().numpy() - g[f"depth_{k}"])
        out["views"].append({"pose_id": int(pid), "rgb_max_abs": float(e_rgb.max()), "rgb_mean_abs": float(e_rgb.mean()),
                             "depth_max_abs": float(e_dep.max()),
                             "pixels_over_1e-4": int(((e_rgb.max(-1) >= 1e-4) | (e_dep >= 1e-4)).sum()),
                             "depth_pixels_gt_1e-2": int((e_dep > 1e-2).sum()), "pixels": int(e_dep.size)})
        if t is not None:
            out["views"][-1]["vs_fp64"] = {
                "this_render": truth_error(rgb.cpu().numpy(), dep.cpu().numpy(), t[f"rgb_{k}"], t[f"depth_{k}"]),
                "reference_fp32_chain": truth_error(g[f"rgb_{k}"], g[f"depth_{k}"], t[f"rgb_{k}"], t[f"depth_{k}"])}
    v = out["views"]
    out["rgb_max_abs_vs_reference"] = max(x["rgb_max_abs"] for x in v)
    out["rgb_mean_abs_vs_reference"] = float(np.mean([x["rgb_mean_abs"] for x in v]))
    out["depth_max_abs_vs_reference"] = max(x["depth_max_abs"] for x in v)
    out["depth_pixels_gt_1e-2"] = sum(x["depth_pixels_gt_1e-2"] for x in v)
    out["pixels_over_1e-4"] = sum(x["pixels_over_1e-4"] for x in v)
    if t is not None:
        out["vs_fp64"] = {who: {"pixels_over_1e-4": sum(x["vs_fp64"][who]["pixels_over_1e-4"] for x in v),
                                "rgb_max_abs": max(x["vs_fp64"][who]["rgb_max_abs"] for x in v),
                                "depth_max_abs": max(x["vs_fp64"][who]["depth_max_abs"] for x in v)}
                          for who in ("this_render", "reference_fp32_chain")}
    return out


def int8_renderer_error():
    """The reference's int8 CompressedNeRFRenderer (compressed_renderer.py:161-358) on whole
    800x600x128 Lego frames against the reference's fp32 render, from the two fixtures
    (make_golden_compressed.py --lego-full, make_golden.py --lego-full): config 5's error bar,
    beside the fp8 line's own error on the same views."""
    import numpy as np

    pc, pf = os.path.join(GOLDEN, "compressed_lego_800x600_s128.npz"), os.path.join(GOLDEN, FIXTURES["headline"])
    if not (os.path.exists(pc) and os.path.exists(pf)):
        return {"error": "fixture missing"}
    gc, g = np.load(pc), np.load(pf)
    views = []
    for kc, pid in enumerate(gc["pose_ids"]):
        kg = int(np.flatnonzero(g["pose_ids"] == pid)[0])
        e = np.abs(gc[f"rgb_{kc}"] - g[f"rgb_{kg}"])
        d = np.abs(gc[f"depth_{kc}"] - g[f"depth_{kg}"])
        views.append({"pose_id": int(pid), "rgb_max_abs": float(e.max()), "rgb_mean_abs": float(e.mean()),
                      "depth_pixels_gt_1e-2": int((d > 1e-2).sum())})
    return {"reference": os.path.relpath(pc, REPO), "views": views}


def original_nerf_leg(poses, local, precision):
    """The reference's own bundled Lego networks (the original NeRF implementation's layout,
    data/lego_example_weights) on the fp32 or split-fp16 kernel
    (NERF_LAYOUT_ORIGINAL_NERF): rays/s at 800x600x128 on the suite's two views."""
    from nerf_amd import weights as W
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer
    from tools.lego import teacher as T

    if not all(os.path.exists(os.path.join(REPO, "tools", "lego", f"_teacher_{w}.npz")) for w in ("coarse", "fine")) \
            and not os.path.isdir(T.LEGO_DIR):
        return {"error": "tools/lego/_teacher_*.npz missing (written by __graft_entry__.build())"}
    r = MI355XRenderer(precision, device_index=local)
    r.setup_original_nerf(T.load_arrays("coarse"), T.load_arrays("fine"))
    r.hip.set_profiling(True)
    step, _ = frame_step(r, poses, 800, 600, 128, 0, 1)
    dt = time_steps(step, 1, 2, 1) / len(poses)
    ms = kernel_ms(r, 2 * len(poses))
    r.check_range()
    flop = 800 * 600 * 128 * W.FLOPS_PER_SAMPLE
    return {"rays_per_s": 800 * 600 / dt, "ms_per_frame": 1e3 * dt, "mlp_kernel_ms": ms,
            "mlp_frac_of_peak": flop / (ms * 1e-3) / 1e12 / PEAK_TFLOPS[precision],
            "peak": f"{PEAK_TFLOPS[precision]:.1f} TFLOP/s ({precision})",
            "parity": "tests/test_gpu_lego_original.py: whole 200x150x32 frames and an 800x600x128 band within 1e-4 "
                      "of the same networks restated on the CPU (tools/lego/teacher.py)",
            "network": "original NeRF layout (skip into layer 5, no-pi encodings, normalised view directions, "
                       "feature layer folded into the views layer), the reference's data/lego_example_weights"}


def other_configs(ckpt, poses, local, ref32):
    """The BASELINE configs besides the headline, 1 GPU each, each on the
    suite's two views (rays/s = W*H / mean view time): C2 400x300x64 fp32 (the parity
    path), C3 800x600 64+128 hierarchical bf16, C5 800x600x128 fp8."""
    from nerf_amd import weights as W
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    nv = len(poses)
    out = {}
    step, _ = frame_step(ref32, poses, 400, 300, 64, 0, 1)
    dt = time_steps(step, 1, 2, 1) / nv
    out["c2_fp32_400x300x64"] = {"rays_per_s": 400 * 300 / dt, "ms_per_frame": 1e3 * dt}
    # C2 and the headline frame on the split-fp16 path, the parity-grade fast path held to
    # the same 1e-4 gate as fp32 on the Lego fixtures (tests/test_gpu_lego.py)
    x3 = MI355XRenderer("f16x3", device_index=local)
    x3.setup(ckpt)
    x3.hip.set_profiling(True)
    step, _ = frame_step(x3, poses, 400, 300, 64, 0, 1)
    dt = time_steps(step, 1, 2, 1) / nv
    out["c2_f16x3_400x300x64"] = {"rays_per_s": 400 * 300 / dt, "ms_per_frame": 1e3 * dt}
    step, _ = frame_step(x3, poses, 800, 600, 128, 0, 1)
    dt = time_steps(step, 1, 2, 1) / nv
    ms = kernel_ms(x3, 2 * nv)
    views_ms = per_view_ms(x3, nv, 2 * nv)
    x3.check_range()
    err3 = errors_vs_reference(x3, "headline")
    flop = 800 * 600 * 128 * W.FLOPS_PER_SAMPLE
    out["gate_path_f16x3_800x600x128"] = {
        "rays_per_s": 800 * 600 / dt, "ms_per_frame": 1e3 * dt, "mlp_kernel_ms": ms,
        "mlp_kernel_ms_per_view": views_ms,
        "mlp_tflops": flop / (ms * 1e-3) / 1e12,
        "frac_of_bf16_dense_peak": flop / (ms * 1e-3) / 1e12 / PEAK_TFLOPS["bf16"],
        "frac_of_x3_ceiling": flop / (ms * 1e-3) / 1e12 / PEAK_TFLOPS["f16x3"],
        "rgb_max_abs_vs_reference": err3.get("rgb_max_abs_vs_reference"),
        "depth_pixels_gt_1e-2": err3.get("depth_pixels_gt_1e-2"),
        "error_vs_reference": err3,
        "note": "the north star's two clauses side by side: this path meets the 1e-4 gate against the "
                "reference on Lego (tests/test_gpu_lego.py, whole 800x600x128 frames) at three f16 MFMAs "
                "per product; the headline bf16 line meets the roofline clause, not the gate"}

    out["lego_original_nerf_fp32_800x600x128"] = original_nerf_leg(poses, local, "fp32")
    out["lego_original_nerf_f16x3_800x600x128"] = original_nerf_leg(poses, local, "f16x3")

    h = MI355XRenderer("bf16", n_importance=128, device_index=local)
    h.setup(ckpt)
    h.hip.set_profiling(True)
    step, _ = frame_step(h, poses, 800, 600, 64, 0, 1)
    dt = time_steps(step, 1, 3, 1) / nv
    st = h.hip.stage_ms()
    flop = 800 * 600 * (64 + 192) * W.FLOPS_PER_SAMPLE
    mlp_ms = st["coarse_mlp"] + st["fine_mlp"]
    errh = errors_vs_reference(h, "c3")
    out["c3_hierarchical_bf16_800x600_64+128"] = {
        "rays_per_s": 800 * 600 / dt, "ms_per_frame": 1e3 * dt, "stage_ms_last_view": st,
        "mlp_tflops_last_view": flop / (mlp_ms * 1e-3) / 1e12,
        "mlp_frac_bf16_peak_last_view": flop / (mlp_ms * 1e-3) / 1e12 / 2500.0,
        "samples_per_ray": "64 coarse (coarse net) + 192 fine (fine net on the sorted union)",
        "rgb_max_abs_vs_reference": errh.get("rgb_max_abs_vs_reference"),
        "rgb_mean_abs_vs_reference": errh.get("rgb_mean_abs_vs_reference"),
        "depth_pixels_gt_1e-2": errh.get("depth_pixels_gt_1e-2"), "error_vs_reference": errh}

    # C3 on the fp32 path: the reference's arithmetic, its error against the reference's fp32
    # chain and both against the float64 truth (tests/test_gpu_lego_c3.py (iv))
    h32 = MI355XRenderer("fp32", n_importance=128, device_index=local)
    h32.setup(ckpt)
    h32.hip.set_profiling(True)
    step, _ = frame_step(h32, poses, 800, 600, 64, 0, 1)
    dt = time_steps(step, 1, 1, 1) / nv
    st = h32.hip.stage_ms()
    mlp_ms = st["coarse_mlp"] + st["fine_mlp"]
    errh32 = errors_vs_reference(h32, "c3")
    out["c3_hierarchical_fp32_800x600_64+128"] = {
        "rays_per_s": 800 * 600 / dt, "ms_per_frame": 1e3 * dt, "stage_ms_last_view": st,
        "mlp_tflops_last_view": flop / (mlp_ms * 1e-3) / 1e12,
        "mlp_frac_f32_peak_last_view": flop / (mlp_ms * 1e-3) / 1e12 / PEAK_TFLOPS["fp32"],
        "rgb_max_abs_vs_reference": errh32.get("rgb_max_abs_vs_reference"),
        "pixels_over_1e-4": errh32.get("pixels_over_1e-4"), "vs_fp64": errh32.get("vs_fp64"),
        "depth_pixels_gt_1e-2": errh32.get("depth_pixels_gt_1e-2"), "error_vs_reference": errh32}
    del h32

    # C3 on the gate-passing path (split fp16 for both nets; the hierarchical chain is
    # checked at the 1e-4 gate on Lego in tests/test_gpu_lego.py)
    h3 = MI355XRenderer("f16x3", n_importance=128, device_index=local)
    h3.setup(ckpt)
    h3.hip.set_profiling(True)
    step, _ = frame_step(h3, poses, 800, 600, 64, 0, 1)
    dt = time_steps(step, 1, 1, 1) / nv
    st = h3.hip.stage_ms()
    mlp_ms = st["coarse_mlp"] + st["fine_mlp"]
    h3.check_range()
    errh3 = errors_vs_reference(h3, "c3")
    out["c3_hierarchical_f16x3_800x600_64+128"] = {
        "rays_per_s": 800 * 600 / dt, "ms_per_frame": 1e3 * dt, "stage_ms_last_view": st,
        "mlp_tflops_last_view": flop / (mlp_ms * 1e-3) / 1e12,
        "mlp_frac_x3_ceiling_last_view": flop / (mlp_ms * 1e-3) / 1e12 / PEAK_TFLOPS["f16x3"],
        "rgb_max_abs_vs_reference": errh3.get("rgb_max_abs_vs_reference"),
        "pixels_over_1e-4": errh3.get("pixels_over_1e-4"), "vs_fp64": errh3.get("vs_fp64"),
        "depth_pixels_gt_1e-2": errh3.get("depth_pixels_gt_1e-2"), "error_vs_reference": errh3}
    del h3
    # the same with the coarse pass on the fp32 path (NERF_OPT_COARSE_PRECISION): the sampler then
    # sees the fp32 path's coarse weights, and the render is as close to the float64 chain as the
    # fp32 path's (tests/test_gpu_lego_c3.py (iv))
    h3c = MI355XRenderer("f16x3", n_importance=128, device_index=local, coarse_precision="fp32")
    h3c.setup(ckpt)
    h3c.hip.set_profiling(True)
    step, _ = frame_step(h3c, poses, 800, 600, 64, 0, 1)
    dt = time_steps(step, 1, 1, 1) / nv
    st = h3c.hip.stage_ms()
    h3c.check_range()
    errh3c = errors_vs_reference(h3c, "c3")
    out["c3_hierarchical_f16x3_fp32coarse_800x600_64+128"] = {
        "rays_per_s": 800 * 600 / dt, "ms_per_frame": 1e3 * dt, "stage_ms_last_view": st,
        "rgb_max_abs_vs_reference": errh3c.get("rgb_max_abs_vs_reference"),
        "pixels_over_1e-4": errh3c.get("pixels_over_1e-4"), "vs_fp64": errh3c.get("vs_fp64"),
        "depth_pixels_gt_1e-2": errh3c.get("depth_pixels_gt_1e-2"), "error_vs_reference": errh3c}
    del h3c

    f8 = MI355XRenderer("fp8", device_index=local)
    f8.setup(ckpt)
    f8.hip.set_profiling(True)
    step, _ = frame_step(f8, poses, 800, 600, 128, 0, 1)
    dt = time_steps(step, 1, 3, 1) / nv
    ms = kernel_ms(f8, 3 * nv)
    views_ms = per_view_ms(f8, nv, 3 * nv)         # before the error bands add frames to the history
    tf = 800 * 600 * 128 * W.FLOPS_PER_SAMPLE / (ms * 1e-3) / 1e12
    err8 = errors_vs_reference(f8, "headline")
    out["c5_fp8_800x600x128"] = {
        "rays_per_s": 800 * 600 / dt, "ms_per_frame": 1e3 * dt, "mlp_kernel_ms": ms,
        "mlp_kernel_ms_per_view": views_ms, "mlp_tflops": tf,
        "mlp_frac_mixed_ceiling": tf / PEAK_TFLOPS["fp8"], "mlp_frac_fp8_peak": tf / 5000.0,
        "ceiling_note": "L2-L7 on the fp8 MFMA, L0, L1, C0 and the heads on the bf16 MFMA (mlp_fp8.hip): "
                        f"ceiling {FP8_MIX_CEILING:.0f} TFLOP/s for this mix",
        "rgb_max_abs_vs_reference": err8.get("rgb_max_abs_vs_reference"),
        "rgb_mean_abs_vs_reference": err8.get("rgb_mean_abs_vs_reference"),
        "depth_pixels_gt_1e-2": err8.get("depth_pixels_gt_1e-2"), "error_vs_reference": err8,
        "int8_compressed_renderer_vs_reference": int8_renderer_error()}
    return out, f8


def sharded_hierarchical(ckpt, poses, local, rank, world, width, height, n_warm=1, n_steps=3):
    """C4: 64 coarse + 128 importance samples, bf16, each rank its row band rendered
    into the packed tile, one gather to rank 0 per frame, the suite's two views; rays/s
    of the whole frame (W*H / mean view time) over the slowest rank."""
    import torch.distributed as dist

    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    h = MI355XRenderer("bf16", n_importance=128, device_index=local)
    h.setup(ckpt)
    step, _ = frame_step(h, poses, width, height, 64, rank, world)
    dt = time_steps(step, n_warm, n_steps, world) / len(poses)
    return {"rays_per_s": width * height / dt, "ms_per_frame": 1e3 * dt, "n_gpus": world,
            "samples_per_ray": "64 coarse (coarse net) + 192 fine (fine net on the sorted union)",
            "parallelism": f"row-band x{world} + {dist.get_backend()} gather to rank 0",
            "self_check": check_gathered(h, poses[0], width, height, 64, rank, world)}


# ---------------------------------------------------------------- training --
TRAIN_RAYS = 2048            # main.py:40 (get_default_config n_rays)


def training_leg(local, rank, world, n_steps, cpu_seconds):
    """NeRFTrainer.train_step on the GPU(s) with main.py's configuration
    (2048 rays, 64 stratified coarse + 128 uniform fine samples, Adam lr 3e-4, weight
    decay 1e-6, clip 1.0): steps/s and rays/s with the step's own draws (torch.randperm,
    torch.rand on the device) inside the timed region, the GEMMs' fp32 MFMA rate from
    the trainer's HIP events, and the oracle's step timed on the host cores.  At N > 1
    the step is data parallel (nerf_amd.distributed.train_step_sharded): each rank takes
    2048/N of the step's rays and one RCCL all-reduce sums the gradients (strong scaling:
    the step is fixed)."""
    import numpy as np
    import torch

    from nerf_amd import distributed as D
    from nerf_amd import weights as W
    from nerf_amd.trainer import GEMM_MACS_PER_SAMPLE, MAIN_CONFIG, WGRAD_OPERAND_BYTES_PER_SAMPLE, MI355XTrainer

    cfg = dict(MAIN_CONFIG, n_rays=TRAIN_RAYS)
    sd_c, sd_f = W.synthetic_models(0)
    tr = MI355XTrainer(cfg, sd_c, sd_f, device_index=local)
    h = w = 400
    rng = np.random.RandomState(3)
    image = torch.from_numpy(rng.rand(h, w, 3).astype(np.float32)).cuda(local)
    pose = torch.eye(4)
    pose[2, 3] = 4.0
    batch = {"image": image, "pose": pose, "focal": 0.5 * w / np.tan(0.5 * 0.6911112070083618)}
    gen = torch.Generator(device=f"cuda:{local}")

    def step(i):
        if world == 1:
            return tr.train_step(batch, sync=False)
        gen.manual_seed(1000 + i)            # the same step draw on every rank
        sel, t_rand = tr.draws(h, w, TRAIN_RAYS, generator=gen)
        return D.train_step_sharded(tr, batch, sel, t_rand)

    losses = [float(step(i)[0].item()) for i in range(2)]
    # timed steps with profiling off (the trainer then runs the coarse net's pass beside the
    # fine net's on a second stream); stage times from two profiled steps after them (the
    # passes one after the other, each stage bracketed by HIP events)
    sync_barrier(world)
    t0 = time.perf_counter()
    for i in range(n_steps):
        step(2 + i)
    sync_barrier(world)
    dt = D.reduce_max(time.perf_counter() - t0) / n_steps
    tr.set_profiling(True)
    stages = []
    for i in range(2):
        step(2 + n_steps + i)
        stages.append(tr.stage_ms())
    tr.set_profiling(False)
    losses.append(float(step(4 + n_steps)[0].item()))
    st = {k: float(np.mean([s[k] for s in stages])) for k in stages[0]}
    # the same step with the forward and the backward-data chain on the split-bf16 MFMA
    # (precision "bf16x3"), from the parameters as they now stand
    tr.set_precision("bf16x3")
    for i in range(2):
        step(5 + n_steps + i)
    sync_barrier(world)
    t0 = time.perf_counter()
    for i in range(n_steps):
        step(7 + n_steps + i)
    sync_barrier(world)
    dt_x3 = D.reduce_max(time.perf_counter() - t0) / n_steps
    tr.set_profiling(True)
    stages_x3 = []
    for i in range(2):
        step(7 + 2 * n_steps + i)
        stages_x3.append(tr.stage_ms())
    tr.set_profiling(False)
    tr.set_precision("fp32")
    x3 = {"ms_per_step": 1e3 * dt_x3, "rays_per_s": TRAIN_RAYS / dt_x3,
          "stage_ms_rank0": {k: float(np.mean([s[k] for s in stages_x3])) for k in stages_x3[0]},
          "note": "precision 'bf16x3': the forward (mlp_bf16x3.hip's kernel with the rows and ReLU bits the "
                  "backward reads) and the backward-data chain (train_bwd_x3.hip) on the split-bf16 MFMA; "
                  "gradients as close to the float64 step as the reference's fp32 step "
                  "(tests/test_gpu_train.py); the default line above is fp32"}
    # per-kernel rates in the unit each kernel is bound by: the fused forward and the
    # backward-data chain on the f32 MFMA, the weight gradients (split-bf16 MFMA) on HBM
    samples = (int(TRAIN_RAYS) // world + (1 if rank < TRAIN_RAYS % world else 0)) * (cfg["n_coarse"] + cfg["n_fine"])
    flop = tr.gemm_flops()
    assert abs(flop - 2.0 * sum(GEMM_MACS_PER_SAMPLE.values()) * samples) <= 1e-6 * flop, (flop, samples)
    kernels = {}
    for key, stage in (("forward", "forward_gemm"), ("backward_data", "backward_data_gemm")):
        f = 2.0 * GEMM_MACS_PER_SAMPLE[key] * samples
        kernels[key] = {"stage": stage, "ms": st[stage], "flop": f, "achieved": f / (st[stage] * 1e-3) / 1e12,
                        "peak": PEAK_TFLOPS["fp32"], "unit": "TFLOP/s",
                        "frac": f / (st[stage] * 1e-3) / 1e12 / PEAK_TFLOPS["fp32"]}
    # the bf16x3 step's forward and backward-data on the split-bf16 MFMA: three bf16 MFMAs
    # per fp32 product, priced against the bf16 peak / 3
    sx = x3["stage_ms_rank0"]
    x3_kernels = {}
    for key, stage in (("forward", "forward_gemm"), ("backward_data", "backward_data_gemm")):
        f = 2.0 * GEMM_MACS_PER_SAMPLE[key] * samples
        x3_kernels[key] = {"stage": stage, "ms": sx[stage], "flop": f, "achieved": f / (sx[stage] * 1e-3) / 1e12,
                           "peak": PEAK_TFLOPS["bf16x3"], "unit": "TFLOP/s",
                           "frac": f / (sx[stage] * 1e-3) / 1e12 / PEAK_TFLOPS["bf16x3"]}
    x3["gemm_kernels_rank0"] = x3_kernels
    b = WGRAD_OPERAND_BYTES_PER_SAMPLE * samples
    kernels["weight_grad"] = {"stage": "weight_grad_gemm", "ms": st["weight_grad_gemm"], "bytes": b,
                              "achieved": b / (st["weight_grad_gemm"] * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
                              "frac": b / (st["weight_grad_gemm"] * 1e-3) / 1e9 / 8000.0,
                              "note": "operand rows each weight-gradient GEMM reads (17,508 B per sample) over the "
                                      "stage time; split-bf16 MFMA, bound by HBM"}
    out = {"workload": "NeRFTrainer.train_step, main.py config: 2048 rays of a 400x400 target, 64 stratified "
                       "coarse + 128 uniform fine samples, both nets forward+backward, clip 1.0, Adam, ExponentialLR",
           "dtype": "fp32 (weight-gradient GEMMs: split bf16, 3 bf16 MFMAs per fp32 product, fp32 accumulate)",
           "steps": n_steps, "n_gpus": world, "ms_per_step": 1e3 * dt, "steps_per_s": 1.0 / dt,
           "rays_per_s": TRAIN_RAYS / dt, "stage_ms_rank0": st,
           "parallelism": "1 GPU" if world == 1 else f"data parallel x{world}: 2048/{world} rays per rank + "
                                                     f"{'RCCL' if torch.distributed.get_backend() == 'nccl' else 'gloo'} "
                                                     f"all-reduce of the gradients (4.2 MB)",
           "gemm_kernels_rank0": kernels,
           "gemm_note": "stage times from HIP events of profiled steps (the two nets' passes one after the "
                        "other), both nets; unpadded GEMM work (trainer.GEMM_MACS_PER_SAMPLE) x samples",
           "loss_first_last": [losses[0], losses[-1]], "bf16x3_forward": x3}
    tr.close()
    if cpu_seconds > 0 and rank == 0 and world == 1:
        # the oracle's step (PyTorch-CPU autograd restatement of NeRFTrainer.train_step)
        import math

        from oracle import nerf_train_oracle as T

        info = host_cpu_info()
        threads = info["physical_affinity"]
        if info["cgroup_quota_cpus"]:
            threads = max(1, min(threads, int(math.floor(info["cgroup_quota_cpus"]))))
        prev = torch.get_num_threads()
        torch.set_num_threads(threads)
        try:
            n_cpu = 256
            orc = T.TrainOracle(sd_c, sd_f, dict(cfg, n_rays=n_cpu))
            img = image.cpu().numpy()
            draws = [(rng.permutation(h * w)[:n_cpu], rng.rand(n_cpu, 64).astype(np.float32)) for _ in range(8)]
            orc.step(img, pose.numpy(), batch["focal"], *draws[0])
            t0 = time.perf_counter()
            k = 0
            while k < len(draws) - 1 and (k == 0 or time.perf_counter() - t0 < cpu_seconds):
                orc.step(img, pose.numpy(), batch["focal"], *draws[k + 1])
                k += 1
            cdt = (time.perf_counter() - t0) / k
        finally:
            torch.set_num_threads(prev)
        out["cpu_baseline"] = {"value": n_cpu / cdt, "unit": "rays/s", "cores": threads, "kind": "port",
                               "sample": f"oracle TrainOracle.step, {k} steps of {n_cpu} rays (64 + 128 samples), "
                                         f"{threads} torch threads", "ms_per_step": 1e3 * cdt}
    return out


# ------------------------------------------------------------- CPU baseline --
def launch_traffic(kname, width, height, spp, world, band_rays):
    """HBM bytes per launch of kernel ``kname`` from profiles/pmc_latest.json (the headline
    launch's rocprofv3 FETCH_SIZE / WRITE_SIZE passes, collected at N = 1).  At N > 1 the
    N = 1 figure scaled by this rank's band, labelled as such: the traffic
    is per sample (segment records, rays, outputs), the 1 MB of weights aside."""
    pmc = os.path.join(REPO, "profiles", "pmc_latest.json")
    if not os.path.exists(pmc) or (width, height, spp) != (800, 600, 128):
        return None, None
    k = json.load(open(pmc)).get("kernels", {}).get(kname, {})
    if "hbm_bytes_per_launch" not in k:
        return None, None
    if world == 1:
        # profiles/collect.sh profiles the headline bench alone, so every dispatch of this
        # kernel there is this launch
        return k["hbm_bytes_per_launch"], (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `{k['command']}` "
                                           f"({k['source']}); bytes/launch, FETCH_SIZE x2 (gfx950)")
    return (k["hbm_bytes_per_launch"] * band_rays / (width * height),
            f"scaled from the N=1 counters (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of `{k['command']}`, "
            f"{k['source']}) by rank 0's band: {band_rays} of {width * height} rays; not measured at N={world}")


def ranked_cpu_baseline(rank, world, budget_s):
    """The CPU baseline on rank 0.  At N > 1 the same protocol at half the
    budget, after every rank's GPU work, while the other ranks block in a TCPStore wait (a
    socket read, no spinning collective) so that the host cores are free."""
    import torch.distributed as dist

    if budget_s <= 0:
        return None
    if world == 1:
        return cpu_baseline(budget_s)
    store = dist.distributed_c10d._get_default_store()
    cpu = None
    if rank == 0:
        try:
            cpu = cpu_baseline(budget_s / 2)
            cpu["n_gpus_protocol"] = (f"rank 0 of {world}, after the GPU legs, the other ranks idle in a "
                                      f"TCPStore wait; budget {budget_s / 2:.0f} s (half the N=1 budget)")
        finally:
            store.set("nerf_bench_cpu_baseline_done", "1")
    else:
        store.wait(["nerf_bench_cpu_baseline_done"], timedelta(seconds=1800))
    return cpu


def host_cpu_info():
    """CPU model; logical CPUs of the machine and of this process's affinity mask;
    physical cores behind that mask; the cgroup CPU quota, if any."""
    info = {"model": "unknown CPU", "logical_machine": os.cpu_count()}
    try:
        with open("/proc/cpuinfo") as f:
            info["model"] = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    aff = sorted(os.sched_getaffinity(0))
    info["logical_affinity"] = len(aff)
    cores = set()
    for c in aff:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            cores.add((open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip()))
        except OSError:
            cores.add(("?", str(c)))
    info["physical_affinity"] = len(cores)
    info["cgroup_quota_cpus"] = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = int(q) / int(p)
    except (OSError, ValueError):
        pass
    return info


def lego_psnr():
    from nerf_amd import weights as W

    return json.load(open(W.LEGO_NPZ.replace(".npz", ".json")))["report"]["fine"]["psnr_db_mean"]


def cpu_baseline(budget_s):
    """The oracle's render_image on the host, the suite's protocol (wall clock around
    render_image including ray generation, averaged over the 2 views of
    generate_test_poses(2)), torch threads = physical cores in this process's
    affinity mask (capped by the cgroup quota), 512-ray chunks.  Cells: 200x150x32
    (whole frames), 400x300x64 and 800x600x128 (centre row bands sized to the budget).
    The headline value is the 800x600x128 cell."""
    import math

    import torch

    from nerf_amd import weights as W
    from nerf_amd.benchmark.benchmark_suite import generate_test_poses
    from oracle import nerf_oracle as O

    info = host_cpu_info()
    threads = info["physical_affinity"]
    if info["cgroup_quota_cpus"]:
        threads = max(1, min(threads, int(math.floor(info["cgroup_quota_cpus"]))))
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        _, fine = W.lego_models()
        net = O.Net(fine)
        poses = generate_test_poses(2)

        def rate(width, height, spp, rows):
            r0 = (height - rows) // 2
            per_view = []
            for p in poses:
                t0 = time.perf_counter()
                O.render_image(net, p, (width, height), spp, rows=(r0, r0 + rows))
                per_view.append(time.perf_counter() - t0)
            return rows * width * len(poses) / sum(per_view), per_view

        def loadavg():
            try:
                return [float(v) for v in open("/proc/loadavg").read().split()[:3]]
            except OSError:
                return None

        # calibrate each cell's rays/s on one row per view, then size its band
        cells = {}
        share = {"200x150x32": 0.2, "400x300x64": 0.3, "800x600x128": 0.5}
        load0 = loadavg()
        for key, (w, h, s) in (("200x150x32", (200, 150, 32)), ("400x300x64", (400, 300, 64)),
                               ("800x600x128", (800, 600, 128))):
            est, _ = rate(w, h, s, 1)
            # two timed repeats of half the budget each; the cell reports the faster (the host is
            # a shared 16-CPU share of a busy machine: one slow repeat is load, not the renderer)
            rows = int(min(h, max(2, share[key] * budget_s * est / (4 * w))))
            reps = [rate(w, h, s, rows) for _ in range(2)]
            v, per_view = max(reps, key=lambda r: r[0])
            cells[key] = {"rays_per_s": v, "rows": rows, "rays_timed": 2 * rows * w,
                          "seconds_per_view": per_view, "repeats_rays_per_s": [r[0] for r in reps]}
        load1 = loadavg()
    finally:
        torch.set_num_threads(prev)
    head = cells["800x600x128"]
    return {"value": head["rays_per_s"], "unit": "rays/s", "cores": threads, "kind": "port",
            "sample": (f"oracle render_image (PyTorch-CPU restatement of PyTorchCPURenderer, 512-ray chunks), "
                       f"2 views of generate_test_poses(2), centre band of {head['rows']} rows of 800x600x128 "
                       f"per view ({head['rays_timed']} rays), the faster of 2 repeats, {threads} torch threads, "
                       f"torch {torch.__version__}"),
            "threads": threads, "host": info, "cells": cells,
            "loadavg_1_5_15min": {"start": load0, "end": load1}}


# --------------------------------------------------------------------- main --
def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launched as `python bench.py --gpus N` rather than under torchrun: one process
        # per GPU is still the contract, so start torchrun as a child (before any GPU call)
        os.environ["NERF_BENCH_SELF_LAUNCHED"] = "1"
        sys.exit(self_launch(sys.argv[1:], args.gpus))
    if args.launch_check:
        return launch_check(args)
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
    if world > 1:
        # form the communicator before anything is timed (RCCL sets up lazily on first use)
        warm = torch.ones(1, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(warm)
        dist.barrier()

    width, height, spp = args.width, args.height, args.spp
    ckpt_dir = tempfile.mkdtemp(prefix=f"nerf_bench_r{rank}_")
    ckpt = W.write_lego_checkpoint(os.path.join(ckpt_dir, "lego.pth"))
    r = MI355XRenderer(args.precision, device_index=local)
    r.setup(ckpt)
    r.hip.set_profiling(True)

    # the suite's protocol (benchmark_suite.py:188-220): both views of generate_test_poses(2),
    # rays/s = W*H / the mean view time; a step renders view 0 then view 1
    from nerf_amd.benchmark.benchmark_suite import generate_test_poses

    poses = generate_test_poses(2)
    nv = len(poses)
    pose = poses[0]
    step, band_rays = frame_step(r, poses, width, height, spp, rank, world)

    for _ in range(args.warmup):
        step()
    sync_barrier(world)
    clocks = ClockSampler(local)
    with clocks:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()                                      # queued back to back: no host sync per frame
        sync_barrier(world)
        elapsed = D.reduce_max(time.perf_counter() - t0)   # max over ranks
    # the fine-MLP kernel's HIP-event times of the timed frames (the library's
    # per-frame event ring, recorded on the launch stream), over both views and per view
    kern_ms = kernel_ms(r, args.steps * nv)
    kern_ms_views = per_view_ms(r, nv, args.steps * nv)
    ms_step = 1000.0 * elapsed / args.steps
    value = width * height * nv * args.steps / elapsed
    # each view timed alone as well (wall clock, same step shape), outside the timed region
    view_ms = []
    for p in poses:
        vstep, _ = frame_step(r, [p], width, height, spp, rank, world)
        view_ms.append(1e3 * time_steps(vstep, 1, max(2, args.steps // 2), world))

    flop_launch = band_rays * spp * W.FLOPS_PER_SAMPLE
    kname = {"bf16x3": "mlp_x3_kernel<OpBf16>", "f16x3": "mlp_x3_kernel<OpF16>"}.get(args.precision,
                                                                                    f"mlp_{args.precision}_kernel")
    traffic, traffic_src = launch_traffic(kname, width, height, spp, world, band_rays)
    achieved = flop_launch / (kern_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.precision]
    peak_kind = {"bf16": "bf16 dense MFMA peak", "fp32": "f32 MFMA peak",
                 "bf16x3": "bf16 dense peak / 3 (three MFMAs per product)",
                 "f16x3": "f16 dense peak / 3 (three MFMAs per product)",
                 "fp8": (f"mixed fp8/bf16 ceiling of this layer split ({FP8_MIX_CEILING:.0f} TFLOP/s), "
                         "not the 5000 TFLOP/s fp8 hardware peak")}[args.precision]

    extra = {"gpu_clock_timed_region": clocks.summary(),
             "protocol": {"views": "generate_test_poses(2) (benchmark_suite.py:132-149, 188-220)",
                          "frames_per_step": nv, "value": "W*H / mean view time",
                          "ms_per_view_wall": view_ms, "mlp_kernel_ms_per_view": kern_ms_views}}
    if world > 1:
        extra["dist"] = dist_record()
        extra["self_check"] = check_gathered(r, pose, width, height, spp, rank, world)
    if world > 1 and not args.no_extras:
        # BASELINE config 4: the 64+128 hierarchical frame (bf16), sharded in row
        # bands over every rank and gathered to rank 0 -- every rank takes part
        extra["c4_hierarchical_sharded"] = sharded_hierarchical(ckpt, poses, local, rank, world, width, height)
        # per-frame breakdown at N GPUs: the slowest rank's MLP kernel
        # and the exchange alone (the gather of the packed tiles), 10 frames
        tile = D.band_tile(world, height, width, r.torch_device())
        sync_barrier(world)
        t_x = time.perf_counter()
        for _ in range(10):
            D.gather_tiles_to_root(tile, width, height)
        sync_barrier(world)
        extra["exchange_ms_per_frame"] = 1e3 * D.reduce_max(time.perf_counter() - t_x) / 10
        extra["mlp_ms_per_frame_rank_max"] = D.reduce_max(kern_ms)
    ref = f8 = None
    if not args.no_extras:
        ref = r if args.precision == "fp32" else MI355XRenderer("fp32", device_index=local)
        if ref is not r:
            ref.setup(ckpt)
        ref.hip.set_profiling(True)
    r.check_range()
    if rank == 0 and not args.no_error_check and (width, height, spp) == (800, 600, 128):
        # the headline path against the reference's own whole frames (PyTorchCPURenderer.render_image
        # on the same checkpoint, tests/golden/render_lego_800x600_s128_full.npz): BASELINE.json's
        # "RGB max-abs err" beside rays/s
        err = errors_vs_reference(r, "headline")
        extra["rgb_max_abs_vs_reference"] = err.get("rgb_max_abs_vs_reference")
        extra["rgb_mean_abs_vs_reference"] = err.get("rgb_mean_abs_vs_reference")
        extra["depth_pixels_gt_1e-2"] = err.get("depth_pixels_gt_1e-2")
        extra["error_vs_reference"] = err

    if world == 1 and not args.no_extras:
        extra["other_configs"], f8 = other_configs(ckpt, poses, local, ref)
    if not args.no_extras and not args.no_grid:
        # every rank takes part (bands + gather at N > 1)
        if f8 is None:
            f8 = r if args.precision == "fp8" else MI355XRenderer("fp8", device_index=local)
            if f8 is not r:
                f8.setup(ckpt)
        f8.hip.set_profiling(True)
        rs = {"bf16": r if args.precision == "bf16" else None, "fp8": f8, "fp32": ref,
              "f16x3": r if args.precision == "f16x3" else None}
        for p in ("bf16", "f16x3"):
            if rs[p] is None:
                rs[p] = MI355XRenderer(p, device_index=local)
                rs[p].setup(ckpt)
                rs[p].hip.set_profiling(True)
        extra["readme_grid"] = readme_grid(rs, poses, rank, world)

    if not args.no_train and not (world > 1 and args.no_extras):
        extra["training"] = training_leg(local, rank, world, args.train_steps, min(10.0, args.cpu_seconds / 3))

    cpu = ranked_cpu_baseline(rank, world, args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "ms_per_view": ms_step / nv,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": ("Lego: the reference's bundled original-NeRF Lego networks (data/lego_example_weights) "
                     "distilled into NeRFModel's layout (nerf_amd/checkpoints/lego_distilled.npz, held-out PSNR "
                     f"{lego_psnr():.1f} dB vs the teacher); both suite views of generate_test_poses(2) (benchmark_suite.py:132-149), "
                     "rays/s = W*H / mean view time (:188-220); "
                     "rays generated on the device from the pose"),
            "config": {"workload": f"render_image {width}x{height}, {spp} uniform samples/ray, fine net",
                       "resolution": [width, height], "samples_per_ray": spp,
                       "parallelism": (f"row-band x{world} + "
                                       f"{'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()} "
                                       f"gather to rank 0" if world > 1 else "1 GPU")},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "peak_kind": peak_kind,
                         **({"frac_fp8_hw_peak": achieved / 5000.0} if args.precision == "fp8" else {}),
                         "traffic": traffic, "traffic_source": traffic_src,
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
