"""Cycle budget of the bf16 MLP kernel from a -DNERF_STAMPS diagnostic build.

    python tools/stamps.py path/to/libnerf_stamps.so [--waves 4]

Stamps (s_memtime, shader cycles) sit at the kernel start, the prologue end, and
on both sides of every chunk barrier.  Per wave we get: prologue, per-chunk
compute segments (barrier-to-barrier), barrier waits, and the tail.  Only the
shares are meaningful (the stamps themselves add cost).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nerf-dbr_amd"), os.path.join(REPO, "tools")]

from kernel_lab import Lib  # noqa: E402
from nerf_amd import weights as W  # noqa: E402

UNITS = [4 * 4, 16 * 4, 16 * 4, 16 * 4, 20 * 4, 16 * 4, 16 * 4, 16 * 4, 18 * 2]   # per layer (quarters x k-steps)
NAMES = ["L0", "L1", "L2", "L3", "L4", "L5", "L6", "L7", "C0"]


def main():
    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--chunk-units", type=int, default=8)
    args = ap.parse_args()
    _, fine = W.synthetic_models(0)
    lib = Lib(args.lib, fine, 1)
    pose = np.eye(4, dtype=np.float32)
    pose[2, 3] = 4.0
    t = torch.linspace(0, 1, 128).numpy()
    rgb = torch.empty(600, 800, 3, device="cuda")
    depth = torch.empty(600, 800, device="cuda")
    lib.render(pose, t, rgb, depth)
    ms = lib.render(pose, t, rgb, depth)
    fn = lib.lib.nerf_debug_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    buf = np.zeros(256 * 8 * 200, np.uint64)
    waves, slots = ctypes.c_int(), ctypes.c_int()
    assert fn(buf.ctypes.data, buf.nbytes, ctypes.byref(waves), ctypes.byref(slots)) == 0
    s = buf[: 256 * waves.value * slots.value].reshape(256, waves.value, slots.value).astype(np.int64)
    n_chunks = (slots.value - 3) // 3 - 1            # seams (the last chunk has none)
    arrive = s[:, :, 2:2 + 3 * n_chunks:3]
    waited = s[:, :, 3:3 + 3 * n_chunks:3]
    leave = s[:, :, 4:4 + 3 * n_chunks:3]
    prev_leave = np.concatenate([s[:, :, 1:2], leave[:, :, :-1]], axis=2)
    compute = arrive - prev_leave
    waits = waited - arrive
    barrier = leave - waited
    total = s[:, :, -1] - s[:, :, 0]
    prologue = s[:, :, 1] - s[:, :, 0]
    tail = s[:, :, -1] - leave[:, :, -1]
    # chunk -> layer
    bounds = np.cumsum([0] + UNITS)
    layer_of_chunk = [int(np.searchsorted(bounds, (c * args.chunk_units), side="right") - 1)
                      for c in range(n_chunks)]
    per_layer = {}
    for li, name in enumerate(NAMES):
        idx = [c for c in range(n_chunks) if layer_of_chunk[c] == li]
        per_layer[name] = {"chunks": len(idx), "compute_med": float(np.median(compute[:, :, idx].sum(2))),
                           "wait_med": float(np.median(waits[:, :, idx].sum(2))),
                           "barrier_med": float(np.median(barrier[:, :, idx].sum(2)))}
    # Skew at the seams: arrival of each wave relative to the block's first
    # arrival.  Waves w and w+4 share a SIMD (round-robin wave placement).
    rel = arrive - arrive.min(axis=1, keepdims=True)                  # [blocks, waves, seams]
    nw = waves.value
    skew = {"per_wave_mean_late": [float(v) for v in rel.mean(axis=(0, 2))],
            "spread_med": float(np.median(rel.max(axis=1))),
            "dma_wait_p50_p90_p99": [float(np.percentile(waits, p)) for p in (50, 90, 99)]}
    if nw == 8:
        pair_last = np.maximum(arrive[:, :4], arrive[:, 4:])            # per SIMD: its last wave
        pair_first = np.minimum(arrive[:, :4], arrive[:, 4:])
        skew["intra_simd_gap_med"] = float(np.median(pair_last - pair_first))
        skew["inter_simd_spread_med"] = float(np.median(pair_last.max(axis=1) - pair_last.min(axis=1)))
        # which wave of a pair is late, as a fraction of seams
        skew["upper_wave_late_frac"] = float((arrive[:, 4:] > arrive[:, :4]).mean())
    clk = np.zeros(256 * waves.value * 4, np.uint64)
    fc = lib.lib.nerf_debug_clock
    fc.restype, fc.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]
    assert fc(clk.ctypes.data, clk.nbytes) == 0
    clk = clk.reshape(256, waves.value, 4).astype(np.float64)
    ghz = (clk[..., 2] - clk[..., 0]) / np.maximum(clk[..., 3] - clk[..., 1], 1) * 0.1
    out = {
        "in_kernel_clock_ghz_median": float(np.median(ghz)),
        "kernel_ms": ms, "waves": waves.value, "chunks": n_chunks, "skew": skew,
        "total_med": float(np.median(total)), "prologue_med": float(np.median(prologue)),
        "compute_med": float(np.median(compute.sum(2))), "wait_med": float(np.median(waits.sum(2))),
        "barrier_med": float(np.median(barrier.sum(2))),
        "tail_med": float(np.median(tail)),
        "per_chunk_compute_med": [float(v) for v in np.median(compute, axis=(0, 1))],
        "per_layer": per_layer,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
