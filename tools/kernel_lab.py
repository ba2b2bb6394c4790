"""Interleaved A/B timing of MLP-kernel builds in one process (GPU box only).

    python tools/kernel_lab.py [--precision bf16] [--rounds 5] lib1.so lib2.so ...

Each library is a full libnerf_mi355x.so build (e.g. the timing-only ablations
from `make -C nerf-dbr_amd/csrc ablate`).  Every round renders 800x600x128 once
per library and records the fine-MLP kernel time from the library's own HIP
events; the report is median / min per library (cdna_hip_programming.md §5.4
rule 24: variants interleaved in one process).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nerf-dbr_amd")]

from nerf_amd import runtime as rt  # noqa: E402
from nerf_amd import weights as W  # noqa: E402


class Lib:
    def __init__(self, spec: str, sd_fine, precision: int):
        # spec: path[:nofuse] -- ':nofuse' turns NERF_OPT_FUSED_COMPOSITE off
        self.path = spec
        path, _, opt = spec.partition(":")
        self.lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
        for name, (res, args) in rt.SIGNATURES.items():
            fn = getattr(self.lib, name, None)          # older builds lack newer entry points
            if fn is not None:
                fn.restype, fn.argtypes = res, args
        self.ctx = ctypes.c_void_p()
        assert self.lib.nerf_ctx_create(0, ctypes.byref(self.ctx)) == 0, self.err()
        keep, ptrs = rt._param_list(sd_fine)
        for net in (0, 1):
            assert self.lib.nerf_ctx_load_weights(self.ctx, net, ptrs, rt.NERF_N_PARAMS) == 0, self.err()
        self.lib.nerf_ctx_set_profiling(self.ctx, 1)
        if opt == "nofuse":
            assert self.lib.nerf_ctx_set_option(self.ctx, rt.NERF_OPT_FUSED_COMPOSITE, 0) == 0, self.err()
        self.precision = precision

    def err(self):
        return self.lib.nerf_last_error().decode()

    def render(self, pose, t, rgb, depth, width=800, height=600):
        fp = ctypes.POINTER(ctypes.c_float)
        rc = self.lib.nerf_render(self.ctx, pose.ctypes.data_as(fp), width, height, 0, height, 800.0, 2.0, 6.0,
                                  t.ctypes.data_as(fp), t.size, 0, None, self.precision, rgb.data_ptr(),
                                  depth.data_ptr(), 0)
        assert rc == 0, self.err()
        ms = (ctypes.c_float * rt.NERF_N_STAGES)()
        assert self.lib.nerf_ctx_stage_ms(self.ctx, ms) == 0, self.err()
        return ms[3], ms[4]


def main():
    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--precision", choices=sorted(rt.PRECISIONS), default="bf16")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--ckpt", choices=["lego", "synthetic"], default="lego")
    # the same instruction stream on different operand values: "lab" (camera on +z at 4),
    # or view 0 / view 1 of the suite's generate_test_poses(2) (view 1 is near-empty content)
    ap.add_argument("--pose", choices=["lab", "view0", "view1"], default="lab")
    args = ap.parse_args()
    _, fine = W.lego_models() if args.ckpt == "lego" else W.synthetic_models(0)
    libs = [Lib(p, fine, rt.PRECISIONS[args.precision]) for p in args.libs]
    pose = np.eye(4, dtype=np.float32)
    pose[2, 3] = 4.0
    if args.pose != "lab":
        from nerf_amd.benchmark.benchmark_suite import generate_test_poses

        pose = np.ascontiguousarray(generate_test_poses(2)[int(args.pose[-1])].numpy().astype(np.float32))
    t = torch.linspace(0, 1, args.spp).numpy()
    rgb = torch.empty(600, 800, 3, device="cuda")
    depth = torch.empty(600, 800, device="cuda")
    times = {lib.path: [] for lib in libs}
    ref = None
    diffs = {}
    for lib in libs:                       # warm-up + agreement with the first library
        lib.render(pose, t, rgb, depth)
        torch.cuda.synchronize()
        img = torch.cat([rgb.reshape(-1), depth.reshape(-1)]).clone()
        if ref is None:
            ref = img
        diffs[lib.path] = float((img - ref).abs().max())
    comp = {lib.path: [] for lib in libs}
    for _ in range(args.rounds):
        for lib in libs:
            mlp_ms, comp_ms = lib.render(pose, t, rgb, depth)
            times[lib.path].append(mlp_ms)
            comp[lib.path].append(comp_ms)
    flop = 800 * 600 * args.spp * W.FLOPS_PER_SAMPLE
    out = {}
    for p, v in times.items():
        med = float(np.median(v))
        out[os.path.basename(p)] = {"median_ms": med, "min_ms": float(np.min(v)),
                                    "composite_median_ms": float(np.median(comp[p])),
                                    "tflops": flop / med / 1e9, "max_abs_vs_first": diffs[p]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
