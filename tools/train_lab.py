"""Interleaved A/B timing of training-kernel builds in one process (GPU box only).

    python tools/train_lab.py [--rounds 10] lib1.so lib2.so ...

Each library is a full libnerf_mi355x.so build (make train_variant NAME=x DEFS=...).
Every round runs one training step (main.py config, 2048 rays) per library and
records the trainer's per-stage HIP-event times; the report is the median per
stage and library (cdna_hip_programming.md §5.4 rule 24).
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nerf-dbr_amd")]

import torch  # noqa: E402

from nerf_amd import runtime as rt  # noqa: E402
from nerf_amd import weights as W  # noqa: E402


class Lib:
    def __init__(self, path, sd_c, sd_f, cfg):
        self.path = path
        self.lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
        for name, (res, args) in rt.SIGNATURES.items():
            fn = getattr(self.lib, name, None)
            if fn is not None:
                fn.restype, fn.argtypes = res, args
        kc, pc = rt._param_list(sd_c)
        kf, pf = rt._param_list(sd_f)
        self.h = ctypes.c_void_p()
        assert self.lib.nerf_trainer_create(0, ctypes.byref(cfg), pc, pf, 22, ctypes.byref(self.h)) == 0, \
            self.lib.nerf_last_error()
        self.lib.nerf_trainer_set_profiling(self.h, 1)

    def set_profiling(self, on):
        self.lib.nerf_trainer_set_profiling(self.h, 1 if on else 0)

    def run(self, image, pose, sel, tr):
        rc = self.lib.nerf_train_step(self.h, image.data_ptr(), image.shape[0], image.shape[1], 555.6,
                                      rt._fptr(pose), sel.data_ptr(), sel.numel(), tr.data_ptr(), 0, None, 0)
        assert rc == 0, self.lib.nerf_last_error()

    def step(self, image, pose, sel, tr):
        rc = self.lib.nerf_train_step(self.h, image.data_ptr(), image.shape[0], image.shape[1], 555.6,
                                      rt._fptr(pose), sel.data_ptr(), sel.numel(), tr.data_ptr(), 0, None, 0)
        assert rc == 0, self.lib.nerf_last_error()
        ms = (ctypes.c_float * 5)()
        assert self.lib.nerf_trainer_stage_ms(self.h, ms) == 0
        return list(ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--wall", type=int, default=0,
                    help="also time this many back-to-back steps per library per round, profiling off "
                         "(wall clock on the stream: the trainer may overlap its two nets' passes)")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    cfg = rt.TrainConfig()
    cfg.lr, cfg.beta1, cfg.beta2, cfg.eps, cfg.weight_decay = 3e-4, 0.9, 0.999, 1e-8, 1e-6
    cfg.lr_gamma, cfg.grad_clip, cfg.n_coarse, cfg.n_fine, cfg.near_, cfg.far_ = 0.1 ** (1 / 250000), 1.0, 64, 128, 2.0, 6.0
    sd_c, sd_f = W.synthetic_models(0)
    libs = [Lib(p, sd_c, sd_f, cfg) for p in a.libs]
    rng = np.random.RandomState(3)
    image = torch.from_numpy(rng.rand(400, 400, 3).astype(np.float32)).cuda()
    pose = np.eye(4, dtype=np.float32)
    pose[2, 3] = 4.0
    sel = torch.randperm(160000, device="cuda")[:2048].to(torch.int32)
    tr = torch.rand(2048, 64, device="cuda")
    res = {l.path: [] for l in libs}
    for _ in range(2):
        for l in libs:
            l.step(image, pose, sel, tr)
    for _ in range(a.rounds):
        for l in libs:
            res[l.path].append(l.step(image, pose, sel, tr))
    if a.wall:
        wall = {l.path: [] for l in libs}
        for l in libs:
            l.set_profiling(False)
        for _ in range(a.rounds):
            for l in libs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.wall):
                    l.run(image, pose, sel, tr)
                e1.record()
                torch.cuda.synchronize()
                wall[l.path].append(e0.elapsed_time(e1) / a.wall)
        for p, v in wall.items():
            print(f"{os.path.basename(p):28s} wall {np.median(v):7.3f} ms per step (min {np.min(v):.3f}), profiling off")
    for p, v in res.items():
        v = np.array(v)
        med = np.median(v, 0)
        print(f"{os.path.basename(p):28s} total {med.sum():7.3f} ms  " +
              "  ".join(f"{n}={x:.3f}" for n, x in zip(rt.TRAIN_STAGES, med)) + f"  (min total {v.sum(1).min():.3f})")


if __name__ == "__main__":
    main()
