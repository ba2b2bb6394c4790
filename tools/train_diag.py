"""Training-step numerics diagnostic (GPU box): per-tensor gradient errors of the
GPU step and of the fp32 oracle, both against a float64 evaluation of the same
step, so the GPU's error can be read against fp32's own noise floor.

    python tools/train_diag.py [n_rays]
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nerf-dbr_amd")]

from oracle import nerf_oracle as O  # noqa: E402
from oracle import nerf_train_oracle as T  # noqa: E402
from nerf_amd import weights as W  # noqa: E402
from nerf_amd.trainer import MI355XTrainer  # noqa: E402


f64_grads = T.step_grads_f64


def rel(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def main(n_rays=256):
    fx = np.load(os.path.join(REPO, "tests", "golden", "train.npz"))
    sd_c, sd_f = W.synthetic_models(0)
    cfg = dict(T.TRAIN_CONFIG, n_rays=n_rays)
    image, pose, focal = fx["image"], fx["pose"], float(fx["focal"])
    sel, tr = fx["step0_select"][:n_rays], fx["step0_t_rand"][:n_rays]
    gpu = MI355XTrainer(cfg, sd_c, sd_f)
    batch = {"image": torch.from_numpy(image), "pose": torch.from_numpy(pose), "focal": focal}
    lg = gpu.train_step(batch, select_inds=sel.astype(np.int32), t_rand=tr, update=False)
    orc = T.TrainOracle(sd_c, sd_f, cfg)
    lo = orc.backward(image, pose, focal, sel, tr)[0]
    l64, g64 = f64_grads(sd_c, sd_f, image, pose, focal, sel, tr, cfg)
    print(f"loss gpu {lg:.10g} oracle32 {lo:.10g} f64 {l64:.10g}")
    print(f"{'tensor':28s} {'gpu-vs-f64':>11s} {'o32-vs-f64':>11s} {'gpu-vs-o32':>11s}")
    for net in (0, 1):
        gg, go = gpu.grads(net), orc.grads(net)
        for k in T.PARAM_ORDER:
            print(f"{net} {k:26s} {rel(gg[k], g64[net][k]):11.3e} {rel(go[k], g64[net][k]):11.3e} "
                  f"{rel(gg[k], go[k]):11.3e}")


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
