"""Generate tests/golden/train.npz from the reference's NeRFTrainer itself.

Run in the development container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train.py [/root/reference]

It imports ``src.training.trainer.NeRFTrainer`` (bypassing ``src/benchmark/__init__.py``
as make_golden.py does), loads the deterministic synthetic checkpoint of
``nerf_amd.weights`` into its coarse and fine models, and runs three
``train_step`` calls (trainer.py:83-138) on a small synthetic target image with
``main.py``'s default training configuration (main.py:25-61; n_rays reduced).
``torch.randperm`` and ``torch.rand_like`` are wrapped to record the draws the
step makes (trainer.py:111, rendering.py:47), so a restatement can be fed the
same ones.  Recorded (data only, no source): the rays of ``_get_rays``, per step
the draws, the loss and the lr; the (clipped) gradients after step 1 and the
parameters after step 3 as fixed index samples of every tensor plus float64
sums and norms of the whole tensors.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "nerf-dbr_amd"))

from nerf_amd import weights as W  # noqa: E402

H, WD = 30, 40
N_RAYS = 256
N_STEPS = 3
SEED = 1234


def sample_index(n: int) -> np.ndarray:
    """Entries of a flattened tensor kept in the fixture: the first 256, then every 61st."""
    return np.unique(np.concatenate([np.arange(min(n, 256)), np.arange(0, n, 61)]))


def target_image() -> np.ndarray:
    rng = np.random.RandomState(7)
    yy, xx = np.mgrid[0:H, 0:WD].astype(np.float32)
    img = np.stack([xx / WD, yy / H, 0.5 + 0.5 * np.sin(xx * 0.3) * np.cos(yy * 0.2)], -1)
    img = 0.8 * img + 0.2 * rng.rand(H, WD, 3)
    return img.astype(np.float32)


def train_pose() -> np.ndarray:
    """A look-at pose in the style of the synthetic dataset's transform_matrix."""
    eye = np.array([1.9, 2.6, 2.2])
    fwd = -eye / np.linalg.norm(eye)
    right = np.cross(fwd, [0.0, 0.0, 1.0])
    right /= np.linalg.norm(right)
    up = np.cross(right, fwd)
    c2w = np.eye(4)
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = right, up, -fwd, eye
    return c2w.astype(np.float32)


def main(ref_root: str = "/root/reference") -> None:
    sys.path.insert(0, ref_root)
    import src  # noqa: F401

    bp = types.ModuleType("src.benchmark")
    bp.__path__ = [os.path.join(ref_root, "src", "benchmark")]
    sys.modules["src.benchmark"] = bp
    import torch
    from src.training.trainer import NeRFTrainer

    config = {
        "device": "cpu", "lr": 3e-4, "lr_decay": 0.1, "decay_steps": 250000, "n_rays": N_RAYS,
        "n_coarse": 64, "n_fine": 128, "hidden_dim": 256, "position_encoding_levels": 10,
        "direction_encoding_levels": 4, "chunk_size": 1024, "near": 2.0, "far": 6.0,
        "gradient_clipping": 1.0, "weight_decay": 1e-6,
    }
    tr = NeRFTrainer(config)
    sd_c, sd_f = W.synthetic_models(0)
    for model, sd in ((tr.coarse_model, sd_c), (tr.fine_model, sd_f)):
        model.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    names = [k for k, _ in tr.coarse_model.named_parameters()]

    image = target_image()
    pose = train_pose()
    focal = 0.5 * WD / np.tan(0.5 * 0.6911112070083618)    # loader.py:36 with the Lego camera angle
    batch = {"image": torch.from_numpy(image), "pose": torch.from_numpy(pose), "focal": focal}

    out = {"image": image, "pose": pose, "focal": np.float64(focal), "n_rays": np.int64(N_RAYS)}
    rays_o, rays_d = tr._get_rays(batch["pose"], image.shape[:2], focal)
    out["rays_o"], out["rays_d"] = rays_o.numpy(), rays_d.numpy()

    draws = {}
    real_randperm, real_rand_like = torch.randperm, torch.rand_like

    def randperm(*a, **k):
        r = real_randperm(*a, **k)
        draws["randperm"] = r.clone()
        return r

    def rand_like(*a, **k):
        r = real_rand_like(*a, **k)
        draws["rand_like"] = r.clone()
        return r

    torch.manual_seed(SEED)
    torch.randperm, torch.rand_like = randperm, rand_like
    try:
        for step in range(N_STEPS):
            loss = tr.train_step(batch)
            out[f"step{step}_select"] = draws["randperm"][:N_RAYS].numpy().astype(np.int64)
            out[f"step{step}_t_rand"] = draws["rand_like"].numpy()
            out[f"step{step}_loss"] = np.float64(loss)
            out[f"step{step}_lr"] = np.float64(tr.optimizer.param_groups[0]["lr"])
            if step == 0:
                for net, model in (("coarse", tr.coarse_model), ("fine", tr.fine_model)):
                    for k, p in model.named_parameters():
                        g = p.grad.detach().numpy().ravel()
                        out[f"grad1_{net}_{k}"] = g[sample_index(g.size)]
                        out[f"grad1_{net}_{k}_stats"] = np.array(
                            [g.astype(np.float64).sum(), np.abs(g.astype(np.float64)).sum(),
                             np.sqrt((g.astype(np.float64) ** 2).sum())])
    finally:
        torch.randperm, torch.rand_like = real_randperm, real_rand_like
    for net, model in (("coarse", tr.coarse_model), ("fine", tr.fine_model)):
        for k, p in model.named_parameters():
            v = p.detach().numpy().ravel()
            out[f"param3_{net}_{k}"] = v[sample_index(v.size)]
            out[f"param3_{net}_{k}_stats"] = np.array([v.astype(np.float64).sum(),
                                                        np.abs(v.astype(np.float64)).sum()])
    out["param_names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "train.npz"), **out)
    print("wrote train.npz:", {k: out[f"step{s}_loss"] for s in range(N_STEPS) for k in ["loss"]})


if __name__ == "__main__":
    main(*sys.argv[1:])
