"""ORACLE -- test infrastructure, not product code.

A CPU (PyTorch fp32, autograd) restatement of the reference's training step,
SURVEY §8f row 4 ("training-side stratified sampling with backward"):
``NeRFTrainer.train_step`` (``src/training/trainer.py:83-138``) with its ray
generation (``_get_rays``, ``:271-292``), its two-pass sampling
(``_render_rays``, ``:294-316``: coarse samples stratified by
``VolumeRenderer.sample_points_on_rays(perturb=True)``, ``src/utils/rendering.py:17-52``;
fine samples uniform), the chunked network query and ``volume_render``
(``_query_network``, ``:318-351``; ``rendering.py:102-143``), the two MSE
losses, backward, gradient clipping, Adam and the exponential lr schedule
(``:50-64``).

The two random draws of a step -- ``torch.randperm`` (``trainer.py:111``) and
``torch.rand_like`` (``rendering.py:47``) -- are inputs here, so the GPU path and
this restatement see the same ones.  The arithmetic the reference delegates to
PyTorch (autograd, ``clip_grad_norm_``, ``optim.Adam``, ``ExponentialLR``) is
PyTorch's own, called as the reference calls it.

Pinned by ``tests/golden/train.npz``, generated from the reference's
``NeRFTrainer`` itself (``tests/golden/make_golden_train.py``;
``tests/test_train_oracle.py``).  Only ``tests/`` and ``bench.py``'s
``cpu_baseline`` leg import this module; the product package never does.
"""
from __future__ import annotations

from typing import Dict, Mapping, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from oracle import nerf_oracle as O

# main.py:25-61 (get_default_config), the configuration `python main.py` trains with
TRAIN_CONFIG = {
    "lr": 3e-4,
    "lr_decay": 0.1,
    "decay_steps": 250000,
    "n_rays": 2048,
    "n_coarse": 64,
    "n_fine": 128,
    "chunk_size": 1024,
    "near": 2.0,
    "far": 6.0,
    "gradient_clipping": 1.0,
    "weight_decay": 1e-6,
}

PARAM_ORDER = ([f"layers.{i}.{k}" for i in range(8) for k in ("weight", "bias")]
               + ["density_head.weight", "density_head.bias"]
               + [f"color_layers.{i}.{k}" for i in range(2) for k in ("weight", "bias")])


def lr_gamma(config: Mapping) -> float:
    """ExponentialLR's gamma, trainer.py:62-64."""
    return config.get("lr_decay", 0.1) ** (1 / config.get("decay_steps", 250000))


def trainer_rays(c2w, height: int, width: int, focal: float):
    """trainer.py:271-292: pixel-corner grid, dir = ((i-W/2)/f, -(j-H/2)/f, -1),
    rays_d = the sum over the three products dir_c * R[r, c]; rays_o = translation."""
    c2w = O._t(c2w)
    cols = torch.linspace(0, width - 1, width)[None, :].expand(height, width)
    rows = torch.linspace(0, height - 1, height)[:, None].expand(height, width)
    f = float(focal)
    d = torch.stack([(cols - width * 0.5) / f, -(rows - height * 0.5) / f, -torch.ones_like(cols)], -1)
    rays_d = (d[..., None, :] * c2w[:3, :3]).sum(-1)
    rays_o = c2w[:3, -1].expand(rays_d.shape)
    return rays_o, rays_d


def volume_render_rgb(sigma, rgb, z, rays_d) -> torch.Tensor:
    """rgb_map of VolumeRenderer.volume_render (rendering.py:102-143), differentiable
    in sigma and rgb (oracle.composite detaches its inputs)."""
    dists = z[..., 1:] - z[..., :-1]
    dists = torch.cat([dists, torch.full_like(dists[..., :1], 1e10)], -1)
    dists = dists * torch.norm(rays_d[..., None, :], dim=-1)
    alpha = 1.0 - torch.exp(-F.relu(sigma[..., 0]) * dists)
    trans = torch.cumprod(1.0 - alpha + 1e-10, -1)
    trans = torch.cat([torch.ones_like(trans[..., :1]), trans[..., :-1]], -1)
    weights = alpha * trans
    return torch.sum(weights[..., None] * rgb, -2)


class TrainOracle:
    """NeRFTrainer's state and step on CPU tensors (coarse and fine NeRFModel
    parameters, one Adam over both, ExponentialLR)."""

    def __init__(self, sd_coarse: Mapping[str, np.ndarray], sd_fine: Mapping[str, np.ndarray],
                 config: Mapping = TRAIN_CONFIG):
        self.config = dict(TRAIN_CONFIG, **config)
        self.nets = [O.Net(sd_coarse), O.Net(sd_fine)]
        params = []
        for net in self.nets:
            for k in PARAM_ORDER:
                net.p[k].requires_grad_(True)
                params.append(net.p[k])
        self.params = params
        c = self.config
        self.optimizer = torch.optim.Adam(params, lr=c["lr"], weight_decay=c["weight_decay"])
        self.scheduler = torch.optim.lr_scheduler.ExponentialLR(self.optimizer, gamma=lr_gamma(c))

    @property
    def lr(self) -> float:
        return self.optimizer.param_groups[0]["lr"]

    def _render(self, net: O.Net, rays_o, rays_d, z) -> torch.Tensor:
        """_query_network (trainer.py:318-351): flatten, chunked query, volume_render."""
        pts = O.sample_points(rays_o, rays_d, z)
        flat = pts.reshape(-1, 3)
        dirs = rays_d[:, None, :].expand_as(pts).reshape(-1, 3)
        chunk = self.config["chunk_size"]
        sig, col = [], []
        for a in range(0, flat.shape[0], chunk):
            s, c = O.nerf_forward(net, flat[a:a + chunk], dirs[a:a + chunk])
            sig.append(s)
            col.append(c)
        sigma = torch.cat(sig).reshape(*pts.shape[:-1], 1)
        rgb = torch.cat(col).reshape(pts.shape)
        return volume_render_rgb(sigma, rgb, z, rays_d)

    def losses(self, image, c2w, focal: float, select, t_rand):
        """The forward half of train_step (trainer.py:96-122): (loss, mse_coarse, mse_fine)
        with the autograd graph attached."""
        image = O._t(image)
        height, width = image.shape[:2]
        rays_o, rays_d = trainer_rays(c2w, height, width, focal)
        sel = torch.as_tensor(np.asarray(select, dtype=np.int64))
        rays_o = rays_o.reshape(-1, 3)[sel]
        rays_d = rays_d.reshape(-1, 3)[sel]
        target = image.reshape(-1, 3)[sel]
        c = self.config
        n = rays_o.shape[0]
        z_c = O.stratified_z(O.uniform_z(c["n_coarse"], c["near"], c["far"]), O._t(t_rand).reshape(n, -1))
        z_f = O.uniform_z(c["n_fine"], c["near"], c["far"]).expand(n, c["n_fine"])
        rgb_c = self._render(self.nets[0], rays_o, rays_d, z_c)
        rgb_f = self._render(self.nets[1], rays_o, rays_d, z_f)
        mse_c = F.mse_loss(rgb_c, target)
        mse_f = F.mse_loss(rgb_f, target)
        return mse_c + mse_f, mse_c, mse_f

    def backward(self, image, c2w, focal: float, select, t_rand) -> Tuple[float, float, float]:
        """zero_grad + backward (trainer.py:121-126): leaves the unclipped gradients."""
        loss, mc, mf = self.losses(image, c2w, focal, select, t_rand)
        self.optimizer.zero_grad()
        loss.backward()
        return float(loss.detach()), float(mc.detach()), float(mf.detach())

    def clip(self) -> None:
        """trainer.py:128-133."""
        if self.config.get("gradient_clipping") is not None:
            torch.nn.utils.clip_grad_norm_(self.params, self.config["gradient_clipping"])

    def update(self) -> None:
        """optimizer.step + scheduler.step (trainer.py:135-136)."""
        self.optimizer.step()
        self.scheduler.step()

    def step(self, image, c2w, focal: float, select, t_rand) -> float:
        """NeRFTrainer.train_step: the step's loss (trainer.py:138)."""
        loss = self.backward(image, c2w, focal, select, t_rand)[0]
        self.clip()
        self.update()
        return loss

    def grads(self, net: int) -> Dict[str, np.ndarray]:
        return {k: self.nets[net].p[k].grad.detach().numpy().copy() for k in PARAM_ORDER}

    def params_np(self, net: int) -> Dict[str, np.ndarray]:
        return {k: self.nets[net].p[k].detach().numpy().copy() for k in PARAM_ORDER}

    def set_grads(self, grads: Sequence[Mapping[str, np.ndarray]]) -> None:
        """Install given gradients (e.g. the GPU's) so clip + Adam can be checked alone."""
        for net, g in zip(self.nets, grads):
            for k in PARAM_ORDER:
                net.p[k].grad = torch.as_tensor(np.asarray(g[k], dtype=np.float32)).clone()


def step_grads_f64(sd_c, sd_f, image, pose, focal, sel, t_rand, config):
    """One step's loss and both nets' gradients evaluated in float64: the ground truth that
    an fp32 step (the reference's, this oracle's) and the GPU's split-bf16 step are each
    measured against (tests/test_gpu_train.py, tools/train_diag.py).  The same graph as
    TrainOracle.backward (nerf.py:24-45, 92-131; rendering.py:102-143; trainer.py:117-126)."""
    dt = torch.float64
    nets = [{k: torch.tensor(np.asarray(v, np.float64), requires_grad=True) for k, v in sd.items()}
            for sd in (sd_c, sd_f)]

    def lin(p, name, x):
        return F.linear(x, p[f"{name}.weight"], p[f"{name}.bias"])

    def pe(x, levels):
        out = [x]
        for k in range(levels):
            a = (2.0 ** k) * np.pi * x
            out += [torch.sin(a), torch.cos(a)]
        return torch.cat(out, -1)

    def fwd(p, pts, dirs):
        e = pe(pts, 10)
        x = e
        for i in range(8):
            if i == 4:
                x = torch.cat([x, e], -1)
            x = F.relu(lin(p, f"layers.{i}", x))
        s = F.relu(lin(p, "density_head", x))
        h = F.relu(lin(p, "color_layers.0", torch.cat([x, pe(dirs, 4)], -1)))
        return s, torch.sigmoid(lin(p, "color_layers.1", h))

    ro, rd = trainer_rays(pose, image.shape[0], image.shape[1], focal)
    ro, rd = ro.reshape(-1, 3)[sel].to(dt), rd.reshape(-1, 3)[sel].to(dt)
    tgt = torch.as_tensor(image).reshape(-1, 3)[sel].to(dt)
    n = ro.shape[0]
    zc = O.stratified_z(O.uniform_z(config["n_coarse"]), torch.as_tensor(t_rand).reshape(n, -1)).to(dt)
    zf = O.uniform_z(config["n_fine"]).expand(n, config["n_fine"]).to(dt)
    loss = 0
    for p, z in zip(nets, (zc, zf)):
        pts = ro[:, None, :] + rd[:, None, :] * z[..., None]
        s, c = fwd(p, pts.reshape(-1, 3), rd[:, None, :].expand_as(pts).reshape(-1, 3))
        rgb = volume_render_rgb(s.reshape(n, -1, 1), c.reshape(n, -1, 3), z, rd)
        loss = loss + F.mse_loss(rgb, tgt)
    loss.backward()
    return float(loss.detach()), [{k: v.grad.numpy() for k, v in p.items()} for p in nets]

