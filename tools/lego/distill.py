"""Distil the original-NeRF Lego networks into the reference's ``NeRFModel`` layout.

    python -m tools.lego.distill --out DIR [--steps-fine N] [--steps-coarse N]

Runs on the GPU box (PyTorch on ``cuda:0``; this is an offline tool that makes a
checkpoint, not part of the render path).  Teacher: ``tools/lego/teacher.py``
(the bundled ``model_fine_200000.npy`` / ``model_200000.npy``, read by the static
parser).  Student: ``NeRFModel`` (``src/models/nerf.py:48-131``) restated with
autograd below, initialised with ``nn.Linear``'s default init under
``torch.manual_seed``.

Every step draws rays the way the reference's renderers form them
(``base_renderer.py:223-258``: unnormalised ``d = R [u, v, -1]``) from random
cameras on the upper hemisphere around the scene (radius 3-5, random roll), plus
the benchmark suite's pose family (translation (0,0,4), rotation about Y;
``benchmark_suite.py:132-149``); 128 stratified samples in [2, 6] plus 64 drawn
from the teacher's weights on them, sorted.  The loss compares student and
teacher on the same samples:

* the ray colour composited with the reference's formula
  (``pytorch_renderers.py:105-125``: black background, last distance 1e10);
* opacity at two spacings, ``1 - exp(-sigma * 0.03)`` and ``1 - exp(-sigma * 0.005)``,
  per sample (geometry and depth at every sample count of the README grid);
* per-sample colour weighted by the teacher's compositing weights.

Adam, learning rate decayed exponentially (5e-4 to 2.5e-5 by default; ``--init``
continues from an earlier run's weights); the networks run under bf16 autocast
(the rendering and the loss in fp32).  At the end both
nets are rendered against the teacher on held-out poses with the reference's
render semantics (uniform samples, black background) and the PSNR is written to
``report.json`` beside ``lego_distilled.npz`` (``coarse/<param>``, ``fine/<param>``,
raw fp32 in ``nn.Linear`` layout).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "nerf-dbr_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

from lego.teacher import load_teacher  # noqa: E402
from nerf_amd import weights as W  # noqa: E402

NEAR, FAR = 2.0, 6.0


class Student(torch.nn.Module):
    """NeRFModel (nerf.py:48-131): PE with pi (nerf.py:41-43), skip cat([x, pe]) before
    layer 4 (nerf.py:108-110), relu density head, colour head on cat([x, pe4(d)])."""

    def __init__(self):
        super().__init__()
        self.lin = torch.nn.ModuleDict()
        for name, o, i in W.LAYER_SPECS:
            self.lin[name.replace(".", "_")] = torch.nn.Linear(i, o)

    @staticmethod
    def pe(x, L):
        out = [x]
        for k in range(L):
            f = float(2.0 ** k) * math.pi
            out.append(torch.sin(x * f))
            out.append(torch.cos(x * f))
        return torch.cat(out, dim=-1)

    def forward(self, x, d):
        pe = self.pe(x, W.POS_L)
        h = pe
        for i in range(8):
            if i == W.SKIP_LAYER:
                h = torch.cat([h, pe], dim=-1)
            h = F.relu(self.lin[f"layers_{i}"](h))
        sigma = F.relu(self.lin["density_head"](h))
        c = F.relu(self.lin["color_layers_0"](torch.cat([h, self.pe(d, W.DIR_L)], dim=-1)))
        return sigma, torch.sigmoid(self.lin["color_layers_1"](c))

    def state_np(self):
        return {f"{name}.{s}": getattr(self.lin[name.replace('.', '_')], s).detach().cpu().numpy().astype(np.float32)
                for name, _, _ in W.LAYER_SPECS for s in ("weight", "bias")}


def composite(sigma, rgb, z, d):
    """pytorch_renderers.py:105-125 on [R,S] sigma, [R,S,3] rgb, [R,S] z, [R,3] d."""
    dists = z[:, 1:] - z[:, :-1]
    dists = torch.cat([dists, torch.full_like(dists[:, :1], 1e10)], dim=-1) * torch.norm(d, dim=-1, keepdim=True)
    alpha = 1.0 - torch.exp(-F.relu(sigma) * dists)
    tr = torch.cumprod(1.0 - alpha + 1e-10, dim=-1)
    tr = torch.cat([torch.ones_like(tr[:, :1]), tr[:, :-1]], dim=-1)
    w = alpha * tr
    return (w[..., None] * rgb).sum(1), (w * z).sum(1), w


def look_at(eye, target, roll):
    """c2w [B,4,4]: camera looks along -z at target (Blender / reference convention)."""
    zc = F.normalize(eye - target, dim=-1)
    up = torch.tensor([0.0, 0.0, 1.0], device=eye.device).expand_as(zc)
    alt = torch.tensor([0.0, 1.0, 0.0], device=eye.device).expand_as(zc)
    up = torch.where((zc[:, 2:3].abs() > 0.999), alt, up)
    xc = F.normalize(torch.cross(up, zc, dim=-1), dim=-1)
    yc = torch.cross(zc, xc, dim=-1)
    c, s = torch.cos(roll)[:, None], torch.sin(roll)[:, None]
    xr, yr = c * xc + s * yc, -s * xc + c * yc
    m = torch.zeros(eye.shape[0], 4, 4, device=eye.device)
    m[:, :3, 0], m[:, :3, 1], m[:, :3, 2], m[:, :3, 3], m[:, 3, 3] = xr, yr, zc, eye, 1.0
    return m


def suite_family(n, g, dev):
    """benchmark_suite.py:132-149's construction at a random angle."""
    a = torch.rand(n, generator=g, device=dev) * 2 * math.pi
    m = torch.zeros(n, 4, 4, device=dev)
    m[:, 0, 0], m[:, 0, 2], m[:, 2, 0], m[:, 2, 2] = torch.cos(a), torch.sin(a), -torch.sin(a), torch.cos(a)
    m[:, 1, 1], m[:, 2, 3], m[:, 3, 3] = 1.0, 4.0, 1.0
    return m


def draw_rays(n, g, dev):
    """n rays, one camera each (reference ray convention, unnormalised directions)."""
    n_suite = n // 5
    n_hemi = n - n_suite
    u = torch.rand(n_hemi, generator=g, device=dev)
    cz = 0.02 + 0.98 * u                          # elevation: cos(theta) in (0.02, 1]
    ph = torch.rand(n_hemi, generator=g, device=dev) * 2 * math.pi
    sz = torch.sqrt(1 - cz * cz)
    rad = 3.0 + 2.0 * torch.rand(n_hemi, generator=g, device=dev)
    eye = torch.stack([sz * torch.cos(ph), sz * torch.sin(ph), cz], -1) * rad[:, None]
    tgt = torch.randn(n_hemi, 3, generator=g, device=dev) * 0.3
    roll = torch.rand(n_hemi, generator=g, device=dev) * 2 * math.pi
    c2w = torch.cat([look_at(eye, tgt, roll), suite_family(n_suite, g, dev)])
    uv = (torch.rand(n, 2, generator=g, device=dev) * 2 - 1) * 0.62
    dirs = torch.cat([uv[:, :1], uv[:, 1:], -torch.ones(n, 1, device=dev)], -1)
    d = (dirs[:, None, :] * c2w[:, :3, :3]).sum(-1)
    o = c2w[:, :3, 3]
    return o, d


def sample_pdf(z, w, n, g):
    """Inverse-CDF draw of n depths per ray from weights w on bin edges between z."""
    mids = 0.5 * (z[:, 1:] + z[:, :-1])
    wt = w[:, 1:-1] + 1e-5
    pdf = wt / wt.sum(-1, keepdim=True)
    cdf = torch.cat([torch.zeros_like(pdf[:, :1]), torch.cumsum(pdf, -1)], -1)
    u = torch.rand(z.shape[0], n, generator=g, device=z.device)
    idx = torch.searchsorted(cdf, u.contiguous(), right=True)
    lo = (idx - 1).clamp(min=0)
    hi = idx.clamp(max=cdf.shape[1] - 1)
    c_lo, c_hi = torch.gather(cdf, 1, lo), torch.gather(cdf, 1, hi)
    b_lo, b_hi = torch.gather(mids, 1, lo), torch.gather(mids, 1, hi)
    den = torch.where(c_hi - c_lo < 1e-5, torch.ones_like(c_lo), c_hi - c_lo)
    return b_lo + (u - c_lo) / den * (b_hi - b_lo)


def _amp(dev):
    return torch.autocast(dev.type, dtype=torch.bfloat16)


def _query(net, o, d, z, dev):
    r, s = z.shape
    p = (o[:, None] + d[:, None] * z[..., None]).reshape(-1, 3)
    with _amp(dev):
        sg, cl = net(p, d[:, None].expand(r, s, 3).reshape(-1, 3))
    return sg.float().reshape(r, s), cl.float().reshape(r, s, 3)


def ray_samples(o, d, teacher, g, s_strat=128, s_imp=64):
    """Sorted depths [R, s_strat + s_imp] and the teacher's (sigma, rgb) on them (the
    stratified part evaluated once, the importance part after it)."""
    r = o.shape[0]
    dev = o.device
    edges = torch.linspace(NEAR, FAR, s_strat + 1, device=dev)
    z = edges[:-1] + (edges[1:] - edges[:-1]) * torch.rand(r, s_strat, generator=g, device=dev)
    with torch.no_grad():
        sg, cl = _query(teacher, o, d, z, dev)
        _, _, w = composite(sg, cl, z, d)
        zi = sample_pdf(z, w, s_imp, g)
        si, ci = _query(teacher, o, d, zi, dev)
        z, order = torch.sort(torch.cat([z, zi], -1), -1)
        st = torch.gather(torch.cat([sg, si], -1), 1, order)
        ct = torch.gather(torch.cat([cl, ci], 1), 1, order[..., None].expand(-1, -1, 3))
    return z, st, ct


def loss_fn(student, o, d, z, st, ct):
    r, s = z.shape
    with torch.no_grad():
        Ct, Dt, wt = composite(st, ct, z, d)
    ss, cs = _query(student, o, d, z, o.device)
    Cs, Ds, _ = composite(ss, cs, z, d)
    l_rgb = F.mse_loss(Cs, Ct)
    l_a = F.mse_loss(1 - torch.exp(-ss * 0.03), 1 - torch.exp(-st * 0.03))
    l_b = F.mse_loss(1 - torch.exp(-ss * 0.005), 1 - torch.exp(-st * 0.005))
    l_col = (wt[..., None] * (cs - ct) ** 2).sum() / (r * 3)
    parts = {"rgb": l_rgb.item(), "alpha": l_a.item(), "col": l_col.item()}
    return l_rgb + l_col + 0.5 * (l_a + l_b), parts


def train(which, steps, rays, seed, budget_s, log, dev, init=None, lr0=5e-4, lr1=2.5e-5):
    """Adam with the rate decayed exponentially 5e-4 -> 2.5e-5 over the run; the run is
    ``steps`` long, or shorter when the pace of steps 20-60 says ``budget_s`` seconds
    would not cover it (the decay is then re-spread over the steps that fit)."""
    teacher = load_teacher(which, dev)
    torch.manual_seed(seed)
    student = Student()
    if init is not None:                      # continue from an earlier run's weights
        for name, _, _ in W.LAYER_SPECS:
            lin = student.lin[name.replace(".", "_")]
            lin.weight.data.copy_(torch.from_numpy(init[f"{which}/{name}.weight"]))
            lin.bias.data.copy_(torch.from_numpy(init[f"{which}/{name}.bias"]))
    student = student.to(dev)
    opt = torch.optim.Adam(student.parameters(), lr=lr0)
    g = torch.Generator(device=dev).manual_seed(seed + 17)
    t0 = time.time()
    last = t0
    it = 0
    while it < steps:
        if it == 20:                           # pace from steps 20..60 (the first ones warm up)
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            t20 = time.time()
        if it == 60:
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            pace = (time.time() - t20) / 40
            steps = max(61, min(steps, 60 + int((budget_s - (time.time() - t0)) / pace)))
            log(f"[{which}] {1e3 * pace:.1f} ms/step -> {steps} steps")
        lr = lr0 * (lr1 / lr0) ** (it / max(1, steps - 1))
        for grp in opt.param_groups:
            grp["lr"] = lr
        o, d = draw_rays(rays, g, dev)
        z, st, ct = ray_samples(o, d, teacher, g)
        loss, parts = loss_fn(student, o, d, z, st, ct)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        if time.time() - last > 20 or it == steps - 1:
            last = time.time()
            log(f"[{which}] step {it + 1}/{steps} loss {float(loss):.3e} {parts} "
                f"psnr_ray {-10 * math.log10(max(parts['rgb'], 1e-12)):.2f} dB  {last - t0:.0f}s")
        it += 1
    return student, teacher, steps


def eval_poses():
    """Held-out poses (fixed seed, not drawn by training): 6 hemisphere views at r=4.03,
    the suite's view 0 and the golden off-axis look-at (tests/golden/make_golden.py)."""
    g = torch.Generator().manual_seed(12345)
    out = []
    for _ in range(6):
        cz = 0.15 + 0.8 * torch.rand(1, generator=g)
        ph = torch.rand(1, generator=g) * 2 * math.pi
        sz = torch.sqrt(1 - cz * cz)
        eye = torch.cat([sz * torch.cos(ph), sz * torch.sin(ph), cz])[None] * 4.03
        out.append(look_at(eye, torch.zeros(1, 3), torch.zeros(1))[0])
    p = torch.eye(4)
    p[2, 3] = 4.0
    out.append(p)
    eye = np.array([2.7, 1.9, 2.3])
    fwd = -eye / np.linalg.norm(eye)
    right = np.cross(fwd, [0.0, 1.0, 0.0])
    right /= np.linalg.norm(right)
    m = np.eye(4)
    m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = right, np.cross(right, fwd), -fwd, eye
    out.append(torch.tensor(m, dtype=torch.float32))
    return out


@torch.no_grad()
def render(net, c2w, w, h, focal, spp, dev, chunk=4096):
    """The reference's render_image semantics (uniform z, black background)."""
    c2w = c2w.to(dev)
    i, j = torch.meshgrid(torch.linspace(0, w - 1, w, device=dev), torch.linspace(0, h - 1, h, device=dev),
                          indexing="ij")
    i, j = i.t(), j.t()
    dirs = torch.stack([(i - w * 0.5) / focal, -(j - h * 0.5) / focal, -torch.ones_like(i)], -1)
    d = torch.sum(dirs[..., None, :] * c2w[:3, :3], -1).reshape(-1, 3)
    o = c2w[:3, -1].expand(d.shape)
    t = torch.linspace(0.0, 1.0, spp, device=dev)
    z = (NEAR * (1.0 - t) + FAR * t).expand(d.shape[0], spp)
    rgb, dep = [], []
    for c in range(0, d.shape[0], chunk):
        oo, dd, zz = o[c:c + chunk], d[c:c + chunk], z[c:c + chunk]
        p = oo[:, None] + dd[:, None] * zz[..., None]
        s_, c_ = net(p.reshape(-1, 3), dd[:, None].expand_as(p).reshape(-1, 3))
        r_, d_, _ = composite(s_.reshape(-1, spp), c_.reshape(-1, spp, 3), zz, dd)
        rgb.append(r_)
        dep.append(d_)
    return torch.cat(rgb).reshape(h, w, 3), torch.cat(dep).reshape(h, w)


def psnr(a, b):
    return float(-10 * torch.log10(F.mse_loss(a, b)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps-fine", type=int, default=12000)
    ap.add_argument("--steps-coarse", type=int, default=6000)
    ap.add_argument("--rays", type=int, default=2048)
    ap.add_argument("--budget-fine", type=float, default=480.0, help="seconds")
    ap.add_argument("--budget-coarse", type=float, default=240.0, help="seconds")
    ap.add_argument("--eval-res", type=int, nargs=2, default=[400, 300])
    ap.add_argument("--init", default=None, help="lego_distilled.npz of an earlier run to continue from")
    ap.add_argument("--lr", type=float, nargs=2, default=[5e-4, 2.5e-5], help="start, end")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    dev = torch.device(os.environ.get("DISTILL_DEVICE", "cuda:0"))

    def log(msg):
        print(msg, flush=True)

    report = {"recipe": {k: v for k, v in vars(args).items() if k != "out"},
              "teacher": "data/lego_example_weights/model{_fine,}_200000.npy (original NeRF, 8x256, args.txt)",
              "student": "NeRFModel (src/models/nerf.py:48-131), nn.Linear default init, torch.manual_seed",
              "torch": torch.__version__}
    ckpt = {}
    w, h = args.eval_res
    focal = 800.0 * w / 800.0
    for which, steps, seed, budget in (("fine", args.steps_fine, 1, args.budget_fine),
                                       ("coarse", args.steps_coarse, 0, args.budget_coarse)):
        t0 = time.time()
        init = dict(np.load(args.init)) if args.init else None
        student, teacher, steps = train(which, steps, args.rays, seed, budget, log, dev, init, *args.lr)
        for k, v in student.state_np().items():
            ckpt[f"{which}/{k}"] = v
        np.savez(os.path.join(args.out, "lego_distilled.npz"), **ckpt)
        rows = []
        for pi, pose in enumerate(eval_poses()):
            for spp in (64, 128):
                rs, ds = render(student, pose, w, h, focal, spp, dev)
                rt, dt = render(teacher, pose, w, h, focal, spp, dev)
                rows.append({"pose": pi, "spp": spp, "psnr_db": psnr(rs, rt),
                             "rgb_max_abs": float((rs - rt).abs().max()),
                             "depth_mean_abs": float((ds - dt).abs().mean()),
                             "teacher_rgb_mean": float(rt.mean())})
        report[which] = {"steps": steps, "seed": seed, "train_seconds": time.time() - t0,
                         "eval": f"{w}x{h}, focal {focal:g} (the 800x600 / focal 800 field of view), uniform "
                                 f"samples in [2, 6], black background (PyTorchCPURenderer semantics)",
                         "views": rows,
                         "psnr_db_mean": float(np.mean([r_["psnr_db"] for r_ in rows]))}
        log(f"[{which}] held-out PSNR mean {report[which]['psnr_db_mean']:.2f} dB")
        with open(os.path.join(args.out, "report.json"), "w") as f:
            json.dump(report, f, indent=1)
    log(json.dumps({k: report[k]["psnr_db_mean"] for k in ("fine", "coarse")}))


if __name__ == "__main__":
    main()
