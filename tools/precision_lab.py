"""Per-layer operand-precision emulation of the NeRF MLP (CPU, PyTorch).

    python tools/precision_lab.py [--ckpt synthetic|lego] [--schemes ...]

Each Linear's operands are rounded to a chosen form before an fp32 matmul (fp32
accumulation, as the MFMA does); split forms add the partial products of the hi/lo
halves.  The rendered RGB / depth are compared with the fp32 forward on the same
rays (render_image semantics: uniform samples, pytorch_renderers.py:105-125), to
find per-layer schemes that stay under the north star's 1e-4 gate with the fewest
MFMAs per product.  The layer list is the 10 Linears of NeRFModel in forward order.

Forms:  f32 | bf16 | fp16 (one product) | fp16w (Wh.Xh + Wl.Xh: weights split) |
        fp16x (Wh.Xh + Wh.Xl: activations split) | fp16x3 / bf16x3 (three products)
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nerf-dbr_amd"))
sys.path.insert(0, REPO)

from nerf_amd import weights as W  # noqa: E402

LAYERS = [n for n, _, _ in W.LAYER_SPECS]
COST = {"f32": 1, "bf16": 1, "fp16": 1, "fp16w": 2, "fp16x": 2, "fp16x3": 3, "bf16x3": 3}


def _r(x, fmt):
    return x.to(fmt).to(torch.float32)


def linear(x, w, b, form):
    """x [N, in] fp32, w [out, in], b [out] -> x W^T + b with the form's operand rounding."""
    if form == "f32":
        return x @ w.t() + b
    fmt = torch.bfloat16 if form.startswith("bf16") else torch.float16
    xh, wh = _r(x, fmt), _r(w, fmt)
    y = xh @ wh.t()
    if form in ("fp16w", "fp16x3", "bf16x3"):
        y = y + xh @ _r(w - wh, fmt).t()
    if form in ("fp16x", "fp16x3", "bf16x3"):
        y = y + _r(x - xh, fmt) @ wh.t()
    return y + b


def pe(x, L):
    out = [x]
    for k in range(L):
        f = float(2.0 ** k) * math.pi
        out += [torch.sin(f * x), torch.cos(f * x)]
    return torch.cat(out, -1)


def forward(sd, pos, dirs, forms):
    p = pe(pos, W.POS_L)
    h = p
    for i in range(8):
        if i == W.SKIP_LAYER:
            h = torch.cat([h, p], -1)
        n = f"layers.{i}"
        h = torch.relu(linear(h, sd[n + ".weight"], sd[n + ".bias"], forms[n]))
    sigma = torch.relu(linear(h, sd["density_head.weight"], sd["density_head.bias"], forms["density_head"]))
    c = torch.relu(linear(torch.cat([h, pe(dirs, W.DIR_L)], -1), sd["color_layers.0.weight"],
                          sd["color_layers.0.bias"], forms["color_layers.0"]))
    rgb = torch.sigmoid(linear(c, sd["color_layers.1.weight"], sd["color_layers.1.bias"], forms["color_layers.1"]))
    return sigma, rgb


def render(sd, pose, w, h, spp, forms, rows=None, chunk=4096):
    from oracle import nerf_oracle as O

    o, d = O.generate_rays(pose, w, h)
    r0, r1 = rows or (0, h)
    o, d = o[r0:r1].reshape(-1, 3), d[r0:r1].reshape(-1, 3)
    z = O.uniform_z(spp)
    rgbs, deps = [], []
    with torch.no_grad():
        for c in range(0, o.shape[0], chunk):
            oo, dd = o[c:c + chunk], d[c:c + chunk]
            zz = z.expand(oo.shape[0], spp)
            pts = oo[:, None] + dd[:, None] * zz[..., None]
            s, col = forward(sd, pts.reshape(-1, 3), dd[:, None].expand_as(pts).reshape(-1, 3), forms)
            r_, d_ = O.composite(s.reshape(-1, spp, 1), col.reshape(-1, spp, 3), zz, dd)
            rgbs.append(r_)
            deps.append(d_)
    return torch.cat(rgbs), torch.cat(deps)


def scheme(default, **over):
    f = {n: default for n in LAYERS}
    for k, v in over.items():
        f[k.replace("__", ".")] = v
    return f


def mean_cost(forms):
    macs = {n: o * i for n, o, i in W.LAYER_SPECS}
    return sum(COST[forms[n]] * macs[n] for n in LAYERS) / sum(macs.values())


SCHEMES = {
    "bf16": scheme("bf16"),
    "fp16": scheme("fp16"),
    "fp16w": scheme("fp16w"),
    "fp16x": scheme("fp16x"),
    "bf16x3": scheme("bf16x3"),
    "fp16x3": scheme("fp16x3"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ckpt", default="synthetic", choices=["synthetic", "lego"])
    ap.add_argument("--schemes", nargs="*", default=list(SCHEMES))
    ap.add_argument("--res", type=int, nargs=3, default=[200, 150, 32])
    ap.add_argument("--per-layer", action="store_true", help="fp16 everywhere but one layer in fp16x3, and vice versa")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    _, fine = W.synthetic_models(0) if args.ckpt == "synthetic" else W.lego_models()
    sd = {k: torch.from_numpy(v) for k, v in fine.items()}
    w, h, spp = args.res
    from nerf_amd.benchmark.benchmark_suite import generate_test_poses

    pose = generate_test_poses(2)[0]
    ref_rgb, ref_dep = render(sd, pose, w, h, spp, scheme("f32"))
    runs = dict((k, SCHEMES[k]) for k in args.schemes)
    if args.per_layer:
        for n in LAYERS:
            runs[f"fp16 but {n} fp16x3"] = scheme("fp16", **{n.replace('.', '__'): "fp16x3"})
            runs[f"fp16x3 but {n} fp16"] = scheme("fp16x3", **{n.replace('.', '__'): "fp16"})
    for name, forms in runs.items():
        rgb, dep = render(sd, pose, w, h, spp, forms)
        er = float((rgb - ref_rgb).abs().max())
        ed = float((dep - ref_dep).abs().max())
        print(f"{name:40s} cost {mean_cost(forms):.3f}  rgb max {er:.3e} mean {float((rgb - ref_rgb).abs().mean()):.2e}"
              f"  depth max {ed:.3e}", flush=True)


if __name__ == "__main__":
    main()
