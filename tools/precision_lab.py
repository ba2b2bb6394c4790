"""Per-layer operand-precision emulation of the NeRF MLP (CPU, PyTorch).

    python tools/precision_lab.py [--ckpt synthetic|lego] [--schemes ...]

Each Linear's operands are rounded to a chosen form before an fp32 matmul (fp32
accumulation, as the MFMA does); split forms add the partial products of the hi/lo
halves.  The rendered RGB / depth are compared with the fp32 forward on the same
rays (render_image semantics: uniform samples, pytorch_renderers.py:105-125), to
find per-layer schemes that stay under the north star's 1e-4 gate with the fewest
MFMAs per product.  The layer list is the 10 Linears of NeRFModel in forward order.

Forms:  f32 | bf16 | fp16 (one product) | fp16w (Wh.Xh + Wl.Xh: weights split) |
        fp16x (Wh.Xh + Wh.Xl: activations split) | fp16x3 / bf16x3 (three products) |
        h<fmt>[<mode>] (round 5: Wh.Xh in fp16 and the two cross products Wh.Xl + Wl.Xh on the
        block-scaled MFMA v_mfma_scale_f32_32x32x64_f8f6f4 with operands in <fmt> = e4m3,
        e5m2, e2m3 or e3m2; every 32-k block of a weight row or of a sample's activations has
        its own power-of-two (E8M0) scale, from the block's max (mode "") or, for the
        activations, one fixed scale per layer (mode "f", the weights keep their block scales))
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
# minifloat formats of the f8f6f4 MFMA: (mantissa bits, smallest normal exponent, largest value)
MINI = {"e4m3": (3, -6, 448.0), "e5m2": (2, -14, 57344.0), "e2m3": (3, 0, 7.5), "e3m2": (2, -2, 28.0)}
# MFMA cycles per 16 k of the cross products (two of them): fp8 64 cycles per 64 k, fp6 32
CROSS_COST = {"e4m3": 0.5, "e5m2": 0.5, "e2m3": 0.25, "e3m2": 0.25}


def mini_round(x, fmt):
    """Round to the nearest value of the minifloat (ties to even), saturating."""
    mb, emin, vmax = MINI[fmt]
    a = x.abs()
    e = torch.floor(torch.log2(a.clamp_min(1e-38))).clamp_min(emin)
    q = torch.exp2(e - mb)
    return (torch.round(x / q) * q).clamp(-vmax, vmax)


def block_scaled(x, fmt, fixed=None, blk=32):
    """x [N, K]: each row's 32-k blocks scaled by 2^ceil(log2(max / vmax)) (or one fixed
    power of two), rounded to fmt, and scaled back."""
    n, k = x.shape
    kp = (k + blk - 1) // blk * blk
    xp = torch.nn.functional.pad(x, (0, kp - k)).reshape(n, kp // blk, blk)
    vmax = MINI[fmt][2]
    if fixed is None:
        m = xp.abs().amax(-1, keepdim=True).clamp_min(1e-30)
        sc = torch.exp2(torch.ceil(torch.log2(m / vmax)))
    else:
        sc = torch.full_like(xp[..., :1], fixed)
    return (mini_round(xp / sc, fmt) * sc).reshape(n, kp)[:, :k]


def _r(x, fmt):
    return x.to(fmt).to(torch.float32)


def mant_cut(v, b):
    """Round an fp16-valued tensor to b explicit mantissa bits (nearest), as an fp16 bit mask would leave it."""
    m, e = torch.frexp(v)
    return torch.ldexp(torch.round(m * 2.0 ** (b + 1)) / 2.0 ** (b + 1), e)


def linear(x, w, b, form):
    """x [N, in] fp32, w [out, in], b [out] -> x W^T + b with the form's operand rounding."""
    b_ = b
    if form == "f32":
        return x @ w.t() + b
    if form.startswith("h"):
        fmt, mode = form[1:5], form[5:]
        xh, wh = _r(x, torch.float16), _r(w, torch.float16)
        xl, wl = x - xh, w - wh
        if mode == "f":   # fixed activation scales: Xh at the layer's max, Xl 2^-11 below it
            sx = float(2.0 ** math.ceil(math.log2(max(float(x.abs().max()), 1e-30) / MINI[fmt][2])))
            qxh, qxl = block_scaled(x, fmt, sx), block_scaled(xl, fmt, sx * 2.0 ** -11)
        else:
            qxh, qxl = block_scaled(x, fmt), block_scaled(xl, fmt)
        return xh @ wh.t() + qxl @ block_scaled(wh, fmt).t() + qxh @ block_scaled(wl, fmt).t() + b
    if form.startswith("fp16x3t"):   # fp16x3 with the lo parts' mantissas cut to b bits (w: weights, x: activations)
        which, b = form[7:-1], int(form[-1])
        xh, wh = _r(x, torch.float16), _r(w, torch.float16)
        wl, xl = _r(w - wh, torch.float16), _r(x - xh, torch.float16)
        if "w" in which:
            wl = mant_cut(wl, b)
        if "x" in which:
            xl = mant_cut(xl, b)
        return xh @ wh.t() + xh @ wl.t() + xl @ wh.t() + b_
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


def cost(form):
    if form.startswith("fp16x3t"):
        return 3
    return 1 + CROSS_COST[form[1:5]] * 2 if form.startswith("h") else COST[form]


def mean_cost(forms):
    macs = {n: o * i for n, o, i in W.LAYER_SPECS}
    return sum(cost(forms[n]) * macs[n] for n in LAYERS) / sum(macs.values())


SCHEMES = {
    "bf16": scheme("bf16"),
    "fp16": scheme("fp16"),
    "fp16w": scheme("fp16w"),
    "fp16x": scheme("fp16x"),
    "bf16x3": scheme("bf16x3"),
    "fp16x3": scheme("fp16x3"),
    "he4m3": scheme("he4m3"),
    "he4m3f": scheme("he4m3f"),
    "he5m2": scheme("he5m2"),
    "he2m3": scheme("he2m3"),
    "he3m2": scheme("he3m2"),
}
for _b in (2, 3, 4, 6):
    for _w in ("w", "x", "wx"):
        SCHEMES[f"fp16x3t{_w}{_b}"] = scheme(f"fp16x3t{_w}{_b}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ckpt", default="synthetic", choices=["synthetic", "lego"])
    ap.add_argument("--schemes", nargs="*", default=list(SCHEMES))
    ap.add_argument("--res", type=int, nargs=3, default=[200, 150, 32])
    ap.add_argument("--per-layer", action="store_true", help="fp16 everywhere but one layer in fp16x3, and vice versa")
    ap.add_argument("--per-layer-form", default=None, help="fp16x3 everywhere but one layer in this form")
    ap.add_argument("--mix", nargs="*", default=[], help="layer=form overrides on an fp16x3 base, one extra scheme")
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
    if args.per_layer_form:
        for n in LAYERS:
            runs[f"fp16x3 but {n} {args.per_layer_form}"] = scheme("fp16x3", **{n.replace('.', '__'): args.per_layer_form})
    if args.mix:
        runs["mix " + " ".join(args.mix)] = scheme("fp16x3", **dict(m.replace(".", "__").split("=") for m in args.mix))
    for name, forms in runs.items():
        rgb, dep = render(sd, pose, w, h, spp, forms)
        er = float((rgb - ref_rgb).abs().max())
        ed = float((dep - ref_dep).abs().max())
        print(f"{name:40s} cost {mean_cost(forms):.3f}  rgb max {er:.3e} mean {float((rgb - ref_rgb).abs().mean()):.2e}"
              f"  depth max {ed:.3e}", flush=True)


if __name__ == "__main__":
    main()
