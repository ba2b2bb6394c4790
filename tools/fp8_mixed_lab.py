"""CPU emulation of mixed fp8 / bf16 layer schemes for config 5 (round 5).

    python tools/fp8_mixed_lab.py [--schemes NAME ...] [--res W H S]

Goal: the fp8 path at least as close to the reference's fp32
render as the reference's own int8 compressed renderer (src/benchmark/compressed_renderer.py:
89-211, 233-269; tests/golden/compressed_lego.npz), in max AND mean RGB, on Lego suite view 0
and the off-axis pose (200x150x32), at the least cost in MFMA time.

Each Linear's operands are rounded before an fp64 matmul (the MFMA accumulates exactly per
group and rounds to fp32; fp64 here is within its rounding): per layer a weight format and
an input format for the hidden part and for the encoding part (layers.0 and layers.4 take the
positional encoding, color_layers.0 the direction encoding):
  e4m3  weights: e4m3 of W / 2^e_r, per-row power-of-two scale (nerf_pack_weights_fp8);
        activations: e4m3 of min(max(x, 0), 448) at scale 1; encodings: e4m3 at scale 1;
  bf16  RNE to bfloat16;   f32  unrounded.
Cost = MFMA time relative to an all-fp8 network (a bf16 MFMA k-step takes twice an fp8 one
per FLOP), over the unpadded MACs of each part.
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nerf-dbr_amd")]

from nerf_amd import weights as W  # noqa: E402

LAYERS = ["layers.%d" % i for i in range(8)] + ["density_head", "color_layers.0", "color_layers.1"]
ENC = {"layers.0": "pos", "layers.4": "pos", "color_layers.0": "dir"}


def _q(x, fmt):
    return x.to(fmt).to(torch.float64)


def wq(w, fmt):
    w = w.to(torch.float32)
    if fmt == "f32":
        return w.double()
    if fmt == "bf16":
        return _q(w, torch.bfloat16)
    e = torch.ceil(torch.log2(torch.clamp(w.abs().amax(1, keepdim=True) / 448.0, min=1e-30)))
    return _q(w / torch.exp2(e), torch.float8_e4m3fn) * torch.exp2(e).double()


def aq(x, fmt, enc=False):
    x = x.to(torch.float32)
    if fmt == "f32":
        return x.double()
    if fmt == "bf16":
        return _q(x, torch.bfloat16)
    return _q(torch.clamp(x, -448 if enc else 0, 448), torch.float8_e4m3fn)


def pe(x, L):
    out = [x]
    for k in range(L):
        c = torch.tensor(2.0 ** k, dtype=torch.float32) * math.pi
        out += [torch.sin(c * x), torch.cos(c * x)]
    return torch.cat(out, -1)


def linear(sd, name, hid, enc, form):
    """form = (w_fmt, hid_fmt, enc_fmt); hid / enc are fp32 inputs (either may be None)."""
    wf, hf, ef = form
    w = sd[name + ".weight"]
    parts, ws, col = [], [], 0
    if hid is not None:
        parts.append(aq(hid, hf))
        ws.append(wq(w[:, col:col + hid.shape[1]], wf if hf != "bf16" or wf != "e4m3" else "e4m3"))
        col += hid.shape[1]
    if enc is not None:
        parts.append(aq(enc, ef, enc=True))
        # an encoding part on the bf16 MFMA takes its weights in bf16 (one MFMA, one operand type)
        ws.append(wq(w[:, col:col + enc.shape[1]], "bf16" if ef == "bf16" and wf == "e4m3" else wf))
    y = sum(p @ q.t() for p, q in zip(parts, ws)) + sd[name + ".bias"].double()
    return y.to(torch.float32)


def forward(sd, pos, dirs, forms):
    p = pe(pos, W.POS_L)
    de = pe(dirs, W.DIR_L)
    h = torch.relu(linear(sd, "layers.0", None, p, forms["layers.0"]))
    for i in range(1, 8):
        n = f"layers.{i}"
        h = torch.relu(linear(sd, n, h, p if i == W.SKIP_LAYER else None, forms[n]))
    sigma = torch.relu(linear(sd, "density_head", h, None, forms["density_head"]))
    c = torch.relu(linear(sd, "color_layers.0", h, de, forms["color_layers.0"]))
    rgb = torch.sigmoid(linear(sd, "color_layers.1", c, None, forms["color_layers.1"]))
    return sigma, rgb


def render(sd, pose, w, h, spp, forms, chunk=4096):
    from oracle import nerf_oracle as O

    o, d = O.generate_rays(pose, w, h)
    o, d = o.reshape(-1, 3), d.reshape(-1, 3)
    z = O.uniform_z(spp)
    rgbs, deps = [], []
    with torch.no_grad():
        for c in range(0, o.shape[0], chunk):
            oo, dd = o[c:c + chunk], d[c:c + chunk]
            zz = z.expand(oo.shape[0], spp)
            pts = O.sample_points(oo, dd, zz)
            s, col = forward(sd, pts.reshape(-1, 3), dd[:, None].expand_as(pts).reshape(-1, 3), forms)
            r_, d_ = O.composite(s.reshape(-1, spp, 1), col.reshape(-1, spp, 3), zz, dd)
            rgbs.append(r_)
            deps.append(d_)
    return torch.cat(rgbs).reshape(h, w, 3), torch.cat(deps).reshape(h, w)


MACS = {"layers.0": (0, 63 * 256), "layers.4": (256 * 256, 63 * 256), "density_head": (256, 0),
        "color_layers.0": (256 * 128, 27 * 128), "color_layers.1": (128 * 3, 0)}
for _i in (1, 2, 3, 5, 6, 7):
    MACS[f"layers.{_i}"] = (256 * 256, 0)


def cost(forms):
    """MFMA time relative to all-fp8: a part on the bf16 MFMA counts twice."""
    t = 0.0
    for n in LAYERS:
        wf, hf, ef = forms[n]
        mh, me = MACS[n]
        t += mh * (2 if "bf16" in (wf, hf) or "f32" in (wf, hf) else 1)
        t += me * (2 if "bf16" in (wf, ef) or "f32" in (wf, ef) else 1)
    return t / sum(a + b for a, b in MACS.values())


def scheme(default=("e4m3", "e4m3", "e4m3"), **over):
    f = {n: default for n in LAYERS}
    f["color_layers.1"] = ("bf16", "bf16", "bf16")          # the shipped kernel's colour head
    for k, v in over.items():
        f[k.replace("__", ".")] = v
    return f


B = ("bf16", "bf16", "bf16")
E = ("e4m3", "e4m3", "e4m3")
EB = ("e4m3", "e4m3", "bf16")       # hidden part fp8, encoding part bf16
SCHEMES = {
    "shipped": scheme(),
    "pe_bf16": scheme(layers__0=B, layers__4=EB, color_layers__0=EB),
    "l0_bf16": scheme(layers__0=B),
    "l0_l4pe_bf16": scheme(layers__0=B, layers__4=EB),
    "pe_bf16+c0": scheme(layers__0=B, layers__4=EB, color_layers__0=B),
    "pe_bf16+l1": scheme(layers__0=B, layers__1=B, layers__4=EB, color_layers__0=EB),
    "pe_bf16+l7": scheme(layers__0=B, layers__4=EB, layers__7=B, color_layers__0=EB),
    "pe_bf16+heads": scheme(layers__0=B, layers__4=EB, density_head=B, color_layers__0=B),
    "pe_bf16+c0+l1": scheme(layers__0=B, layers__1=B, layers__4=EB, color_layers__0=B),
    "pe_bf16+c0+l1+l5": scheme(layers__0=B, layers__1=B, layers__4=EB, layers__5=B, color_layers__0=B),
    "pe_bf16+c0+l1+l2": scheme(layers__0=B, layers__1=B, layers__2=B, layers__4=EB, color_layers__0=B),
    "pe_bf16+c0+l1+l2+l5+l6": scheme(layers__0=B, layers__1=B, layers__2=B, layers__4=EB, layers__5=B, layers__6=B,
                                     color_layers__0=B),
    # the round-5 kernel (mlp_fp8.hip): L0, L1, C0 and the heads on the bf16 MFMA (all encodings bf16),
    # L2-L7 fp8 (L4's encoding k-steps bf16)
    "mix": scheme(layers__0=B, layers__1=B, layers__4=EB, density_head=B, color_layers__0=B),
    "mix-l1": scheme(layers__0=B, layers__4=EB, density_head=B, color_layers__0=B),
    "bf16_act_e4m3_w": scheme(("e4m3", "bf16", "bf16")),
    "all_bf16": scheme(B),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--schemes", nargs="*", default=list(SCHEMES))
    ap.add_argument("--per-layer", action="store_true", help="pe_bf16 plus each one layer in bf16")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    _, fine = W.lego_models()
    sd = {k: torch.from_numpy(v) for k, v in fine.items()}
    gold = np.load(os.path.join(REPO, "tests", "golden", "render_lego_200x150_s32.npz"))
    comp = np.load(os.path.join(REPO, "tests", "golden", "compressed_lego.npz"))
    views = [(0, 0), (2, 1)]          # (index in render_lego_200x150_s32, index in compressed_lego)
    line = "int8 reference (compressed_lego.npz):"
    for kg, kc in views:
        e = np.abs(comp[f"rgb_{kc}"] - gold[f"rgb_{kg}"])
        line += f"  view {int(gold['pose_ids'][kg])}: max {e.max():.3e} mean {e.mean():.3e}"
    print(line, flush=True)
    runs = {k: SCHEMES[k] for k in args.schemes}
    if args.per_layer:
        for n in LAYERS:
            base = dict(SCHEMES["pe_bf16"])
            base[n] = B
            runs[f"pe_bf16 + {n} bf16"] = base
    for name, forms in runs.items():
        line = f"{name:28s} cost {cost(forms):.3f}"
        for kg, kc in views:
            rgb, dep = render(sd, torch.from_numpy(gold["poses"][kg]), 200, 150, 32, forms)
            e = np.abs(rgb.numpy() - gold[f"rgb_{kg}"])
            ed = np.abs(dep.numpy() - gold[f"depth_{kg}"])
            line += f"  view {int(gold['pose_ids'][kg])}: max {e.max():.3e} mean {e.mean():.3e} dflip {(ed > 1e-2).sum()}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
