"""CPU emulation of the fp8 path's activation formats (round 3's contract choice).

    python tools/fp8_format_lab.py > profiles/round3/fp8_static/format_lab.txt

Every Linear of NeRFModel with e4m3 weights (per-row power-of-two scale, as
nerf_pack_weights_fp8) and its input activations in one of:
  blk    e4m3, one power-of-two scale per sample and 64-feature block mapping the
         block's maximum into [128, 256) (rounds 1-2's kernel);
  cal    e4m3, one static scale per layer from a calibration sweep (8192 points
         uniform in [-4, 4]^3, random unit directions), maximum into [128, 256),
         saturated;
  one    e4m3 at scale 1, saturated at 448 (round 3's kernel: v_med3_f32 + convert);
  e5m2   bf8 at scale 1 (no scale, no clamp: e5m2 has infinities).
Encodings e4m3 at scale 1, bias and accumulation fp32, colour head bf16, as in
mlp_fp8.hip.  Rendered with the reference's compositing (uniform samples) and
compared with the fp32 forward; the reference's int8 compressed renderer
(oracle.compressed_render_image) is the C5 error bar.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nerf-dbr_amd"), os.path.join(REPO, "tools")]

import precision_lab as P  # noqa: E402
from nerf_amd import weights as W  # noqa: E402


def _q(x, fmt):
    return x.to(fmt).to(torch.float32)


def _wq(w):
    e = torch.ceil(torch.log2(torch.clamp(w.abs().amax(1, keepdim=True) / 448.0, min=1e-30)))
    return _q(w / torch.exp2(e), torch.float8_e4m3fn) * torch.exp2(e)


class Fp8Net:
    def __init__(self, mode, cal=None):
        self.mode, self.cal, self.seen = mode, cal, {}

    def act(self, x, layer):
        if self.mode == "record":
            self.seen[layer] = max(self.seen.get(layer, 0.0), float(x.max()))
            return x
        if self.mode == "blk":
            n, k = x.shape
            xb = x.reshape(n, k // 64, 64)
            s = torch.exp2(torch.frexp(xb.amax(2, keepdim=True))[1].float() - 8)
            return (_q(xb / s, torch.float8_e4m3fn) * s).reshape(n, k)
        if self.mode == "e5m2":
            return _q(x, torch.float8_e5m2)
        s = 2.0 ** (int(np.frexp(np.float32(self.cal[layer]))[1]) - 8) if self.mode == "cal" else 1.0
        return _q(torch.clamp(x, 0, 448 * s) / s, torch.float8_e4m3fn) * s

    def __call__(self, sd, pos, dirs, forms=None):
        pe = _q(torch.clamp(P.pe(pos, W.POS_L), -448, 448), torch.float8_e4m3fn)
        de = _q(P.pe(dirs, W.DIR_L), torch.float8_e4m3fn)
        h = None
        for i in range(8):
            n = f"layers.{i}"
            inp = pe if i == 0 else (torch.cat([self.act(h, i), pe], -1) if i == W.SKIP_LAYER else self.act(h, i))
            h = torch.relu(inp @ _wq(sd[n + ".weight"]).t() + sd[n + ".bias"])
        h7 = self.act(h, 8)
        sigma = torch.relu(h7 @ _wq(sd["density_head.weight"]).t() + sd["density_head.bias"])
        c = torch.relu(torch.cat([h7, de], -1) @ _wq(sd["color_layers.0.weight"]).t() + sd["color_layers.0.bias"])
        rgb = torch.sigmoid(_q(c, torch.bfloat16) @ _q(sd["color_layers.1.weight"], torch.bfloat16).t()
                            + sd["color_layers.1.bias"])
        return sigma, rgb


def main():
    from nerf_amd.benchmark.benchmark_suite import generate_test_poses
    from oracle import nerf_oracle as O

    torch.set_num_threads(os.cpu_count() or 8)
    g = torch.Generator().manual_seed(0)
    f32_forward = P.forward
    for ck in ("synthetic", "lego"):
        _, fine = W.synthetic_models(0) if ck == "synthetic" else W.lego_models()
        sd = {k: torch.from_numpy(v) for k, v in fine.items()}
        rec = Fp8Net("record")
        with torch.no_grad():
            rec(sd, (torch.rand(8192, 3, generator=g) * 2 - 1) * 4.0,
                torch.nn.functional.normalize(torch.randn(8192, 3, generator=g), dim=-1))
        print(f"{ck}: calibration maxima per layer input {dict((k, round(v, 2)) for k, v in rec.seen.items())}")
        for w, h, spp, view in [(64, 48, 32, "eye"), (200, 150, 32, "suite view 0")]:
            if view == "eye":
                pose = torch.eye(4)
                pose[2, 3] = 4.0
            else:
                pose = generate_test_poses(2)[0]
            P.forward = f32_forward
            r32, d32 = P.render(sd, pose, w, h, spp, P.scheme("f32"))
            cells = []
            for mode in ("blk", "cal", "one", "e5m2"):
                P.forward = Fp8Net(mode, rec.seen)
                r8, d8 = P.render(sd, pose, w, h, spp, None)
                cells.append(f"{mode} rgb max {float((r8 - r32).abs().max()):.3e} mean "
                             f"{float((r8 - r32).abs().mean()):.2e} depth max {float((d8 - d32).abs().max()):.2e}")
            line = f"  {w}x{h}x{spp} {view}: " + " | ".join(cells)
            if ck == "synthetic" and view == "eye":
                rc, _ = O.compressed_render_image(O.compressed_weights(fine), pose, (w, h), spp)
                rc = torch.as_tensor(rc).reshape(-1, 3)
                line += (f" | reference int8 compressed rgb max {float((rc - r32).abs().max()):.3e} "
                         f"mean {float((rc - r32).abs().mean()):.2e}")
            print(line, flush=True)
    P.forward = f32_forward


if __name__ == "__main__":
    main()
