"""Diagnostic (GPU box): how often do the bf16 / fp8 kernels' outputs equal the
MFMA-order restatements bit for bit, with the k-step dot rounded once (fl32(acc +
dot)) or twice (fl32(acc + fl32(dot)))?  Prints one JSON line per precision/mode."""
import json
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "nerf-dbr_amd")]

from nerf_amd import runtime as rt  # noqa: E402
from nerf_amd import weights as W  # noqa: E402
from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402


def enc(prec, x, nf):
    xd = torch.as_tensor(np.ascontiguousarray(x, np.float32)).cuda()
    out = torch.empty(xd.shape[0], 3 + 6 * nf, device="cuda")
    rt.positional_encoding(rt.PRECISIONS[prec], xd, nf, out)
    return out.cpu().numpy().T.astype(np.float64)


def main():
    g = np.load(os.path.join(REPO, "tests", "golden", "mlp.npz"))
    pos, dirs = g["pos"], g["dirs"]
    ckpt = W.write_synthetic_checkpoint(os.path.join(tempfile.mkdtemp(), "c.pth"), seed=0)
    _, f = W.synthetic_models(0)
    for prec in ("bf16", "fp8"):
        r = MI355XRenderer(prec)
        r.setup(ckpt)
        s, c = r.query_nerf_networks(torch.from_numpy(pos), torch.from_numpy(dirs))
        s, c = s.cpu().numpy()[:, 0], c.cpu().numpy()
        pe, dpe = enc(prec, pos, 10), enc(prec, dirs, 4)
        for mode in (["group8"] if prec == "bf16" else ["window", "exact"]):
            O.MFMA_FP8_MODEL = mode
            fn = O.bf16_mlp_restated if prec == "bf16" else O.fp8_mlp_restated
            sr, cr = fn(f, pe, dpe)
            cr = cr.T
            es = np.abs(s - sr)
            ec = np.abs(c - cr).max(1)
            print(json.dumps({"precision": prec, "model": mode, "sigma_bit_exact": float(np.mean(es == 0)),
                              "rgb_within_2e-7": float(np.mean(ec <= 2e-7)),
                              "sigma_rel_le_1e-6": float(np.mean(es / (1 + np.abs(sr)) <= 1e-6)),
                              "sigma_rel_max": float((es / (1 + np.abs(sr))).max()), "rgb_max": float(ec.max()),
                              "frac_le": {str(t): [float(np.mean(es / (1 + np.abs(sr)) <= t)), float(np.mean(ec <= t))]
                                          for t in (1e-5, 1e-4, 1e-3)}}),
                  flush=True)


if __name__ == "__main__":
    main()
