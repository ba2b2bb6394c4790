"""Debug: which term of a random e4m3 MFMA dot differs from exact arithmetic (GPU box)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mfma_accum_probe import run8  # noqa: E402

rng = np.random.default_rng(1)
dec = lambda c: torch.from_numpy(np.ascontiguousarray(c, np.uint8)).view(torch.float8_e4m3fn).float().numpy().astype(np.float64)  # noqa: E731
for name, codes in (("all", [c for c in range(256) if (c & 0x7F) != 0x7F]),
                    ("exp<15", [c for c in range(256) if ((c >> 3) & 15) < 15]),
                    ("exp 1..14", [c for c in range(256) if 1 <= ((c >> 3) & 15) < 15]),
                    ("small ints", None)):
    if codes is None:
        Am = rng.integers(-4, 5, (32, 64)).astype(np.float64)
        Bm = rng.integers(-4, 5, (64, 32)).astype(np.float64)
    else:
        codes = np.array(codes, np.uint8)
        Am = dec(rng.choice(codes, (32, 64)))
        Bm = dec(rng.choice(codes, (64, 32)))
    Cm = np.zeros((32, 32))
    D = run8(Am, Bm, Cm)
    ex = Am @ Bm
    once = ex.astype(np.float32).astype(np.float64)
    bad = D != once
    info = {"codes": name, "frac_exact": float(np.mean(~bad))}
    if bad.any():
        r, c = np.argwhere(bad)[0]
        diff = D[r, c] - ex[r, c]
        prods = Am[r] * Bm[:, c]
        info.update({"D": float(D[r, c]), "exact": float(ex[r, c]), "diff": float(diff),
                     "max_prod": float(np.abs(prods).max()),
                     "k_with_prod_eq_diff": [int(k) for k in np.where(np.isclose(prods, -diff))[0]],
                     "rel_err": float(abs(diff) / max(abs(ex[r, c]), 1e-30))})
    print(json.dumps(info), flush=True)
