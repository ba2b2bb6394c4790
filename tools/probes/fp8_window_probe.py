"""fp8 MFMA: big + tiny (no cancellation), D vs fl32(exact), for placements (GPU box)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import mfma_accum_probe as M  # noqa: E402


def test(kb, kt_list, n_tiny, big=(16.0, 16.0), c=0.0):
    """rows r: tiny exponent -(r) (2^-r at each of n_tiny k's in kt_list); col c: unused (same)."""
    Am = np.zeros((32, 64))
    Bm = np.zeros((64, 32))
    Am[:, kb] = big[0]
    Bm[kb, :] = big[1]
    for kt in kt_list[:n_tiny]:
        Am[:, kt] = np.exp2(-(np.arange(32) % 10))          # 2^0 .. 2^-9
        Bm[kt, :] = np.exp2(-(np.arange(32) // 3 % 10))     # col-dependent 2^0 .. 2^-9
    Cm = np.full((32, 32), c)
    D = M.run8(Am, Bm, Cm)
    ex = Am @ Bm + Cm
    once = ex.astype(np.float32)
    out = {}
    bigp = big[0] * big[1] + c
    for r in range(32):
        for cc in range(32):
            gap = int(round(np.log2(bigp) - np.log2(Am[r, kt_list[0]] * Bm[kt_list[0], cc])))
            key = str(gap)
            ok = D[r, cc] == once[r, cc]
            lost = D[r, cc] == np.float32(bigp)
            v = "exact" if ok else ("lost" if lost else f"other({(D[r, cc] - bigp) / (ex[r, cc] - bigp):.3f})")
            out.setdefault(key, set()).add(v)
    return {k: sorted(v) for k, v in sorted(out.items(), key=lambda kv: int(kv[0]))}


cases = {
    "big k1, 1 tiny k0": test(1, [0], 1),
    "big k0, 1 tiny k1": test(0, [1], 1),
    "big k0, 1 tiny k40": test(0, [40], 1),
    "big k0, 3 tiny k1,2,3": test(0, [1, 2, 3], 3),
    "big k0, 3 tiny k1,33,50": test(0, [1, 33, 50], 3),
    "C=256, 1 tiny k5": test(0, [5], 1, big=(0.0, 0.0), c=256.0),
}
for k, v in cases.items():
    print(json.dumps({"case": k, "by_gap": v}), flush=True)
