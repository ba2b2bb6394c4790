"""How v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3) and v_mfma_f32_32x32x16_bf16 add
their products: cancellation tests (GPU box; uses tools/probes/libfp8num.so).
D[r, c] = big - big + tiny(r, c) for several placements of the three terms in k;
exact accumulation gives tiny, an alignment window of p bits below the largest
term loses tiny once it is 2^-p below it."""
import ctypes
import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libfp8num.so"))
_P, _I = ctypes.c_void_p, ctypes.c_int
lib.probe_mfma8.argtypes = [_P, _P, _P, _P, _P, _P, _I]
lib.probe_mfma16.argtypes = [_P, _P, _P, _P, _I]


def acc_row(i, h):
    return (i & 3) + 8 * (i >> 2) + 4 * h


def run8(Am, Bm, Cm):
    """Am [32, 64], Bm [64, 32] float (e4m3-representable), Cm [32, 32] -> D [32, 32]."""
    enc = lambda v: torch.from_numpy(np.ascontiguousarray(v, np.float32)).to(torch.float8_e4m3fn).view(torch.uint8).numpy()  # noqa: E731
    A = np.zeros((1, 64, 32), np.uint8)
    B = np.zeros((1, 64, 32), np.uint8)
    C = np.zeros((1, 64, 16), np.float32)
    for l in range(64):
        r, h = l & 31, l >> 5
        A[0, l] = enc(Am[r, 32 * h: 32 * h + 32])
        B[0, l] = enc(Bm[32 * h: 32 * h + 32, r])
        for i in range(16):
            C[0, l, i] = Cm[acc_row(i, h), r]
    sa = np.full((1, 64), 127, np.int32)
    sb = np.full((1, 64), 127, np.int32)
    D = np.zeros((1, 64, 16), np.float32)
    assert lib.probe_mfma8(A.ctypes.data, B.ctypes.data, sa.ctypes.data, sb.ctypes.data, C.ctypes.data, D.ctypes.data, 1) == 0
    out = np.zeros((32, 32))
    for l in range(64):
        for i in range(16):
            out[acc_row(i, l >> 5), l & 31] = D[0, l, i]
    return out


def run16(Am, Bm, Cm):
    A = np.zeros((1, 64, 8), np.float32)
    B = np.zeros((1, 64, 8), np.float32)
    C = np.zeros((1, 64, 16), np.float32)
    for l in range(64):
        r, h = l & 31, l >> 5
        A[0, l] = Am[r, 8 * h: 8 * h + 8]
        B[0, l] = Bm[8 * h: 8 * h + 8, r]
        for i in range(16):
            C[0, l, i] = Cm[acc_row(i, h), r]
    a16 = np.ascontiguousarray(torch.from_numpy(A).to(torch.bfloat16).view(torch.int16).numpy())
    b16 = np.ascontiguousarray(torch.from_numpy(B).to(torch.bfloat16).view(torch.int16).numpy())
    D = np.zeros((1, 64, 16), np.float32)
    assert lib.probe_mfma16(a16.ctypes.data, b16.ctypes.data, C.ctypes.data, D.ctypes.data, 1) == 0
    out = np.zeros((32, 32))
    for l in range(64):
        for i in range(16):
            out[acc_row(i, l >> 5), l & 31] = D[0, l, i]
    return out


def cancel_test(run, K, big_a, big_b, tiny_exp, kb0, kb1, kt, c_big=False):
    """rows r, cols c: tiny = 2^-(r%S) * 2^-(c%S) * 2^tiny_exp at k=kt; +big at kb0, -big at kb1
    (or C = +big and only -big at kb1)."""
    Am = np.zeros((32, K))
    Bm = np.zeros((K, 32))
    Cm = np.zeros((32, 32))
    S = 10
    ea = -(np.arange(32) % S)
    eb = -(np.arange(32) % S)
    Am[:, kt] = np.exp2(ea + tiny_exp)
    Bm[kt, :] = np.exp2(eb)
    if c_big:
        Cm[:, :] = big_a * big_b
    else:
        Am[:, kb0] = big_a
        Bm[kb0, :] = big_b
    Am[:, kb1] = -big_a
    Bm[kb1, :] = big_b
    D = run(Am, Bm, Cm)
    tiny = np.exp2(ea[:, None] + eb[None, :] + tiny_exp)
    rel = np.log2(big_a * big_b) - np.log2(tiny)          # how far below the big term
    res = {}
    for d in sorted(set(np.round(rel.ravel(), 2))):
        m = np.isclose(rel, d)
        res[float(d)] = "exact" if np.all(D[m] == tiny[m]) else ("zero" if np.all(D[m] == 0) else
                                                                 f"other:{float(D[m][0] / tiny[m][0]):.4g}")
    return res


def main():
    out = {}
    out["fp8 C=big, -big k7, tiny k3"] = cancel_test(run8, 64, 448.0, 448.0, 0, 0, 7, 3, c_big=True)
    for e in (2, 5, 8):
        out[f"bf16 big(2^{2*e}) k0,k1 tiny k2"] = cancel_test(run16, 16, 2.0 ** e, 2.0 ** e, 0, 0, 1, 2)
        out[f"bf16 tiny k0 big(2^{2*e}) k7,k8"] = cancel_test(run16, 16, 2.0 ** e, 2.0 ** e, 0, 7, 8, 0)
        out[f"bf16 C=big(2^{2*e}), -big k9, tiny k3"] = cancel_test(run16, 16, 2.0 ** e, 2.0 ** e, 0, 0, 9, 3, c_big=True)
    for k, v in out.items():
        print(json.dumps({"case": k, "result_by_log2_gap": v}), flush=True)


if __name__ == "__main__":
    main()
