"""Pin the operand maps of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3) on the GPU box.

    make -C nerf-dbr_amd/csrc probes && python tools/probes/fp8_mfma_probe.py

Hypotheses checked with exact small-integer data (every product and sum exact):
  H1  A lane (row r=l&31, half h=l>>5) byte j and B lane (col c=l&31, half h) byte j
      carry the same k (so any k order folded into packing works if A and B agree);
  H2  D uses the bf16 32x32 accumulator map: reg i -> row (i&3)+8(i>>2)+4h, col l&31;
  H3  scale operand byte = E8M0 exponent: 127 -> x1, 128 -> x2, per lane's row/col block.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "..", "..", "nerf-dbr_amd", "csrc", "build", "probes", "libfp8probe.so")


def e4m3(x):
    return torch.from_numpy(np.asarray(x, np.float32)).to(torch.float8_e4m3fn).view(torch.uint8).numpy()


def acc_row(i, h):
    return (i & 3) + 8 * (i >> 2) + 4 * h


def run(lib, A, B, sa, sb):
    a, b = e4m3(A).reshape(64, 32), e4m3(B).reshape(64, 32)
    d = np.zeros((64, 16), np.float32)
    sa = np.ascontiguousarray(sa, np.int32)
    sb = np.ascontiguousarray(sb, np.int32)
    assert lib.fp8_probe(a.ctypes.data, b.ctypes.data, sa.ctypes.data, sb.ctypes.data, d.ctypes.data) == 0
    D = np.zeros((32, 32))
    for l in range(64):
        for i in range(16):
            D[acc_row(i, l >> 5), l & 31] = d[l, i]
    return D


def main():
    lib = ctypes.CDLL(LIB)
    lib.fp8_probe.argtypes = [ctypes.c_void_p] * 5
    rng = np.random.default_rng(0)
    A = rng.integers(-4, 5, (64, 32)).astype(np.float32)     # [lane][byte]
    B = rng.integers(-4, 5, (64, 32)).astype(np.float32)
    ones = np.full(64, 127)
    D = run(lib, A, B, ones, ones)
    # H1: pair (h, j) with (h, j)
    ref = np.zeros((32, 32))
    for r in range(32):
        for c in range(32):
            ref[r, c] = sum(A[r + 32 * h] @ B[c + 32 * h] for h in range(2))
    out = {"H1_H2_symmetric_pairing": bool(np.array_equal(D, ref))}
    # H3: scale exponents.  Row-dependent A scale: lanes of row 5 get 128 (x2).
    sa = ones.copy()
    sa[5] = 128
    sa[37] = 128
    D2 = run(lib, A, B, sa, ones)
    ref2 = ref.copy()
    ref2[5] *= 2
    out["H3_row_scale_x2"] = bool(np.array_equal(D2, ref2))
    sa = ones.copy()
    sa[37] = 128                                        # only half h=1 of row 5
    D3 = run(lib, A, B, sa, ones)
    ref3 = ref.copy()
    ref3[5] = [A[5] @ B[c] + 2 * (A[37] @ B[c + 32]) for c in range(32)]
    out["H3_scale_per_row_and_k_half"] = bool(np.array_equal(D3, ref3))
    sb = ones.copy()
    sb[7] = 126                                         # column 7, half 0: x0.5
    D4 = run(lib, A, B, ones, sb)
    ref4 = ref.copy()
    ref4[:, 7] = [0.5 * (A[r] @ B[7]) + A[r + 32] @ B[39] for r in range(32)]
    out["H3_col_scale_per_k_half"] = bool(np.array_equal(D4, ref4))
    sb = ones.copy()
    sb[7] = sb[39] = 128                                # column 7, both lane halves: x2
    D5 = run(lib, A, B, ones, sb)
    ref5 = ref.copy()
    ref5[:, 7] *= 2
    out["H3_col_scale_x2"] = bool(np.array_equal(D5, ref5))
    # scale-byte granularity: which lane's scale applies to which (row, k) part
    gran = {}
    for lane in (5, 37):
        for byte in range(4):
            sa = ones.copy()
            sa[lane] = 127 | (1 << (8 * byte)) if byte else 128
            gran[f"lane{lane}_byte{byte}_changes"] = bool(not np.array_equal(run(lib, A, B, sa, ones), ref))
    out["scale_bytes"] = gran
    # H4: conversions.  v_cvt_scalef32_pk_fp8_f32(x, s): fp8(x * s) or fp8(x / s)?
    lib.fp8_cvt_probe.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int]
    xs = np.array([1.0, 3.0, 0.75, -2.0, 448.0, 500.0, 1e6, -1e6, 0.001, 0.0], np.float32)
    sc = np.array([2.0, 0.5, 1.0, 4.0, 8.0], np.float32)
    o = np.zeros(10, np.uint32)
    assert lib.fp8_cvt_probe(xs.ctypes.data, sc.ctypes.data, o.ctypes.data, 5) == 0
    dec = lambda v: torch.tensor([v & 0xFF, v >> 8], dtype=torch.uint8).view(torch.float8_e4m3fn).float().tolist()
    out["cvt_scalef32"] = {f"({xs[2*i]},{xs[2*i+1]})/s={sc[i]}": dec(int(o[2 * i])) for i in range(5)}
    out["cvt_pk_plain"] = {f"({xs[2*i]},{xs[2*i+1]})": dec(int(o[2 * i + 1])) for i in range(5)}
    print(json.dumps(out, indent=1))
    return 0 if out["H1_H2_symmetric_pairing"] else 1


if __name__ == "__main__":
    sys.exit(main())
