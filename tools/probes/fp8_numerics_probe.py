"""Numerics of the fp8 / bf16 MFMA path's instructions against exact host arithmetic
(GPU box; build: hipcc -shared -fPIC --offload-arch=gfx950 -O2
tools/probes/fp8_numerics_probe.hip -o tools/probes/libfp8num.so).  One JSON line
per question; the answers decide how oracle.fp8_mlp_restated / bf16_mlp_restated
state the kernels' arithmetic."""
import ctypes
import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libfp8num.so"))
_P, _I = ctypes.c_void_p, ctypes.c_int
lib.probe_cvt.argtypes = [_P, _P, _P, _P, _I]
lib.probe_mfma8.argtypes = [_P, _P, _P, _P, _P, _P, _I]
lib.probe_mfma16.argtypes = [_P, _P, _P, _P, _I]
rng = np.random.default_rng(0)


def e4m3_codes(x):
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(torch.float8_e4m3fn).view(torch.uint8).numpy()


def e4m3_vals(codes):
    return torch.from_numpy(np.ascontiguousarray(codes, np.uint8)).view(torch.float8_e4m3fn).float().numpy()


def acc_row(i, h):
    return (i & 3) + 8 * (i >> 2) + 4 * h


# 1. conversions
n = 1 << 16
mag = np.exp2(rng.uniform(-14, 9, 2 * n)).astype(np.float32)
x = (mag * rng.choice([-1, 1], 2 * n)).astype(np.float32)
e = rng.integers(-4, 5, n)
s = np.exp2(e).astype(np.float32)
x = np.clip(x, -440 * np.repeat(s, 2), 440 * np.repeat(s, 2)).astype(np.float32)
o1 = np.zeros(n, np.uint32)
o2 = np.zeros(n, np.uint32)
assert lib.probe_cvt(x.ctypes.data, s.ctypes.data, o1.ctypes.data, o2.ctypes.data, n) == 0
got_s = np.stack([o1 & 0xFF, o1 >> 8], 1).reshape(-1).astype(np.uint8)
got_p = np.stack([o2 & 0xFF, o2 >> 8], 1).reshape(-1).astype(np.uint8)
ref_s = e4m3_codes(x / np.repeat(s, 2))
xp = np.clip(x, -448, 448)
ref_p = e4m3_codes(xp)
sub = np.abs(x / np.repeat(s, 2)) < 2 ** -6
print(json.dumps({"q": "cvt_scalef32_pk_fp8_f32 == torch e4m3(x/s)", "frac_equal": float(np.mean(got_s == ref_s)),
                  "frac_equal_subnormal": float(np.mean((got_s == ref_s)[sub])),
                  "frac_equal_normal": float(np.mean((got_s == ref_s)[~sub])),
                  "examples": [[float(a), float(b), int(c), int(d)] for a, b, c, d in
                               zip(x[got_s != ref_s][:6], np.repeat(s, 2)[got_s != ref_s][:6],
                                   got_s[got_s != ref_s][:6], ref_s[got_s != ref_s][:6])]}), flush=True)
ok = np.abs(x) <= 448
print(json.dumps({"q": "cvt_pk_fp8_f32 == torch e4m3(x)", "frac_equal": float(np.mean((got_p == ref_p)[ok]))}),
      flush=True)

# 2. fp8 MFMA: trials of random e4m3 A, B (finite codes), scales, random C
T = 256
codes = np.array([c for c in range(256) if (c & 0x7F) != 0x7F], np.uint8)
A = rng.choice(codes, (T, 64, 32)).astype(np.uint8)
B = rng.choice(codes, (T, 64, 32)).astype(np.uint8)
SCALES = os.environ.get("PROBE_SCALES", "random")
sa = rng.integers(120, 134, (T, 64)).astype(np.int32)
sb = rng.integers(120, 134, (T, 64)).astype(np.int32)
if SCALES == "unit":
    sa[:] = 127
    sb[:] = 127
# same scale for lanes r and r+32 (the kernel's use)
sa[:, 32:] = sa[:, :32]
sb[:, 32:] = sb[:, :32]
C = (rng.standard_normal((T, 64, 16)) * np.exp2(rng.integers(-4, 8, (T, 64, 16)))).astype(np.float32)
D = np.zeros((T, 64, 16), np.float32)
assert lib.probe_mfma8(A.ctypes.data, B.ctypes.data, sa.ctypes.data, sb.ctypes.data, C.ctypes.data, D.ctypes.data,
                       T) == 0
Av, Bv = e4m3_vals(A).astype(np.float64), e4m3_vals(B).astype(np.float64)
res = {"exact_once": 0, "total": 0}
dev = []
for t in range(T):
    Am = np.zeros((32, 64))
    Bm = np.zeros((64, 32))
    for l in range(64):
        r, h = l & 31, l >> 5
        Am[r, 32 * h: 32 * h + 32] = Av[t, l]
        Bm[32 * h: 32 * h + 32, r] = Bv[t, l]
    dot = (Am @ Bm) * np.exp2(sa[t, :32, None] - 127.0) * np.exp2(sb[t, None, :32] - 127.0)
    Cm = np.zeros((32, 32))
    Dm = np.zeros((32, 32))
    for l in range(64):
        for i in range(16):
            Cm[acc_row(i, l >> 5), l & 31] = C[t, l, i]
            Dm[acc_row(i, l >> 5), l & 31] = D[t, l, i]
    once = (Cm + dot).astype(np.float32)
    res["exact_once"] += int(np.sum(once == Dm))
    res["total"] += Dm.size
    ulp = np.spacing(np.abs(once).astype(np.float32))
    dev.append(np.abs(Dm - once.astype(np.float64)) / ulp)
dev = np.concatenate([d.ravel() for d in dev])
print(json.dumps({"q": f"mfma_scale 32x32x64 e4m3 ({SCALES} scales): D == fl32(C + exact scaled dot)",
                  "frac": res["exact_once"] / res["total"], "ulp_p99": float(np.percentile(dev, 99)),
                  "ulp_max": float(dev.max())}), flush=True)

# 3. bf16 MFMA, the same question
Ab = (rng.standard_normal((T, 64, 8)) * np.exp2(rng.integers(-6, 6, (T, 64, 8)))).astype(np.float32)
Bb = (rng.standard_normal((T, 64, 8)) * np.exp2(rng.integers(-6, 6, (T, 64, 8)))).astype(np.float32)
ab = torch.from_numpy(Ab).to(torch.bfloat16)
bb = torch.from_numpy(Bb).to(torch.bfloat16)
Av, Bv = ab.double().numpy(), bb.double().numpy()
D = np.zeros((T, 64, 16), np.float32)
ab16 = np.ascontiguousarray(ab.view(torch.int16).numpy())
bb16 = np.ascontiguousarray(bb.view(torch.int16).numpy())
assert lib.probe_mfma16(ab16.ctypes.data, bb16.ctypes.data, C.ctypes.data, D.ctypes.data, T) == 0
cnt = {"once": 0, "halves": 0, "total": 0}
for t in range(T):
    Am = np.zeros((32, 16))
    Bm = np.zeros((16, 32))
    for l in range(64):
        r, h = l & 31, l >> 5
        Am[r, 8 * h: 8 * h + 8] = Av[t, l]
        Bm[8 * h: 8 * h + 8, r] = Bv[t, l]
    Cm = np.zeros((32, 32))
    Dm = np.zeros((32, 32))
    for l in range(64):
        for i in range(16):
            Cm[acc_row(i, l >> 5), l & 31] = C[t, l, i]
            Dm[acc_row(i, l >> 5), l & 31] = D[t, l, i]
    once = (Cm + Am @ Bm).astype(np.float32)
    halves = (Cm + Am[:, :8] @ Bm[:8]).astype(np.float32)
    halves = (halves.astype(np.float64) + Am[:, 8:] @ Bm[8:]).astype(np.float32)
    cnt["once"] += int(np.sum(once == Dm))
    cnt["halves"] += int(np.sum(halves == Dm))
    cnt["total"] += Dm.size
print(json.dumps({"q": "mfma 32x32x16 bf16: D == fl32(C + exact dot) / == fl32(fl32(C + dot k0-7) + dot k8-15)",
                  "frac_once": cnt["once"] / cnt["total"], "frac_halves": cnt["halves"] / cnt["total"]}), flush=True)
