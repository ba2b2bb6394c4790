"""Collect (A, B, scales, C, D) of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3) and
v_mfma_f32_32x32x16_bf16 on random data of several distributions (GPU box), so
that the instructions' accumulation arithmetic can be fitted on the host
(tools/probes/mfma_model.py).  Writes gpurun_out/mfma_dataset.npz."""
import ctypes
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libfp8num.so"))
_P, _I = ctypes.c_void_p, ctypes.c_int
lib.probe_mfma8.argtypes = [_P, _P, _P, _P, _P, _P, _I]
lib.probe_mfma16.argtypes = [_P, _P, _P, _P, _I]
rng = np.random.default_rng(7)
T = 64


def e4m3(x):
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(torch.float8_e4m3fn).view(torch.uint8).numpy()


def dist(kind, shape):
    if kind == "wide":
        return np.exp2(rng.uniform(-9, 8, shape)) * rng.choice([-1, 1], shape)
    if kind == "normal":
        return rng.standard_normal(shape) * 8
    if kind == "relu":
        return np.maximum(rng.standard_normal(shape), 0) * 100
    if kind == "narrow":
        return rng.uniform(0.5, 1.0, shape) * rng.choice([-1, 1], shape)
    raise ValueError(kind)


out = {}
for ka, kb in (("wide", "wide"), ("normal", "relu"), ("narrow", "narrow"), ("normal", "normal")):
    A = e4m3(np.clip(dist(ka, (T, 64, 32)), -448, 448))
    B = e4m3(np.clip(dist(kb, (T, 64, 32)), -448, 448))
    sa = rng.integers(118, 136, (T, 64)).astype(np.int32)
    sb = rng.integers(118, 136, (T, 64)).astype(np.int32)
    sa[:, 32:] = sa[:, :32]
    sb[:, 32:] = sb[:, :32]
    C = (rng.standard_normal((T, 64, 16)) * np.exp2(rng.integers(-6, 12, (T, 64, 16)))).astype(np.float32)
    C[: T // 4] = 0
    D = np.zeros((T, 64, 16), np.float32)
    assert lib.probe_mfma8(A.ctypes.data, B.ctypes.data, sa.ctypes.data, sb.ctypes.data, C.ctypes.data,
                           D.ctypes.data, T) == 0
    tag = f"f8_{ka}_{kb}"
    out.update({f"{tag}_A": A, f"{tag}_B": B, f"{tag}_sa": sa, f"{tag}_sb": sb, f"{tag}_C": C, f"{tag}_D": D})

for ka, kb in (("wide", "wide"), ("normal", "relu"), ("narrow", "narrow"), ("normal", "normal")):
    a = torch.from_numpy(dist(ka, (T, 64, 8)).astype(np.float32)).to(torch.bfloat16)
    b = torch.from_numpy(dist(kb, (T, 64, 8)).astype(np.float32)).to(torch.bfloat16)
    A = np.ascontiguousarray(a.view(torch.int16).numpy())
    B = np.ascontiguousarray(b.view(torch.int16).numpy())
    C = (rng.standard_normal((T, 64, 16)) * np.exp2(rng.integers(-6, 12, (T, 64, 16)))).astype(np.float32)
    C[: T // 4] = 0
    D = np.zeros((T, 64, 16), np.float32)
    assert lib.probe_mfma16(A.ctypes.data, B.ctypes.data, C.ctypes.data, D.ctypes.data, T) == 0
    tag = f"b16_{ka}_{kb}"
    out.update({f"{tag}_A": A, f"{tag}_B": B, f"{tag}_C": C, f"{tag}_D": D})

os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/mfma_dataset.npz", **out)
print("saved", len(out), "arrays")
