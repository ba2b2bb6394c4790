"""Overflow behaviour of v_cvt_scalef32_pk_fp8_f32 on the GPU box.

    python tools/probes/fp8_cvt_probe.py   (builds nothing: the .so is built in-tree beforehand,
    hipcc -shared -fPIC --offload-arch=gfx950 -O2 tools/probes/fp8_cvt_probe.hip
          -o nerf-dbr_amd/csrc/build/probes/libfp8cvtprobe.so)

Prints, per input value, the e4m3 byte the hardware produced at scale 1 and at
scale 2, beside torch's float8_e4m3fn cast of x / scale.
"""
import ctypes
import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "..", "..", "nerf-dbr_amd", "csrc", "build", "probes", "libfp8cvtprobe.so")

VALUES = [0.0, 1.0, 240.0, 448.0, 460.0, 464.0, 480.0, 512.0, 1000.0, 1e6, 3.0e38, float("inf"),
          -448.0, -464.0, -1000.0, float("-inf"), float("nan"), 2.0 ** -10, -0.0, 5.0]


def main():
    lib = ctypes.CDLL(LIB)
    lib.fp8_cvt_probe.restype = ctypes.c_int
    lib.fp8_cvt_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_void_p]
    x = np.array(VALUES + ([0.0] if len(VALUES) % 2 else []), np.float32)
    res = {}
    for scale in (1.0, 2.0):
        out = np.zeros(len(x) // 2, np.uint32)
        assert lib.fp8_cvt_probe(x.ctypes.data, len(x) // 2, scale, out.ctypes.data) == 0
        hw = [(int(o) >> (8 * j)) & 0xFF for o in out for j in (0, 1)]
        ref = torch.from_numpy(x / scale).to(torch.float8_e4m3fn).view(torch.uint8).numpy().tolist()
        res[str(scale)] = [{"x": float(v), "hw": f"0x{h:02x}", "torch": f"0x{r:02x}"} for v, h, r in zip(x, hw, ref)]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
