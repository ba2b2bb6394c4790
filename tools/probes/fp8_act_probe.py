"""A candidate fp8 activation conversion (round 3 lab, measured and not kept: DESIGN.md
section 7) on the GPU box, bit for bit against its contract e4m3(min(max(x, 0), 256)),
NaN and -0 -> +0: v_pk_mul_f32 by 2^-8 with the clamp bit, then
v_cvt_scalef32_pk_fp8_f32 at scale 2^-8.

    python tools/probes/fp8_act_probe.py   (the .so is built in-tree beforehand:
    hipcc -shared -fPIC --offload-arch=gfx950 -O2 tools/probes/fp8_act_probe.hip
          -o nerf-dbr_amd/csrc/build/probes/libfp8actprobe.so)
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "..", "..", "nerf-dbr_amd", "csrc", "build", "probes", "libfp8actprobe.so")
SPECIAL = [0.0, -0.0, 1.0, 2.0 ** -10, 3 * 2.0 ** -10, 2.0 ** -9, 2.0 ** -6, 1.0625, 239.9, 248.0, 255.9, 256.0,
           256.1, 448.0, 464.0, 480.0, 1e4, 3.0e38, float("inf"), float("-inf"), float("nan"), -1.0, -256.0,
           1e-40, -1e-40, 2.0 ** -126, 2.0 ** -130]


def restated(x):
    """e4m3 of min(max(x, 0), 256), NaN and -0 -> +0 (RNE)."""
    x = np.nan_to_num(np.asarray(x, np.float64), nan=0.0)
    return np.clip(x, 0.0, 256.0) + 0.0


def main():
    lib = ctypes.CDLL(LIB)
    lib.fp8_act_probe.restype = ctypes.c_int
    lib.fp8_act_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(1 << 18) * s for s in (1e-3, 0.05, 1.0, 30.0, 150.0, 1e3)]
                       + [np.ldexp(rng.uniform(1, 2, 1 << 16), rng.integers(-140, 12, 1 << 16))
                          * rng.choice([-1, 1], 1 << 16)])
    x = np.concatenate([np.array(SPECIAL), x]).astype(np.float32)
    x = np.concatenate([x, np.zeros((-len(x)) % 4, np.float32)])
    out = np.zeros(len(x) // 4, np.uint32)
    assert lib.fp8_act_probe(x.ctypes.data, len(x) // 4, out.ctypes.data) == 0
    hw = out.view(np.uint8)
    ref = torch.from_numpy(restated(x).astype(np.float32)).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    bad = np.nonzero(hw != ref)[0]
    res = {"values": int(len(x)), "mismatches": int(len(bad)),
           "first_mismatches": [{"x": float(x[i]), "hw": f"0x{hw[i]:02x}", "restated": f"0x{ref[i]:02x}"}
                                for i in bad[:20]],
           "special": [{"x": float(v), "hw": f"0x{hw[i]:02x}", "restated": f"0x{ref[i]:02x}"}
                       for i, v in enumerate(SPECIAL)]}
    print(json.dumps(res, indent=1))
    sys.exit(0 if len(bad) == 0 else 1)


if __name__ == "__main__":
    main()
