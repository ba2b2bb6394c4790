"""How far two fp32 CPU implementations of BASELINE config 3's chain are from its float64 result
(tests/golden/render_lego_800x600_c3_fp64.npz): the reference's own pieces (the fp32 fixture
render_lego_800x600_c3_full.npz, make_golden.py --lego-c3) and the oracle's restatement
(oracle.render_image_hierarchical: the same arithmetic, other GEMM shapes, so other summation
orders).  The spread between the two is what "as close to the truth as the reference" can mean
for an fp32 implementation at all; tests/test_gpu_lego_c3.py (iv) holds the GPU to it.

    python tools/c3_truth_spread.py [out.json]        (CPU, about 6 min a frame on 8 cores)
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nerf-dbr_amd")]

from nerf_amd import weights as W  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402

G = os.path.join(REPO, "tests", "golden")


def stats(rgb, dep, t_rgb, t_dep):
    e_rgb = np.abs(np.asarray(rgb, np.float64).reshape(-1, 3) - t_rgb.reshape(-1, 3)).max(-1)
    e_dep = np.abs(np.asarray(dep, np.float64).reshape(-1) - t_dep.reshape(-1))
    return {"rgb_max": float(e_rgb.max()), "rgb_mean": float(e_rgb.mean()), "depth_max": float(e_dep.max()),
            "depth_mean": float(e_dep.mean()), "over_1e-4": int(((e_rgb >= 1e-4) | (e_dep >= 1e-4)).sum())}


def main(out_path):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g, t = np.load(os.path.join(G, "render_lego_800x600_c3_full.npz")), np.load(os.path.join(G, "render_lego_800x600_c3_fp64.npz"))
    coarse, fine = (O.Net(sd) for sd in W.lego_models())
    out = {"truth": "tests/golden/render_lego_800x600_c3_fp64.npz", "views": []}
    for k in range(len(g["pose_ids"])):
        t0 = time.time()
        rgb, dep = O.render_image_hierarchical(coarse, fine, torch.from_numpy(g["poses"][k]), (800, 600), 64, 128,
                                               chunk=4096)
        v = {"pose_id": int(g["pose_ids"][k]), "oracle_seconds": time.time() - t0,
             "reference_fp32_chain": stats(g[f"rgb_{k}"], g[f"depth_{k}"], t[f"rgb_{k}"], t[f"depth_{k}"]),
             "oracle_fp32_chain": stats(rgb.numpy(), dep.numpy(), t[f"rgb_{k}"], t[f"depth_{k}"])}
        print(json.dumps(v), flush=True)
        out["views"].append(v)
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "round6", "c3_truth", "cpu_spread.json"))
