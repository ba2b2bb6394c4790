"""How far two fp32 CPU implementations of BASELINE config 3's chain are from its float64 result
(tests/golden/render_lego_800x600_c3_fp64.npz): the reference's own pieces (the fp32 fixture
render_lego_800x600_c3_full.npz, make_golden.py --lego-c3) and the oracle's restatement
(oracle.render_image_hierarchical: the same arithmetic, other GEMM shapes, so other summation
orders).  The spread between the two is what "as close to the truth as the reference" can mean
for an fp32 implementation at all; tests/test_gpu_lego_c3.py (iv) holds the GPU to it.

    python tools/c3_truth_spread.py [out.json] [view index ...]     (CPU, 10-20 min a frame)

Run in the build container, the oracle's oneDNN GEMMs reproduce the reference chain bit for bit
(the same host library and CPU); run on a GPU box's host (another CPU, other GEMM kernels) it is
a second fp32 implementation (profiles/round6/c3_truth/).
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


def main(out_path, views=None):
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    g, t = np.load(os.path.join(G, "render_lego_800x600_c3_full.npz")), np.load(os.path.join(G, "render_lego_800x600_c3_fp64.npz"))
    coarse, fine = (O.Net(sd) for sd in W.lego_models())
    out = {"truth": "tests/golden/render_lego_800x600_c3_fp64.npz", "views": [], "threads": torch.get_num_threads(),
           "cpu": next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), "?"),
           "torch": torch.__version__}
    for k in (views if views else range(len(g["pose_ids"]))):
        t0 = time.time()
        parts = []
        for r0 in range(0, 600, 40):     # row bands, so a long run prints progress
            parts.append(O.render_image_hierarchical(coarse, fine, torch.from_numpy(g["poses"][k]), (800, 600), 64,
                                                     128, chunk=4096, rows=(r0, r0 + 40)))
            print(f"view {k}: rows {r0 + 40} of 600, {time.time() - t0:.0f} s", flush=True)
        rgb, dep = torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])
        v = {"pose_id": int(g["pose_ids"][k]), "oracle_seconds": time.time() - t0,
             "reference_fp32_chain": stats(g[f"rgb_{k}"], g[f"depth_{k}"], t[f"rgb_{k}"], t[f"depth_{k}"]),
             "oracle_fp32_chain": stats(rgb.numpy(), dep.numpy(), t[f"rgb_{k}"], t[f"depth_{k}"])}
        print(json.dumps(v), flush=True)
        out["views"].append(v)
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "round6", "c3_truth", "cpu_spread.json"),
         [int(v) for v in sys.argv[2:]])
