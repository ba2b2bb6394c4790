"""Oracle render_image throughput vs torch thread count on this host (the CPU
baseline's scaling): 800x600x128 and 200x150x32 centre rows, view 0.  One JSON line."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "nerf-dbr_amd")]
sys.stdout, out = sys.stderr, sys.stdout
from bench import host_cpu_info  # noqa: E402
from nerf_amd import weights as W  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402

_, f = W.synthetic_models(0)
net = O.Net(f)
pose = torch.eye(4)
pose[2, 3] = 4.0
res = {"host": host_cpu_info(), "rays_per_s": {}}
for th in (1, 2, 4, 8, 16):
    torch.set_num_threads(th)
    O.render_image(net, pose, (800, 600), 128, rows=(300, 301))          # warm
    t0 = time.perf_counter()
    O.render_image(net, pose, (800, 600), 128, rows=(299, 302))
    dt = time.perf_counter() - t0
    res["rays_per_s"][th] = 3 * 800 / dt
print(json.dumps(res), file=out, flush=True)
