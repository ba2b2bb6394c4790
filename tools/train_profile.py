"""Training-step workload for rocprofv3 (GPU box): main.py's configuration
(2048 rays, 64 + 128 samples), `steps` steps after 2 warm-up steps.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python tools/train_profile.py [steps]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nerf-dbr_amd")]

from nerf_amd import weights as W  # noqa: E402
from nerf_amd.trainer import MI355XTrainer  # noqa: E402


def main(steps=5, precision="fp32"):
    cfg = {"lr": 3e-4, "weight_decay": 1e-6, "gradient_clipping": 1.0, "n_rays": 2048, "precision": precision}
    sd_c, sd_f = W.synthetic_models(0)
    tr = MI355XTrainer(cfg, sd_c, sd_f)
    # profiling on: the two nets' passes run one after the other on one stream, so each
    # kernel's trace duration is its own (unprofiled steps overlap the coarse net's pass
    # with the fine net's on a second stream)
    tr.set_profiling(True)
    rng = np.random.RandomState(3)
    image = torch.from_numpy(rng.rand(400, 400, 3).astype(np.float32)).cuda()
    pose = torch.eye(4)
    pose[2, 3] = 4.0
    batch = {"image": image, "pose": pose, "focal": 555.6}
    for _ in range(2 + steps):
        tr.train_step(batch, sync=False)
    torch.cuda.synchronize()
    print("loss", tr.train_step(batch))


if __name__ == "__main__":
    main(*[int(a) if a.isdigit() else a for a in sys.argv[1:]])   # [steps] [fp32|bf16x3]
