"""The original-NeRF Lego network (the distillation teacher), restated in PyTorch.

``data/lego_example_weights/model_200000.npy`` (coarse) and
``model_fine_200000.npy`` (fine) in the reference hold the 24 arrays of the
original NeRF implementation's Keras model (``args.txt``: netdepth 8, netwidth
256, multires 10, multires_views 4, use_viewdirs, skip after layer 4, white
background).  Dense kernels are stored ``[in, out]``:

====  ==============================  =====================================
idx   shape                           role
====  ==============================  =====================================
0-15  (63|256|319, 256), (256,)       8 trunk layers, ReLU; layer 5's input is
                                      ``cat([pe(x), h])`` (319 = 63 + 256)
16    (256, 256), (256,)              feature ("bottleneck"), no activation
18    (283, 128), (128,)              views layer on ``cat([feature, pe(d)])``, ReLU
20    (128, 3), (3,)                  rgb (sigmoid in raw2outputs)
22    (256, 1), (1,)                  alpha / sigma (ReLU in raw2outputs)
====  ==============================  =====================================

Unlike the reference's ``NeRFModel`` (``src/models/nerf.py:16-131``) the
positional encoding has no pi (``sin(2^k x)``), the skip feeds layer 5 rather
than layer 4 and puts the encoding first, view directions are normalised, and
the colour branch has a linear feature layer.  That is why the teacher cannot
be re-laid out into ``NeRFModel`` exactly and is distilled instead
(``tools/lego/distill.py``).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn.functional as F

from .npy_static import read_object_npy

LEGO_DIR = "/root/reference/data/lego_example_weights"
# Blender lego, full resolution 800x800: focal = 0.5 * 800 / tan(0.5 * camera_angle_x)
CAMERA_ANGLE_X = 0.6911112070083618


def embed(x: torch.Tensor, L: int) -> torch.Tensor:
    """[x, sin(2^0 x), cos(2^0 x), ..., sin(2^(L-1) x), cos(2^(L-1) x)] (no pi)."""
    out = [x]
    for k in range(L):
        f = float(2.0 ** k)
        out.append(torch.sin(x * f))
        out.append(torch.cos(x * f))
    return torch.cat(out, dim=-1)


def load_arrays(which: str, lego_dir: str = LEGO_DIR):
    """The 24 arrays of ``model_200000.npy`` ("coarse") or ``model_fine_200000.npy`` ("fine"),
    read by the static parser.  A ``.npz`` copy (``tools/lego/_teacher_<which>.npz``, written by
    ``export_npz``) is used when the reference checkout is absent (the GPU box)."""
    cache = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"_teacher_{which}.npz")
    if not os.path.isdir(lego_dir) and os.path.exists(cache):
        z = np.load(cache)
        return [z[f"a{i}"] for i in range(24)]
    name = {"coarse": "model_200000.npy", "fine": "model_fine_200000.npy"}[which]
    return read_object_npy(os.path.join(lego_dir, name))


def export_npz(lego_dir: str = LEGO_DIR) -> None:
    here = os.path.dirname(os.path.abspath(__file__))
    for which in ("coarse", "fine"):
        arrs = load_arrays(which, lego_dir)
        np.savez(os.path.join(here, f"_teacher_{which}.npz"), **{f"a{i}": a for i, a in enumerate(arrs)})


class Teacher(torch.nn.Module):
    def __init__(self, arrays):
        super().__init__()
        t = [torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)) for a in arrays]
        if len(t) != 24 or tuple(t[10].shape) != (319, 256) or tuple(t[22].shape) != (256, 1):
            raise ValueError("not the original-NeRF 8x256 layout")
        self.trunk_w = torch.nn.ParameterList([torch.nn.Parameter(t[2 * i], requires_grad=False) for i in range(8)])
        self.trunk_b = torch.nn.ParameterList([torch.nn.Parameter(t[2 * i + 1], requires_grad=False) for i in range(8)])
        names = ["feat_w", "feat_b", "views_w", "views_b", "rgb_w", "rgb_b", "alpha_w", "alpha_b"]
        for n, a in zip(names, t[16:]):
            setattr(self, n, torch.nn.Parameter(a, requires_grad=False))

    def forward(self, x: torch.Tensor, d: torch.Tensor):
        """(sigma >= 0 [N,1], rgb in (0,1) [N,3]) at points x seen along directions d
        (any length: normalised here, as the original's ``viewdirs``)."""
        pe = embed(x, 10)
        ve = embed(d / torch.linalg.norm(d, dim=-1, keepdim=True), 4)
        h = pe
        for i in range(8):
            h = F.relu(h @ self.trunk_w[i] + self.trunk_b[i])
            if i == 4:
                h = torch.cat([pe, h], dim=-1)
        sigma = F.relu(h @ self.alpha_w + self.alpha_b)
        feat = h @ self.feat_w + self.feat_b
        h2 = F.relu(torch.cat([feat, ve], dim=-1) @ self.views_w + self.views_b)
        rgb = torch.sigmoid(h2 @ self.rgb_w + self.rgb_b)
        return sigma, rgb


def load_teacher(which: str, device="cpu") -> Teacher:
    return Teacher(load_arrays(which)).to(device).eval()
