"""The NeRF-synthetic (Blender) dataset reader the training mode consumes.

Same contract as the reference's ``src/data/loader.py`` (``SyntheticDataset``,
``load_synthetic_data``, ``loader.py:13-129``): ``transforms_<split>.json`` gives
``camera_angle_x`` and per-frame ``file_path`` / ``transform_matrix``; each PNG is
read as RGBA, resized to ``img_wh`` (800x800 by default) with Lanczos filtering,
scaled to [0, 1] and composited on a white background; ``focal = 0.5 W /
tan(0.5 camera_angle_x)``; items are ``{'image' [H,W,3], 'pose' [4,4], 'focal'}``.
A missing split is skipped with the reference's warning.  This is host-side data
plumbing for ``MI355XTrainer.train`` (the device work is ``nerf_train_step``).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Tuple

import numpy as np


class SyntheticDataset:
    def __init__(self, data_dir: str, split: str = "train", img_wh: Tuple[int, int] = (800, 800),
                 device: str = "cpu"):
        import torch
        from PIL import Image

        self.data_dir, self.split, self.device = data_dir, split, device
        self.img_w, self.img_h = img_wh
        with open(os.path.join(data_dir, f"transforms_{split}.json")) as f:
            self.meta = json.load(f)
        self.focal = 0.5 * self.img_w / np.tan(0.5 * self.meta["camera_angle_x"])
        images, poses = [], []
        for frame in self.meta["frames"]:
            img = Image.open(os.path.join(data_dir, frame["file_path"] + ".png")).convert("RGBA")
            a = np.array(img.resize((self.img_w, self.img_h), Image.LANCZOS)) / 255.0
            images.append(a[..., :3] * a[..., 3:4] + (1 - a[..., 3:4]))
            poses.append(np.array(frame["transform_matrix"]))
        self.images = torch.FloatTensor(np.stack(images)).to(device)
        self.poses = torch.FloatTensor(np.stack(poses)).to(device)
        print(f"Loaded {len(self.images)} images from {split} split")

    def __len__(self) -> int:
        return len(self.images)

    def __getitem__(self, idx: int):
        return {"image": self.images[idx], "pose": self.poses[idx], "focal": self.focal}


def load_synthetic_data(data_dir: str, device: str = "cpu", img_wh: Tuple[int, int] = (800, 800)
                        ) -> Dict[str, SyntheticDataset]:
    datasets = {}
    for split in ("train", "val", "test"):
        try:
            datasets[split] = SyntheticDataset(data_dir, split, img_wh, device)
        except FileNotFoundError:
            print(f"Warning: {split} split not found in {data_dir}")
    return datasets
