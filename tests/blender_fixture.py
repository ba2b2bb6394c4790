"""A tiny Blender-format (NeRF-synthetic) dataset written on the fly for the loader tests."""
import json
import os

import numpy as np


def look_at(eye):
    eye = np.asarray(eye, dtype=np.float64)
    fwd = -eye / np.linalg.norm(eye)
    right = np.cross(fwd, [0.0, 0.0, 1.0])
    right /= np.linalg.norm(right)
    c2w = np.eye(4)
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = right, np.cross(right, fwd), -fwd, eye
    return c2w


def write_blender_dataset(root, splits=(("train", 2), ("val", 1)), size=(12, 10), seed=0):
    """transforms_<split>.json + RGBA PNGs (random colour, random alpha); returns the
    RGBA arrays per split."""
    from PIL import Image

    rng = np.random.RandomState(seed)
    out = {}
    for split, n in splits:
        os.makedirs(os.path.join(root, split), exist_ok=True)
        frames, imgs = [], []
        for k in range(n):
            a = 2 * np.pi * k / max(n, 1)
            rgba = rng.randint(0, 256, size=(size[1], size[0], 4)).astype(np.uint8)
            Image.fromarray(rgba, "RGBA").save(os.path.join(root, split, f"r_{k}.png"))
            frames.append({"file_path": f"./{split}/r_{k}",
                           "transform_matrix": look_at([3.0 * np.cos(a), 3.0 * np.sin(a), 1.5]).tolist()})
            imgs.append(rgba)
        with open(os.path.join(root, f"transforms_{split}.json"), "w") as f:
            json.dump({"camera_angle_x": 0.6911112070083618, "frames": frames}, f)
        out[split] = imgs
    return out
