"""The benchmark-renderer plugin interface, restated for this package.

Same contract as the reference's ``BaseUnifiedRenderer``
(``src/benchmark/base_renderer.py:90-281``) and ``SharedNeRFModel``
(``base_renderer.py:16-87``), so a renderer written against either works with
either suite:

* ``__init__(name, device)`` sets ``name``, ``device``, ``near=2.0``, ``far=6.0``,
  ``last_render_time``, ``peak_memory_mb``;
* ``setup(checkpoint_path)`` loads the shared (coarse, fine) networks;
* ``performance_monitor()`` times a render (wall clock, device synchronised)
  and samples peak RSS every 10 ms;
* ``render_image(pose[4,4], (W, H), samples_per_ray)`` -> ``(rgb[H,W,3], depth[H,W])``;
* ``execute_volume_rendering(sigma[N,S,1], rgb[N,S,3], z[N,S], d[N,3])`` -> ``(rgb[N,3], depth[N])``.

Differences, all deliberate: checkpoints are read with ``weights_only=True``
(nothing in a checkpoint executes), and the shared model caches the weights
as host arrays -- device placement belongs to each renderer.
"""
from __future__ import annotations

import threading
import time
from abc import ABC, abstractmethod
from contextlib import contextmanager
from typing import Dict, Tuple

import psutil

from .. import weights as W


class SharedNeRFModel:
    """Process-wide (coarse, fine) weights, loaded once per checkpoint (base_renderer.py:16-87)."""

    _instance = None
    _models: Dict[str, Tuple[W.StateDict, W.StateDict]] = {}
    _loaded_checkpoint = None

    def __new__(cls):
        if cls._instance is None:
            cls._instance = super().__new__(cls)
        return cls._instance

    def load_models(self, checkpoint_path: str, device: str = "cpu"):
        if checkpoint_path in self._models:
            print(f"Using cached models for device: {device}")
            self._loaded_checkpoint = checkpoint_path
            return
        print(f"Loading shared NeRF models from {checkpoint_path} for device: {device}")
        try:
            coarse, fine = W.load_checkpoint(checkpoint_path)
            print("Shared models loaded successfully")
        except FileNotFoundError:
            # the reference's behaviour (base_renderer.py:62-76): random weights
            print("Checkpoint not found, using randomly initialized models")
            coarse, fine = W.synthetic_models(0, conditioned=False)
        self._models[checkpoint_path] = (coarse, fine)
        self._loaded_checkpoint = checkpoint_path

    def get_models(self, device: str = "cpu"):
        if self._loaded_checkpoint is None:
            raise RuntimeError(f"Models not loaded for device {device}. Call load_models() first.")
        return self._models[self._loaded_checkpoint]

    @classmethod
    def reset(cls) -> None:
        cls._models = {}
        cls._loaded_checkpoint = None


class BaseUnifiedRenderer(ABC):
    """Plugin interface (base_renderer.py:90-281)."""

    def __init__(self, name: str, device: str = "cpu"):
        self.name = name
        self.device = device
        self.shared_model = SharedNeRFModel()
        self.last_render_time = 0.0
        self.peak_memory_mb = 0.0
        self._monitoring = False
        self.near = 2.0
        self.far = 6.0
        print(f"Initialized {self.name} renderer on {device}")

    def setup(self, checkpoint_path: str):
        self.shared_model.load_models(checkpoint_path, self.device)

    def synchronize(self) -> None:
        if self.device == "cuda":
            import torch

            torch.cuda.synchronize()

    @contextmanager
    def performance_monitor(self):
        """Wall-clock a render with the device synchronised on both sides (base_renderer.py:118-147)."""
        memory_thread = threading.Thread(target=self._monitor_memory)
        self.peak_memory_mb = psutil.Process().memory_info().rss / 1024 / 1024
        self._monitoring = True
        memory_thread.start()
        try:
            self.synchronize()
            start = time.time()
            yield
            self.synchronize()
            self.last_render_time = time.time() - start
        finally:
            self._monitoring = False
            memory_thread.join()

    def _monitor_memory(self):
        while self._monitoring:
            self.peak_memory_mb = max(self.peak_memory_mb, psutil.Process().memory_info().rss / 1024 / 1024)
            time.sleep(0.01)

    def get_device_info(self) -> str:
        return f"CPU - {psutil.cpu_count()} cores"

    # The reference gives these three a generic torch body; here the concrete
    # renderer supplies them (this package computes nothing outside the HIP
    # library), so the base raises.  Abstract are exactly the reference's two.
    def query_nerf_networks(self, positions, directions, use_fine: bool = True):
        """(density [N,1], rgb [N,3]) of the shared network (base_renderer.py:165-188)."""
        raise NotImplementedError(f"{type(self).__name__} does not implement query_nerf_networks")

    @abstractmethod
    def execute_volume_rendering(self, densities, colors, z_vals, ray_directions):
        """(rgb [N,3], depth [N]) (base_renderer.py:190-205)."""

    @abstractmethod
    def render_image(self, camera_pose, resolution: Tuple[int, int], samples_per_ray: int = 64):
        """(rgb [H,W,3], depth [H,W]) (base_renderer.py:207-221)."""

    def generate_rays(self, camera_pose, width: int, height: int, focal: float = 800.0):
        """(rays_o, rays_d), each [H,W,3] (base_renderer.py:223-258)."""
        raise NotImplementedError(f"{type(self).__name__} does not implement generate_rays")

    def sample_points_on_rays(self, rays_o, rays_d, n_samples: int = 64):
        """(points [N,S,3], z [N,S]) (base_renderer.py:260-281)."""
        raise NotImplementedError(f"{type(self).__name__} does not implement sample_points_on_rays")
