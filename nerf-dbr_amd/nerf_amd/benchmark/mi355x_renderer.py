"""MI355X (gfx950) renderer plugin: the reference's render path on hand-written HIP kernels.

Drop-in for the reference's GPU renderer plugins (``PyTorchCUDARenderer``,
``src/benchmark/pytorch_renderers.py:173-246``): construct it (``RuntimeError``
when no MI355X or no built library, like the reference's probe at
``benchmark_suite.py:88-92``), ``setup(checkpoint)``, then ``render_image``.

Every stage runs in ``libnerf_mi355x.so`` (``include/nerf_mi355x.h``):

=============================  =========================================  ======================
reference                      here                                       kernel
=============================  =========================================  ======================
generate_rays                  ``generate_rays``                          rays_kernel
sample_points_on_rays + MLP    fused in ``render_image``                  mlp_{f32,bf16}_kernel
query_nerf_networks            ``query_nerf_networks``                    mlp_*_kernel (points)
execute_volume_rendering       ``execute_volume_rendering``               composite_kernel
importance_sample (broken)     ``render_image`` with ``n_importance``     importance_kernel
=============================  =========================================  ======================

The whole image is one launch per stage (no 512/4096-ray chunking: a frame's
61 M samples x 16 B of MLP output is 1 GB of HBM), and the outputs stay on
the device; the suite's ``.detach().cpu()`` moves them when it needs them.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from .. import runtime as rt
from .base_renderer import BaseUnifiedRenderer

FOCAL = 800.0   # base_renderer.py:224 (fixed for every resolution)


def _pose_np(camera_pose) -> np.ndarray:
    if hasattr(camera_pose, "detach"):
        camera_pose = camera_pose.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(camera_pose, dtype=np.float32).reshape(4, 4))


def t_vals(n: int) -> np.ndarray:
    """The reference's ``torch.linspace(0, 1, n)`` table (base_renderer.py:274), bit for bit."""
    import torch

    return torch.linspace(0.0, 1.0, n).numpy()


class MI355XRenderer(BaseUnifiedRenderer):
    """Uniform-sampling renderer (the reference benchmark's semantics) on MI355X.

    precision: "fp32" (f32-input MFMA; the parity path) or "bf16" (bf16 MFMA,
    fp32 accumulate; the throughput path).  n_importance > 0 turns on the
    build-defined hierarchical mode: ``samples_per_ray`` coarse samples on the
    coarse net, ``n_importance`` inverse-CDF samples, fine net on the sorted
    union.  ``coarse_precision`` runs that coarse pass at another precision
    than the fine pass (e.g. "fp32" under "f16x3": the sampler amplifies the coarse weights'
    rounding, so the coarse pass's accumulation sets how close the render is to the float64
    result of the same chain; include/nerf_mi355x.h NERF_OPT_COARSE_PRECISION).
    """

    def __init__(self, precision: str = "bf16", n_importance: int = 0, device_index: Optional[int] = None,
                 name: Optional[str] = None, coarse_precision: Optional[str] = None):
        import torch

        if precision not in rt.PRECISIONS or (coarse_precision is not None and coarse_precision not in rt.PRECISIONS):
            raise ValueError(f"precision must be one of {sorted(rt.PRECISIONS)}")
        if not torch.cuda.is_available():
            raise RuntimeError("no ROCm/HIP device available")
        idx = torch.cuda.current_device() if device_index is None else int(device_index)
        self.hip = rt.Device(idx)                      # raises RuntimeError without gfx950 / library
        self.device_index = idx
        self.precision = precision
        self.n_importance = int(n_importance)
        self.coarse_precision = coarse_precision
        if coarse_precision is not None:
            self.hip.set_coarse_precision(rt.PRECISIONS[coarse_precision])
        self.focal = FOCAL
        if name is None:
            name = f"MI355X HIP {precision}" + (f" hier+{self.n_importance}" if self.n_importance else "")
            if coarse_precision is not None and self.n_importance:
                name += f" ({coarse_precision} coarse)"
        super().__init__(name, "cuda")
        self._u_cache = {}

    # ------------------------------------------------------------------ setup --
    def setup(self, checkpoint_path: str):
        super().setup(checkpoint_path)
        coarse, fine = self.shared_model.get_models(self.device)
        self.hip.load_weights(rt.NERF_NET_COARSE, coarse)
        self.hip.load_weights(rt.NERF_NET_FINE, fine)

    def setup_original_nerf(self, coarse_arrays, fine_arrays) -> None:
        """Instead of ``setup``: the original NeRF implementation's networks (the 24 arrays each
        of the reference's bundled ``data/lego_example_weights``), rendered
        with this renderer's path and semantics on the fp32 or the split-fp16 kernel
        (include/nerf_mi355x.h NERF_LAYOUT_ORIGINAL_NERF).  Not part of the reference's plugin
        interface."""
        if self.precision not in ("fp32", "f16x3"):
            raise ValueError("the original-NeRF layout renders on fp32 and f16x3 only")
        self.hip.load_original_nerf(rt.NERF_NET_COARSE, coarse_arrays)
        self.hip.load_original_nerf(rt.NERF_NET_FINE, fine_arrays)

    def get_device_info(self) -> str:
        return f"MI355X - {self.hip.name()}"

    def synchronize(self) -> None:
        import torch

        torch.cuda.synchronize(self.device_index)

    # ------------------------------------------------------------- hot path --
    def _u(self, n: int) -> np.ndarray:
        if n not in self._u_cache:
            self._u_cache[n] = t_vals(n)           # deterministic draw: linspace(0, 1, n)
        return self._u_cache[n]

    def render_rows(self, camera_pose, resolution: Tuple[int, int], samples_per_ray: int, row0: int, row1: int,
                    rgb_out=None, depth_out=None, t_rand=None, u=None):
        """Rows [row0, row1) of the image: rgb [rows, W, 3], depth [rows, W] (device tensors).

        Optional per-ray draws (training-style sampling, rendering.py:36-50 / :79):
        ``t_rand`` [rows*W, S] stratifies the first-pass samples; ``u`` [rows*W, n_importance]
        (ascending per ray) replaces the deterministic linspace importance draw."""
        import torch

        width, height = resolution
        rows = row1 - row0
        dev = torch.device("cuda", self.device_index)
        if rgb_out is None:
            rgb_out = torch.empty(rows, width, 3, dtype=torch.float32, device=dev)
        if depth_out is None:
            depth_out = torch.empty(rows, width, dtype=torch.float32, device=dev)
        u_shared = self._u(self.n_importance) if self.n_importance else None
        tr = None if t_rand is None else t_rand.to(dev, torch.float32).reshape(rows * width, -1).contiguous()
        ur = None if u is None else u.to(dev, torch.float32).reshape(rows * width, -1).contiguous()
        with torch.cuda.device(self.device_index):
            self.hip.render(_pose_np(camera_pose), width, height, row0, row1, self.focal, self.near, self.far,
                            t_vals(samples_per_ray), self.n_importance, u_shared, rt.PRECISIONS[self.precision],
                            rgb_out, depth_out, t_rand=tr, u_rays=ur)
        return rgb_out, depth_out

    def torch_device(self):
        import torch

        return torch.device("cuda", self.device_index)

    def render_band(self, camera_pose, resolution: Tuple[int, int], samples_per_ray: int, row0: int, row1: int,
                    out=None):
        """Rows [row0, row1) as one packed device tensor [rows, W, 4] = (r, g, b, depth)
        (nerf_render_band): the tile the multi-GPU gather moves, written in place."""
        import torch

        width, height = resolution
        rows = row1 - row0
        if out is None:
            out = torch.empty(rows, width, 4, dtype=torch.float32, device=self.torch_device())
        u_shared = self._u(self.n_importance) if self.n_importance else None
        with torch.cuda.device(self.device_index):
            self.hip.render_band(_pose_np(camera_pose), width, height, row0, row1, self.focal, self.near, self.far,
                                 t_vals(samples_per_ray), self.n_importance, u_shared,
                                 rt.PRECISIONS[self.precision], out)
        return out

    def render_image(self, camera_pose, resolution: Tuple[int, int], samples_per_ray: int = 64):
        """PyTorchCPURenderer.render_image semantics (pytorch_renderers.py:127-154).  On f16x3
        the frame is checked against fp16's activation range before it is returned
        (NerfRangeError instead of an image with inf / NaN; nerf_ctx_range_status)."""
        width, height = resolution
        out = self.render_rows(camera_pose, resolution, samples_per_ray, 0, height)
        self.check_range()
        return out

    def check_range(self) -> None:
        """f16x3 only: synchronize and raise NerfRangeError if a launch since the last check met
        an activation outside fp16's range.  render_rows / render_band queue work without a host
        synchronization; a caller of those on f16x3 calls this once its frames are done."""
        if self.precision == "f16x3":
            import torch

            with torch.cuda.device(self.device_index):
                self.hip.range_status()

    # ------------------------------------------------ granular plugin methods --
    def generate_rays(self, camera_pose, width: int, height: int, focal: float = FOCAL):
        import torch

        dev = torch.device("cuda", self.device_index)
        o = torch.empty(height, width, 3, dtype=torch.float32, device=dev)
        d = torch.empty_like(o)
        with torch.cuda.device(self.device_index):
            self.hip.generate_rays(_pose_np(camera_pose), width, height, 0, height, focal, o, d)
        return o, d

    def sample_points_on_rays(self, rays_o, rays_d, n_samples: int = 64, t_rand=None):
        """base_renderer.py:260-281 -> (points [N,S,3], z [N,S]) on the device (sample_kernel;
        the render path fuses this step into the MLP kernel).  With ``t_rand`` [N,S] (uniform
        draws in [0,1)) the samples are stratified as VolumeRenderer.sample_points_on_rays
        (perturb=True) does (rendering.py:42-47) with its torch.rand_like injected."""
        import torch

        dev = torch.device("cuda", self.device_index)
        o = rays_o.to(dev, torch.float32).reshape(-1, 3).contiguous()
        d = rays_d.to(dev, torch.float32).reshape(-1, 3).contiguous()
        n = o.shape[0]
        tr = None if t_rand is None else t_rand.to(dev, torch.float32).reshape(n, n_samples).contiguous()
        z = torch.empty(n, n_samples, dtype=torch.float32, device=dev)
        pts = torch.empty(n, n_samples, 3, dtype=torch.float32, device=dev)
        with torch.cuda.device(self.device_index):
            self.hip.sample_points(o, d, t_vals(n_samples), self.near, self.far, z, pts, tr)
        return pts, z

    def query_nerf_networks(self, positions, directions, use_fine: bool = True):
        import torch

        dev = torch.device("cuda", self.device_index)
        pos = positions.to(dev, torch.float32).contiguous()
        dirs = directions.to(dev, torch.float32).contiguous()
        out = torch.empty(pos.shape[0], 4, dtype=torch.float32, device=dev)
        net = rt.NERF_NET_FINE if use_fine else rt.NERF_NET_COARSE
        with torch.cuda.device(self.device_index):
            self.hip.query(net, rt.PRECISIONS[self.precision], pos, dirs, out)
        self.check_range()
        return out[:, :1], out[:, 1:]

    def execute_volume_rendering(self, densities, colors, z_vals, ray_directions, with_weights: bool = False):
        import torch

        dev = torch.device("cuda", self.device_index)
        n, s = z_vals.shape
        sig = densities.to(dev, torch.float32).reshape(n, s).contiguous()
        col = colors.to(dev, torch.float32).reshape(n, s, 3).contiguous()
        z = z_vals.to(dev, torch.float32).contiguous()
        d = ray_directions.to(dev, torch.float32).reshape(n, 3).contiguous()
        rgb = torch.empty(n, 3, dtype=torch.float32, device=dev)
        depth = torch.empty(n, dtype=torch.float32, device=dev)
        acc = torch.empty(n, dtype=torch.float32, device=dev) if with_weights else None
        w = torch.empty(n, s, dtype=torch.float32, device=dev) if with_weights else None
        with torch.cuda.device(self.device_index):
            self.hip.composite(sig, 1, col, 3, z, s, d, n, s, rgb, depth, acc, w)
        return (rgb, depth, acc, w) if with_weights else (rgb, depth)

    def render_rays_z(self, rays_o, rays_d, z, use_fine: bool = True, with_weights: bool = False):
        """MLP + compositing for explicit rays [N,3] and per-ray samples z [N,S] (the
        body of _render_ray_chunk, pytorch_renderers.py:156-170, with z given)."""
        import torch

        dev = torch.device("cuda", self.device_index)
        o = rays_o.to(dev, torch.float32).reshape(-1, 3).contiguous()
        d = rays_d.to(dev, torch.float32).reshape(-1, 3).contiguous()
        zz = z.to(dev, torch.float32).contiguous()
        n, s = zz.shape
        out = torch.empty(n * s, 4, dtype=torch.float32, device=dev)
        net = rt.NERF_NET_FINE if use_fine else rt.NERF_NET_COARSE
        with torch.cuda.device(self.device_index):
            self.hip.mlp_forward(net, rt.PRECISIONS[self.precision], o, d, zz, s, n, s, out)
        rgb = torch.empty(n, 3, dtype=torch.float32, device=dev)
        depth = torch.empty(n, dtype=torch.float32, device=dev)
        acc = torch.empty(n, dtype=torch.float32, device=dev) if with_weights else None
        w = torch.empty(n, s, dtype=torch.float32, device=dev) if with_weights else None
        with torch.cuda.device(self.device_index):
            self.hip.composite(out, 4, out[:, 1:], 4, zz, s, d, n, s, rgb, depth, acc, w)
        self.check_range()
        return (rgb, depth, acc, w) if with_weights else (rgb, depth)

    def importance_sample(self, z_coarse, weights, u):
        """Fixed VolumeRenderer.importance_sample (rendering.py:54-100): sorted union [N, S+Ni].
        ``u`` [N, Ni] or [Ni], ascending along the last axis."""
        import torch

        dev = torch.device("cuda", self.device_index)
        z = z_coarse.to(dev, torch.float32).contiguous()
        w = weights.to(dev, torch.float32).contiguous()
        uu = u.to(dev, torch.float32).contiguous()
        n, s = z.shape
        ni = uu.shape[-1]
        out = torch.empty(n, s + ni, dtype=torch.float32, device=dev)
        with torch.cuda.device(self.device_index):
            self.hip.importance_sample(z, s, w, uu, ni if uu.dim() == 2 else 0, n, s, ni, out)
        return out
