"""Benchmark harness counterpart of the reference's ``UnifiedBenchmarkSuite``
(``src/benchmark/benchmark_suite.py:34-422``): renderer registry probed with
try/except, the same test poses, timing protocol, rays/s formula and CSV schema,
so results from either suite line up column for column.

* registry: ``add_available_renderers`` adds the MI355X plugins, each probed with
  ``except RuntimeError`` like the reference's GPU renderers (``:80-92``); any other
  ``BaseUnifiedRenderer`` (including the reference's own) can be appended to
  ``suite.renderers`` -- the suite only uses the plugin interface;
* poses: ``generate_test_poses`` (``:132-149``): rotation about Y by 2*pi*i/n,
  translation (0, 0, 4) not rotated;
* timing: ``performance_monitor`` around ``render_image``; rays/s = W*H / mean time
  over the views (``:216-220``);
* outputs: ``<out>/benchmark_results.csv`` with the reference's columns (``:244-255``),
  sample renders ``<out>/sample_renders/<name>/view_k_{rgb,depth}.png`` (``:96-124``)
  and a performance plot (``:304-373``).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

CSV_COLUMNS = ["Method", "Device", "Resolution", "Samples/Ray", "Render Time (s)", "Memory (MB)",
               "Rays/Second", "Device Info"]


@dataclass
class BenchmarkResult:
    method_name: str
    device: str
    resolution: str
    samples_per_ray: int
    render_time: float
    memory_mb: float
    rays_per_second: float
    device_info: str


def generate_test_poses(n_views: int = 3):
    import torch

    poses = []
    for i in range(n_views):
        a = i * 2 * math.pi / n_views
        c2w = torch.eye(4, dtype=torch.float32)
        c2w[0, 0] = np.cos(a)
        c2w[0, 2] = np.sin(a)
        c2w[2, 0] = -np.sin(a)
        c2w[2, 2] = np.cos(a)
        c2w[2, 3] = 4.0
        poses.append(c2w)
    return poses


class UnifiedBenchmarkSuite:
    def __init__(self, output_dir: str = "outputs", warmup: int = 1):
        self.renderers = []
        self.results: List[BenchmarkResult] = []
        self.output_dir = output_dir
        self.warmup = warmup
        os.makedirs(os.path.join(output_dir, "sample_renders"), exist_ok=True)

    def add_available_renderers(self, precisions=("fp32", "bf16"), hierarchical: int = 0):
        """MI355X plugins; each probe failure is reported and skipped, as in the reference."""
        from .mi355x_renderer import MI355XRenderer

        print("Detecting available execution methods...")
        for p in precisions:
            try:
                self.renderers.append(MI355XRenderer(p))
                print(f"✓ MI355X HIP {p} renderer added")
            except RuntimeError as e:
                print(f"✗ MI355X HIP {p} not available: {e}")
        if hierarchical:
            try:
                self.renderers.append(MI355XRenderer("bf16", n_importance=hierarchical))
                print(f"✓ MI355X HIP bf16 hierarchical (+{hierarchical}) renderer added")
            except RuntimeError as e:
                print(f"✗ MI355X hierarchical not available: {e}")
        print(f"Total renderers: {len(self.renderers)}")

    def setup_renderers(self, checkpoint_path: str):
        print(f"Setting up renderers with checkpoint: {checkpoint_path}")
        for r in self.renderers:
            r.setup(checkpoint_path)

    generate_test_poses = staticmethod(generate_test_poses)

    def _save_render_samples(self, name: str, view_idx: int, rgb, depth) -> Tuple[str, str]:
        from PIL import Image

        d = os.path.join(self.output_dir, "sample_renders", name.replace(" ", "_"))
        os.makedirs(d, exist_ok=True)
        rgb_np = rgb.detach().cpu().numpy()
        depth_np = depth.detach().cpu().numpy()
        rgb8 = (rgb_np * 255).astype(np.uint8) if rgb_np.max() <= 1.0 else np.clip(rgb_np, 0, 255).astype(np.uint8)
        dn = (depth_np - depth_np.min()) / (depth_np.max() - depth_np.min() + 1e-8)
        rp, dp = os.path.join(d, f"view_{view_idx}_rgb.png"), os.path.join(d, f"view_{view_idx}_depth.png")
        Image.fromarray(rgb8).save(rp)
        Image.fromarray((dn * 255).astype(np.uint8)).save(dp)
        return rp, dp

    def run_benchmark(self, checkpoint_path: str, resolutions=((400, 300), (800, 600)),
                      samples_per_ray_options=(64, 128), n_views: int = 2, save_samples: bool = True):
        self.setup_renderers(checkpoint_path)
        poses = self.generate_test_poses(n_views)
        for r in self.renderers:
            print(f"\nTesting {r.name}...")
            for res in resolutions:
                for spp in samples_per_ray_options:
                    for _ in range(self.warmup):          # first-call allocation/JIT out of the timing
                        r.render_image(poses[0], tuple(res), spp)
                    times, mems = [], []
                    for vi, pose in enumerate(poses):
                        try:
                            with r.performance_monitor():
                                rgb, depth = r.render_image(pose, tuple(res), spp)
                            if save_samples and tuple(res) == tuple(resolutions[0]) and spp == samples_per_ray_options[0]:
                                self._save_render_samples(r.name, vi, rgb, depth)
                            times.append(r.last_render_time)
                            mems.append(r.peak_memory_mb)
                            print(f"    View {vi + 1}: {r.last_render_time:.4f}s")
                        except Exception as e:   # a failing view is skipped (reference :212-214)
                            print(f"    View {vi + 1}: FAILED - {e}")
                    if times:
                        t = float(np.mean(times))
                        rays = res[0] * res[1]
                        self.results.append(BenchmarkResult(r.name, r.device, f"{res[0]}x{res[1]}", spp, t,
                                                            float(np.mean(mems)), rays / t, r.get_device_info()))
                        print(f"    Average: {t:.4f}s, {rays / t:.0f} rays/s")

    def generate_report(self, plot: bool = True):
        import pandas as pd

        rows = [[r.method_name, r.device, r.resolution, r.samples_per_ray, r.render_time, r.memory_mb,
                 r.rays_per_second, r.device_info] for r in self.results]
        df = pd.DataFrame(rows, columns=CSV_COLUMNS)
        if df.empty:
            print("No results to report")
            return df
        path = os.path.join(self.output_dir, "benchmark_results.csv")
        df.to_csv(path, index=False)
        print(f"Results saved to {path}")
        if plot:
            self._plot(df)
        return df

    def _plot(self, df) -> Optional[str]:
        try:
            import matplotlib

            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
        except Exception:
            return None
        fig, ax = plt.subplots(figsize=(9, 5))
        for name, g in df.groupby("Method"):
            lab = g["Resolution"] + "@" + g["Samples/Ray"].astype(str)
            ax.plot(lab, g["Rays/Second"], marker="o", label=name)
        ax.set_yscale("log")
        ax.set_ylabel("rays / s")
        ax.legend()
        ax.tick_params(axis="x", rotation=45)
        fig.tight_layout()
        p = os.path.join(self.output_dir, "performance_comparison.png")
        fig.savefig(p)
        plt.close(fig)
        return p
