"""Generate the golden vectors in tests/golden/ from the reference itself.

Run in the development container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [/root/reference]
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --lego [/root/reference]
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --lego-full [/root/reference]

It imports the reference's Python renderer, model and volume-render utilities
(bypassing ``src/benchmark/__init__.py``, whose ``numba`` import is absent here
-- SURVEY §8c import recipe), feeds them the deterministic synthetic checkpoint
of ``nerf_amd.weights`` and records inputs and outputs as ``.npz`` data.  Only
data is committed; no reference source is copied.

Fixtures (every array fp32 unless noted):
  rays.npz        generate_rays        base_renderer.py:223-258
  tvals.npz       sample_points_on_rays base_renderer.py:260-281 (z only)
  pe.npz          PositionalEncoding.encode nerf.py:24-45, L=10 and L=4
  mlp.npz         NeRFModel.forward    nerf.py:92-131 (coarse and fine)
  composite.npz   execute_volume_rendering pytorch_renderers.py:105-125 and
                  VolumeRenderer.volume_render rendering.py:102-143
  stratified.npz  VolumeRenderer.sample_points_on_rays(perturb=True) rendering.py:17-52
  render_*.npz    PyTorchCPURenderer.render_image pytorch_renderers.py:127-170
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "nerf-dbr_amd"))

from nerf_amd import weights as W  # noqa: E402


def import_reference(ref_root: str):
    sys.path.insert(0, ref_root)
    import src  # noqa: F401

    bp = types.ModuleType("src.benchmark")
    bp.__path__ = [os.path.join(ref_root, "src", "benchmark")]
    sys.modules["src.benchmark"] = bp
    from src.benchmark.pytorch_renderers import PyTorchCPURenderer
    from src.models.nerf import NeRFModel, PositionalEncoding
    from src.utils.rendering import VolumeRenderer

    return PyTorchCPURenderer, NeRFModel, PositionalEncoding, VolumeRenderer


def suite_poses(n_views: int = 2):
    """Same construction as benchmark_suite.py:132-149 (data, not imported)."""
    import torch

    poses = []
    for i in range(n_views):
        a = i * 2 * np.pi / n_views
        c2w = torch.eye(4, dtype=torch.float32)
        c2w[0, 0] = np.cos(a)
        c2w[0, 2] = np.sin(a)
        c2w[2, 0] = -np.sin(a)
        c2w[2, 2] = np.cos(a)
        c2w[2, 3] = 4.0
        poses.append(c2w)
    return poses


def off_axis_pose():
    """A look-at pose that is not axis-aligned (exercises every rotation term)."""
    import torch

    eye = np.array([2.7, 1.9, 2.3], dtype=np.float64)
    fwd = -eye / np.linalg.norm(eye)
    up = np.array([0.0, 1.0, 0.0])
    right = np.cross(fwd, up)
    right /= np.linalg.norm(right)
    up2 = np.cross(right, fwd)
    c2w = np.eye(4)
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = right, up2, -fwd, eye
    return torch.tensor(c2w, dtype=torch.float32)


def main(ref_root: str = "/root/reference") -> None:
    import torch

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    PyTorchCPURenderer, NeRFModel, PositionalEncoding, VolumeRenderer = import_reference(ref_root)

    coarse_sd, fine_sd = W.synthetic_models(0)
    ckpt_path = os.path.join(tempfile.mkdtemp(prefix="nerf_golden_"), "synthetic.pth")
    W.save_checkpoint(ckpt_path, coarse_sd, fine_sd)

    def net(sd):
        m = NeRFModel()
        m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in sd.items()})
        return m.eval()

    coarse, fine = net(coarse_sd), net(fine_sd)
    renderer = PyTorchCPURenderer()
    renderer.setup(ckpt_path)
    poses = suite_poses(2) + [off_axis_pose()]
    pose_arr = np.stack([p.numpy() for p in poses])
    meta = {
        "torch": torch.__version__,
        "numpy": np.__version__,
        "coarse_digest": W.state_dict_digest(coarse_sd),
        "fine_digest": W.state_dict_digest(fine_sd),
        "seed": 0,
        "poses": "suite views 0,1 (benchmark_suite.py:132-149) + off-axis look-at",
    }
    save = lambda name, **kw: np.savez_compressed(os.path.join(HERE, name), **kw)  # noqa: E731

    # ---- rays -------------------------------------------------------------
    rays = {"poses": pose_arr}
    for (w, h) in [(64, 48), (37, 23), (200, 150)]:
        for pi, p in enumerate(poses):
            ro, rd = renderer.generate_rays(p, w, h)
            rays[f"o_{w}x{h}_{pi}"] = ro.numpy()
            rays[f"d_{w}x{h}_{pi}"] = rd.numpy()
    save("rays.npz", **rays)

    # ---- t_vals / z_vals ----------------------------------------------------
    tv = {}
    ro = torch.zeros(1, 3)
    rd = torch.ones(1, 3)
    for s in [1, 2, 3, 16, 32, 64, 128, 192, 256]:
        _, z = renderer.sample_points_on_rays(ro, rd, s)
        tv[f"z_{s}"] = z[0].numpy()
        tv[f"t_{s}"] = torch.linspace(0.0, 1.0, s).numpy()
    save("tvals.npz", **tv)

    # ---- positional encoding -----------------------------------------------
    g = torch.Generator().manual_seed(1234)
    x = torch.cat([
        (torch.rand(2048, 3, generator=g) * 2 - 1) * 2.0,
        (torch.rand(1024, 3, generator=g) * 2 - 1) * 10.5,     # suite view 1 reaches |z|~10
        torch.tensor([[0.0, -0.0, 1.0], [10.0, -10.0, 7.25], [1e-8, -3e-39, 2.5]]),
    ])
    pe10 = PositionalEncoding(10).encode(x)
    pe4 = PositionalEncoding(4).encode(x)
    save("pe.npz", x=x.numpy(), pe10=pe10.numpy(), pe4=pe4.numpy())

    # ---- MLP forward (points taken from real rays of both views) -------------
    ro0, rd0 = renderer.generate_rays(poses[0], 64, 48)
    ro1, rd1 = renderer.generate_rays(poses[2], 64, 48)
    pts0, _ = renderer.sample_points_on_rays(ro0.reshape(-1, 3)[:64], rd0.reshape(-1, 3)[:64], 32)
    pts1, _ = renderer.sample_points_on_rays(ro1.reshape(-1, 3)[-64:], rd1.reshape(-1, 3)[-64:], 32)
    pos = torch.cat([pts0.reshape(-1, 3), pts1.reshape(-1, 3)])
    dirs = torch.cat([rd0.reshape(-1, 3)[:64].repeat_interleave(32, 0),
                      rd1.reshape(-1, 3)[-64:].repeat_interleave(32, 0)])
    with torch.no_grad():
        sf, cf = fine(pos, dirs)
        sc, cc = coarse(pos, dirs)
    save("mlp.npz", pos=pos.numpy(), dirs=dirs.numpy(), sigma_fine=sf.numpy(), rgb_fine=cf.numpy(),
         sigma_coarse=sc.numpy(), rgb_coarse=cc.numpy())

    # ---- compositing ---------------------------------------------------------
    vr = VolumeRenderer("cpu")
    comp = {}
    g = torch.Generator().manual_seed(99)
    cases = {}
    for s in [16, 32, 64, 128]:
        n = 96
        sig = torch.rand(n, s, 1, generator=g) * 3.0 - 0.5          # includes negatives (ReLU)
        col = torch.rand(n, s, 3, generator=g)
        _, zz = renderer.sample_points_on_rays(torch.zeros(n, 3), torch.ones(n, 3), s)
        dd = torch.randn(n, 3, generator=g)
        cases[f"rand{s}"] = (sig, col, zz.contiguous(), dd)
    s = 64
    n = 8
    _, zz = renderer.sample_points_on_rays(torch.zeros(n, 3), torch.ones(n, 3), s)
    dd = torch.randn(n, 3, generator=g)
    col = torch.rand(n, s, 3, generator=g)
    edge = torch.zeros(n, s, 1)
    edge[1] = 1e4                                  # huge density everywhere
    edge[2, -1] = 5.0                              # density only at the last sample (dist 1e10)
    edge[3, -1] = 1e-9                             # tiny density at the last sample
    edge[4, :, 0] = torch.linspace(-1, 1, s)       # ramp through zero
    edge[5, 10] = 50.0                             # a single opaque slab
    edge[6] = 1e-7
    edge[7, :, 0] = torch.tensor([1e-30 * (k + 1) for k in range(s)])   # denormal-ish
    cases["edge64"] = (edge, col, zz.contiguous(), dd)
    for name, (sig, col, zz, dd) in cases.items():
        rgb, depth = renderer.execute_volume_rendering(sig, col, zz, dd)
        rgb2, depth2, acc, wts = vr.volume_render(sig, col, zz, dd)
        comp[f"{name}_sigma"] = sig.numpy()
        comp[f"{name}_rgb_in"] = col.numpy()
        comp[f"{name}_z"] = zz.numpy()
        comp[f"{name}_d"] = dd.numpy()
        comp[f"{name}_rgb"] = rgb.numpy()
        comp[f"{name}_depth"] = depth.numpy()
        comp[f"{name}_acc"] = acc.numpy()
        comp[f"{name}_weights"] = wts.numpy()
        assert torch.equal(rgb, rgb2) and torch.equal(depth, depth2)
    save("composite.npz", **comp)

    # ---- stratified (perturbed) sampling with captured t_rand -----------------
    ro_s, rd_s = renderer.generate_rays(poses[0], 16, 8)
    ro_s, rd_s = ro_s.reshape(-1, 3), rd_s.reshape(-1, 3)
    torch.manual_seed(7)
    pts_s, z_s = vr.sample_points_on_rays(ro_s, rd_s, 2.0, 6.0, 32, perturb=True)
    torch.manual_seed(7)
    t_rand = torch.rand(ro_s.shape[0], 32)
    save("stratified.npz", rays_o=ro_s.numpy(), rays_d=rd_s.numpy(), t_rand=t_rand.numpy(),
         z=z_s.numpy(), pts=pts_s.numpy())

    # ---- full renders --------------------------------------------------------
    timing = {}
    for (w, h, s, pose_ids) in [(64, 48, 16, [0, 1, 2]), (37, 23, 7, [2]), (200, 150, 32, [0, 1, 2]),
                                (400, 300, 64, [0])]:
        out = {"poses": pose_arr[pose_ids], "pose_ids": np.array(pose_ids, dtype=np.int32),
               "W": np.int32(w), "H": np.int32(h), "S": np.int32(s)}
        for k, pi in enumerate(pose_ids):
            t0 = time.time()
            rgb, depth = renderer.render_image(poses[pi], (w, h), s)
            timing[f"{w}x{h}x{s}_view{pi}"] = time.time() - t0
            out[f"rgb_{k}"] = rgb.numpy()
            out[f"depth_{k}"] = depth.numpy()
        save(f"render_{w}x{h}_s{s}.npz", **out)

    # a band of the 800x600x128 headline image, rendered with the reference's own
    # per-chunk path on rows [296, 304) only (chunking is result-neutral: SURVEY a7)
    band = {"rows": np.array([296, 304], dtype=np.int32), "W": np.int32(800), "H": np.int32(600),
            "S": np.int32(128), "poses": pose_arr[[0, 2]]}
    for k, pi in enumerate([0, 2]):
        ro, rd = renderer.generate_rays(poses[pi], 800, 600)
        ro = ro[296:304].reshape(-1, 3)
        rd = rd[296:304].reshape(-1, 3)
        rgbs, depths = [], []
        for c in range(0, ro.shape[0], 512):
            r_, d_ = renderer._render_ray_chunk(ro[c:c + 512], rd[c:c + 512], 128)
            rgbs.append(r_)
            depths.append(d_)
        band[f"rgb_{k}"] = torch.cat(rgbs).reshape(8, 800, 3).numpy()
        band[f"depth_{k}"] = torch.cat(depths).reshape(8, 800).numpy()
    save("render_800x600_s128_band.npz", **band)

    meta["render_seconds"] = timing
    with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta, indent=1))


def main_lego(ref_root: str = "/root/reference") -> None:
    """Fixtures on the distilled Lego checkpoint (nerf_amd.weights.LEGO_NPZ, SURVEY §8f
    row 1), rendered by the reference's own PyTorchCPURenderer: the BASELINE configs'
    content.  lego_mlp.npz (NeRFModel.forward, both nets, points on rays through the
    scene), render_lego_200x150_s32 (suite views 0, 1 + off-axis), render_lego_400x300_s64
    (config 2: view 0 + off-axis) and a band of the 800x600x128 headline frame (rows
    [296, 304), view 0 + off-axis)."""
    import torch

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    PyTorchCPURenderer, NeRFModel, _, _ = import_reference(ref_root)
    coarse_sd, fine_sd = W.lego_models()
    ckpt_path = os.path.join(tempfile.mkdtemp(prefix="nerf_golden_lego_"), "lego.pth")
    W.save_checkpoint(ckpt_path, coarse_sd, fine_sd)

    def net(sd):
        m = NeRFModel()
        m.load_state_dict({k: torch.from_numpy(v.copy()) for k, v in sd.items()})
        return m.eval()

    coarse, fine = net(coarse_sd), net(fine_sd)
    renderer = PyTorchCPURenderer()
    renderer.setup(ckpt_path)
    poses = suite_poses(2) + [off_axis_pose()]
    pose_arr = np.stack([p.numpy() for p in poses])
    save = lambda name, **kw: np.savez_compressed(os.path.join(HERE, name), **kw)  # noqa: E731
    meta = {"torch": torch.__version__, "numpy": np.__version__, "checkpoint": "nerf_amd/checkpoints/lego_distilled.npz",
            "coarse_digest": W.state_dict_digest(coarse_sd), "fine_digest": W.state_dict_digest(fine_sd),
            "poses": "suite views 0,1 (benchmark_suite.py:132-149) + off-axis look-at"}

    # MLP forward on points of rays through the scene (view 0 centre rows, off-axis centre rows)
    pos, dirs = [], []
    for pi in (0, 2):
        ro, rd = renderer.generate_rays(poses[pi], 800, 600)
        ro, rd = ro[300, 300:364].reshape(-1, 3), rd[300, 300:364].reshape(-1, 3)
        pts, _ = renderer.sample_points_on_rays(ro, rd, 64)
        pos.append(pts.reshape(-1, 3))
        dirs.append(rd.repeat_interleave(64, 0))
    pos, dirs = torch.cat(pos), torch.cat(dirs)
    with torch.no_grad():
        sf, cf = fine(pos, dirs)
        sc, cc = coarse(pos, dirs)
    save("lego_mlp.npz", pos=pos.numpy(), dirs=dirs.numpy(), sigma_fine=sf.numpy(), rgb_fine=cf.numpy(),
         sigma_coarse=sc.numpy(), rgb_coarse=cc.numpy())

    timing = {}
    for (w, h, s, pose_ids) in [(200, 150, 32, [0, 1, 2]), (400, 300, 64, [0, 2])]:
        out = {"poses": pose_arr[pose_ids], "pose_ids": np.array(pose_ids, dtype=np.int32),
               "W": np.int32(w), "H": np.int32(h), "S": np.int32(s)}
        for k, pi in enumerate(pose_ids):
            t0 = time.time()
            rgb, depth = renderer.render_image(poses[pi], (w, h), s)
            timing[f"{w}x{h}x{s}_view{pi}"] = time.time() - t0
            out[f"rgb_{k}"] = rgb.numpy()
            out[f"depth_{k}"] = depth.numpy()
        save(f"render_lego_{w}x{h}_s{s}.npz", **out)
    band = {"rows": np.array([296, 304], dtype=np.int32), "W": np.int32(800), "H": np.int32(600),
            "S": np.int32(128), "poses": pose_arr[[0, 2]]}
    for k, pi in enumerate([0, 2]):
        ro, rd = renderer.generate_rays(poses[pi], 800, 600)
        ro, rd = ro[296:304].reshape(-1, 3), rd[296:304].reshape(-1, 3)
        rgbs, depths = [], []
        for c in range(0, ro.shape[0], 512):
            r_, d_ = renderer._render_ray_chunk(ro[c:c + 512], rd[c:c + 512], 128)
            rgbs.append(r_)
            depths.append(d_)
        band[f"rgb_{k}"] = torch.cat(rgbs).reshape(8, 800, 3).numpy()
        band[f"depth_{k}"] = torch.cat(depths).reshape(8, 800).numpy()
    save("render_lego_800x600_s128_band.npz", **band)
    meta["render_seconds"] = timing
    with open(os.path.join(HERE, "golden_lego_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta, indent=1))


def main_lego_full(ref_root: str = "/root/reference") -> None:
    """The whole 800x600x128 headline frame on the Lego checkpoint, rendered by the
    reference's own ``PyTorchCPURenderer.render_image`` (pytorch_renderers.py:127-170)
    for suite views 0 and 1 (benchmark_suite.py:132-149, the bench's two-view protocol)
    and the off-axis pose: render_lego_800x600_s128_full.npz (about 3 min a frame on
    8 cores)."""
    import torch

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    PyTorchCPURenderer, _, _, _ = import_reference(ref_root)
    coarse_sd, fine_sd = W.lego_models()
    ckpt_path = os.path.join(tempfile.mkdtemp(prefix="nerf_golden_lego_full_"), "lego.pth")
    W.save_checkpoint(ckpt_path, coarse_sd, fine_sd)
    renderer = PyTorchCPURenderer()
    renderer.setup(ckpt_path)
    poses = suite_poses(2) + [off_axis_pose()]
    pose_ids = [0, 1, 2]
    out = {"poses": np.stack([poses[i].numpy() for i in pose_ids]), "pose_ids": np.array(pose_ids, dtype=np.int32),
           "W": np.int32(800), "H": np.int32(600), "S": np.int32(128)}
    timing = {}
    for k, pi in enumerate(pose_ids):
        t0 = time.time()
        rgb, depth = renderer.render_image(poses[pi], (800, 600), 128)
        timing[f"800x600x128_view{pi}"] = time.time() - t0
        print(f"view {pi}: {timing[f'800x600x128_view{pi}']:.1f} s", flush=True)
        out[f"rgb_{k}"] = rgb.numpy()
        out[f"depth_{k}"] = depth.numpy()
    np.savez_compressed(os.path.join(HERE, "render_lego_800x600_s128_full.npz"), **out)
    meta_path = os.path.join(HERE, "golden_lego_meta.json")
    with open(meta_path) as f:
        meta = json.load(f)
    meta.setdefault("render_seconds", {}).update(timing)
    meta["full_frame_digest_check"] = {"fine_digest": W.state_dict_digest(fine_sd)}
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


def main_lego_c3(ref_root: str = "/root/reference") -> None:
    """BASELINE config 3 (800x600, 64 coarse + 128 importance) on the Lego checkpoint, whole
    frames, for suite view 0 and the off-axis pose: render_lego_800x600_c3_full.npz.

    The reference's intended chain (src/utils/rendering.py:54-143) with the reference's own
    pieces wherever one runs: rays and the 64 uniform coarse samples from
    ``generate_rays`` / ``sample_points_on_rays`` (base_renderer.py:223-281), the COARSE
    ``NeRFModel`` through ``query_nerf_networks(use_fine=False)`` (:165-188),
    ``VolumeRenderer.volume_render`` for the weights (rendering.py:102-143); then the oracle's
    fixed-gather sampler with u = linspace(0, 1, 128) (the reference's ``importance_sample``
    crashes at its gather, rendering.py:85-90, SURVEY F3 -- build-defined), the sorted union
    of 192 depths, the FINE ``NeRFModel`` and ``volume_render`` again.  512-ray chunks as
    ``PyTorchCPURenderer`` (pytorch_renderers.py:137).  Besides RGB and depth, the fixture
    keeps a 32-bit digest of each ray's 192 fine depths (``oracle.z_row_digest``) so that a GPU
    test can tell which rays it rendered on the very same samples.  About 6 min a frame on 8
    cores."""
    import torch

    sys.path.insert(0, REPO)
    from oracle import nerf_oracle as O

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    PyTorchCPURenderer, _, _, VolumeRenderer = import_reference(ref_root)
    coarse_sd, fine_sd = W.lego_models()
    ckpt_path = os.path.join(tempfile.mkdtemp(prefix="nerf_golden_lego_c3_"), "lego.pth")
    W.save_checkpoint(ckpt_path, coarse_sd, fine_sd)
    renderer = PyTorchCPURenderer()
    renderer.setup(ckpt_path)
    vr = VolumeRenderer("cpu")
    poses = suite_poses(2) + [off_axis_pose()]
    pose_ids = [0, 2]
    w_, h_, nc, ni = 800, 600, 64, 128
    out = {"poses": np.stack([poses[i].numpy() for i in pose_ids]), "pose_ids": np.array(pose_ids, dtype=np.int32),
           "W": np.int32(w_), "H": np.int32(h_), "S_coarse": np.int32(nc), "S_importance": np.int32(ni)}
    timing = {}
    for k, pi in enumerate(pose_ids):
        t0 = time.time()
        ro, rd = renderer.generate_rays(poses[pi], w_, h_)
        ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
        rgbs, depths, digests = [], [], []
        for c in range(0, ro.shape[0], 512):
            o, d = ro[c:c + 512], rd[c:c + 512]
            m = o.shape[0]
            pts, zc = renderer.sample_points_on_rays(o, d, nc)
            dirs = d[:, None, :].expand(m, nc, 3).reshape(-1, 3)
            sig, col = renderer.query_nerf_networks(pts.reshape(-1, 3), dirs, use_fine=False)
            _, _, _, wts = vr.volume_render(sig.reshape(m, nc, 1), col.reshape(m, nc, 3), zc, d)
            zf = O.fine_z(zc.contiguous(), wts, O.default_u(m, ni))
            pts = o[..., None, :] + d[..., None, :] * zf[..., :, None]
            dirs = d[:, None, :].expand(m, nc + ni, 3).reshape(-1, 3)
            sig, col = renderer.query_nerf_networks(pts.reshape(-1, 3), dirs, use_fine=True)
            rgb, depth, _, _ = vr.volume_render(sig.reshape(m, -1, 1), col.reshape(m, -1, 3), zf, d)
            rgbs.append(rgb)
            depths.append(depth)
            digests.append(O.z_row_digest(zf))
            if c % (512 * 100) == 0:
                print(f"view {pi}: ray {c} of {ro.shape[0]}, {time.time() - t0:.0f} s", flush=True)
        out[f"rgb_{k}"] = torch.cat(rgbs).reshape(h_, w_, 3).numpy()
        out[f"depth_{k}"] = torch.cat(depths).reshape(h_, w_).numpy()
        out[f"zf_digest_{k}"] = np.concatenate(digests).reshape(h_, w_)
        timing[f"800x600_c3_64+128_view{pi}"] = time.time() - t0
        print(f"view {pi}: {timing[f'800x600_c3_64+128_view{pi}']:.1f} s", flush=True)
    np.savez_compressed(os.path.join(HERE, "render_lego_800x600_c3_full.npz"), **out)
    meta_path = os.path.join(HERE, "golden_lego_meta.json")
    with open(meta_path) as f:
        meta = json.load(f)
    meta.setdefault("render_seconds", {}).update(timing)
    meta["c3_full_frame"] = {
        "fine_digest": W.state_dict_digest(fine_sd), "coarse_digest": W.state_dict_digest(coarse_sd),
        "chain": "reference generate_rays/sample_points_on_rays(64)/coarse NeRFModel/volume_render -> "
                 "oracle.fine_z (fixed gather, u=linspace(0,1,128), sorted union) -> reference fine NeRFModel/"
                 "volume_render; build-defined sampler (reference importance_sample crashes, SURVEY F3)"}
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


def _fine_z_f64(z, weights, u):
    """The oracle's fixed-gather sampler (oracle.importance_sample / fine_z, after
    rendering.py:72-95) with the dtype of its inputs kept: the float64 truth's sampler."""
    import torch

    n = z.shape[-1]
    w = weights + 1e-5
    pdf = w / torch.cumsum(w, -1)[..., -1:]
    cdf = torch.cat([torch.zeros_like(pdf[..., :1]), torch.cumsum(pdf, -1)], -1)
    idx = torch.searchsorted(cdf.contiguous(), u.contiguous(), right=True)
    below, above = torch.clamp(idx - 1, 0, n - 1), torch.clamp(idx, 0, n - 1)
    cdf_b, cdf_a = torch.gather(cdf, -1, below), torch.gather(cdf, -1, above)
    z_b, z_a = torch.gather(z, -1, below), torch.gather(z, -1, above)
    denom = cdf_a - cdf_b
    denom = torch.where(denom < 1e-5, torch.ones_like(denom), denom)
    z_imp = z_b + (u - cdf_b) / denom * (z_a - z_b)
    return torch.sort(torch.cat([z, z_imp], -1), -1).values


def main_lego_c3_fp64(ref_root: str = "/root/reference") -> None:
    """The float64 truth of BASELINE config 3: the same chain as
    ``main_lego_c3`` -- the reference's ``generate_rays`` / ``sample_points_on_rays``
    (base_renderer.py:223-281), its coarse and fine ``NeRFModel`` (nerf.py:92-131) and
    ``VolumeRenderer.volume_render`` (rendering.py:102-143) with the fixed-gather sampler in
    between -- run with every tensor in float64 (torch's default dtype set to float64, the
    models ``NeRFModel()`` built in float64 and loaded with the fp32 checkpoint's values, the
    pose cast up), for suite view 0 and the off-axis pose: render_lego_800x600_c3_fp64.npz.
    The fp32 fixture (render_lego_800x600_c3_full.npz) and the GPU renders are both measured
    against it in tests/test_gpu_lego_c3.py.  About 25 min a frame on 8 cores."""
    import torch

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    PyTorchCPURenderer, NeRFModel, _, VolumeRenderer = import_reference(ref_root)
    coarse_sd, fine_sd = W.lego_models()
    ckpt_path = os.path.join(tempfile.mkdtemp(prefix="nerf_golden_lego_c3_fp64_"), "lego.pth")
    W.save_checkpoint(ckpt_path, coarse_sd, fine_sd)
    renderer = PyTorchCPURenderer()
    renderer.setup(ckpt_path)
    poses = suite_poses(2) + [off_axis_pose()]
    torch.set_default_dtype(torch.float64)

    def net(sd):
        m = NeRFModel()
        m.load_state_dict({k: torch.from_numpy(v.astype(np.float64)) for k, v in sd.items()})
        assert all(p.dtype == torch.float64 for p in m.parameters())
        return m.eval()

    coarse, fine = net(coarse_sd), net(fine_sd)
    vr = VolumeRenderer("cpu")
    pose_ids = [0, 2]
    w_, h_, nc, ni, chunk = 800, 600, 64, 128, 4096
    out = {"poses": np.stack([poses[i].numpy() for i in pose_ids]), "pose_ids": np.array(pose_ids, dtype=np.int32),
           "W": np.int32(w_), "H": np.int32(h_), "S_coarse": np.int32(nc), "S_importance": np.int32(ni)}
    timing = {}
    with torch.no_grad():
        for k, pi in enumerate(pose_ids):
            t0 = time.time()
            ro, rd = renderer.generate_rays(poses[pi].double(), w_, h_)
            assert ro.dtype == torch.float64 and rd.dtype == torch.float64
            ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
            rgbs, depths = [], []
            for c in range(0, ro.shape[0], chunk):
                o, d = ro[c:c + chunk], rd[c:c + chunk]
                m = o.shape[0]
                pts, zc = renderer.sample_points_on_rays(o, d, nc)
                sig, col = coarse(pts.reshape(-1, 3), d[:, None, :].expand(m, nc, 3).reshape(-1, 3))
                _, _, _, wts = vr.volume_render(sig.reshape(m, nc, 1), col.reshape(m, nc, 3), zc, d)
                u = torch.linspace(0.0, 1.0, ni).expand(m, ni)
                zf = _fine_z_f64(zc.contiguous(), wts, u)
                pts = o[..., None, :] + d[..., None, :] * zf[..., :, None]
                sig, col = fine(pts.reshape(-1, 3), d[:, None, :].expand(m, nc + ni, 3).reshape(-1, 3))
                rgb, depth, _, _ = vr.volume_render(sig.reshape(m, -1, 1), col.reshape(m, -1, 3), zf, d)
                assert rgb.dtype == torch.float64
                rgbs.append(rgb)
                depths.append(depth)
                if c % (chunk * 20) == 0:
                    print(f"view {pi}: ray {c} of {ro.shape[0]}, {time.time() - t0:.0f} s", flush=True)
            out[f"rgb_{k}"] = torch.cat(rgbs).reshape(h_, w_, 3).numpy()
            out[f"depth_{k}"] = torch.cat(depths).reshape(h_, w_).numpy()
            timing[f"800x600_c3_64+128_fp64_view{pi}"] = time.time() - t0
            print(f"view {pi}: {timing[f'800x600_c3_64+128_fp64_view{pi}']:.1f} s", flush=True)
    torch.set_default_dtype(torch.float32)
    np.savez_compressed(os.path.join(HERE, "render_lego_800x600_c3_fp64.npz"), **out)
    meta_path = os.path.join(HERE, "golden_lego_meta.json")
    with open(meta_path) as f:
        meta = json.load(f)
    meta.setdefault("render_seconds", {}).update(timing)
    meta["c3_full_frame_fp64"] = {
        "fine_digest": W.state_dict_digest(fine_sd), "coarse_digest": W.state_dict_digest(coarse_sd),
        "chain": "the c3_full_frame chain with torch's default dtype float64: reference generate_rays/"
                 "sample_points_on_rays/NeRFModel (float64 parameters)/volume_render, float64 fixed-gather sampler"}
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    if "--lego-c3-fp64" in sys.argv:
        main_lego_c3_fp64(args[0] if args else "/root/reference")
    elif "--lego-c3" in sys.argv:
        main_lego_c3(args[0] if args else "/root/reference")
    elif "--lego-full" in sys.argv:
        main_lego_full(args[0] if args else "/root/reference")
    elif "--lego" in sys.argv:
        main_lego(args[0] if args else "/root/reference")
    else:
        main(args[0] if args else "/root/reference")
