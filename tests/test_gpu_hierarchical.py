"""GPU parity of the hierarchical (64+128) render's hand-offs, end to end.

The reference's importance sampler crashes, so the hierarchical mode
is build-defined and the oracle's restatement is its checker.
Stage-wise parity (each stage fed the oracle's inputs) is in test_gpu_parity.py.
Here the GPU's *own* intermediate results are carried forward, so that the
whole chain inside one ``nerf_render`` is checked at the parity gate:

  * fp32: the GPU's coarse weights -> the oracle's importance sampler (must give
    the render's fine samples bit for bit, read back with nerf_ctx_last_fine_z)
    -> the oracle's fine pass -> RGB/depth within 1e-4 of the GPU's render;
  * bf16 / fp8 with the coarse pass composited in the MLP epilogue (the
    default): its fine samples against the sequential composite's (same MLP
    outputs), and the render's fine pass against the GPU fine MLP's samples
    composited by the oracle on those fine samples.
"""
import os

import numpy as np
import pytest
import torch

from nerf_amd import runtime as rt
from nerf_amd import weights as W

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TOL_RENDER = 1e-4


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    p = tmp_path_factory.mktemp("ckpt_h") / "synthetic.pth"
    return W.write_synthetic_checkpoint(str(p), seed=0)


def _pose(i):
    return torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][i])


def _last_fine_z(r, n_rays, per_ray):
    z = torch.empty(n_rays, per_ray, dtype=torch.float32, device="cuda")
    r.hip.last_fine_z(n_rays, per_ray, z)
    torch.cuda.synchronize()
    return z.cpu()


def maxabs(a, b):
    a = a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)
    b = b.detach().cpu().numpy() if hasattr(b, "detach") else np.asarray(b)
    return float(np.abs(a - b).max()) if a.size else 0.0


@pytest.mark.parametrize("res,nc,pose_id", [((40, 30), 64, 0), ((37, 23), 64, 2), ((24, 16), 128, 1)])
def test_hierarchical_fp32_end_to_end_at_gate(ckpt, res, nc, pose_id):
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer
    from oracle import nerf_oracle as O

    ni = 128
    r = MI355XRenderer("fp32", n_importance=ni)
    r.setup(ckpt)
    c, f = W.synthetic_models(0)
    pose = _pose(pose_id)
    w, h = res
    rgb, depth = [t.clone() for t in r.render_image(pose, res, nc)]
    zf_render = _last_fine_z(r, w * h, nc + ni)
    o, d = O.generate_rays(pose, w, h)
    o, d = o.reshape(-1, 3), d.reshape(-1, 3)
    n = o.shape[0]
    zc = O.uniform_z(nc).expand(n, nc).contiguous()
    # the GPU's coarse weights (same f32 MLP + composite kernels as the render's coarse pass)
    _, _, _, w_gpu = r.render_rays_z(o, d, zc, use_fine=False, with_weights=True)
    zf = O.fine_z(zc, w_gpu.cpu(), O.default_u(n, ni))
    assert torch.equal(zf, zf_render), "the render's fine samples are the oracle sampler's on the GPU weights"
    # the oracle's fine pass on them
    pts = O.sample_points(o, d, zf)
    s_, c_ = O.nerf_forward(O.Net(f), pts.reshape(-1, 3), d[:, None].expand_as(pts).reshape(-1, 3))
    rgb_ref, dep_ref = O.composite(s_.reshape(n, -1, 1), c_.reshape(n, -1, 3), zf, d)
    er, ed = maxabs(rgb.reshape(-1, 3), rgb_ref), maxabs(depth.reshape(-1), dep_ref)
    print(f"hierarchical fp32 {res} {nc}+{ni} (GPU coarse weights -> oracle): rgb {er:.2e} depth {ed:.2e}")
    assert er < TOL_RENDER and ed < TOL_RENDER


@pytest.mark.parametrize("precision", ["bf16", "fp8"])
@pytest.mark.parametrize("res,nc", [((40, 30), 64), ((37, 23), 64), ((19, 7), 128)])
def test_hierarchical_fused_coarse_handoff(ckpt, precision, res, nc):
    """NERF_OPT_FUSED_COMPOSITE bit 2 (default): the coarse weights come from the MLP
    epilogue (in-segment weight x the earlier segments' transmittance) instead of
    the sequential composite.  Same network outputs, regrouped sums: the fine
    samples agree at fp32 rounding level with the sequential path's, which is
    itself the GPU sampler on the GPU's sequential weights, bit for bit."""
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer
    from oracle import nerf_oracle as O

    ni = 128
    r = MI355XRenderer(precision, n_importance=ni)
    r.setup(ckpt)
    pose = _pose(2)
    w, h = res
    n, nf = w * h, nc + ni
    rgb_fused, dep_fused = [t.clone() for t in r.render_image(pose, res, nc)]     # default: both passes fused
    zf_fused = _last_fine_z(r, n, nf)
    r.hip.set_fused_composite(True, coarse=False)                                  # coarse pass sequential
    try:
        r.render_image(pose, res, nc)
        zf_seq = _last_fine_z(r, n, nf)
    finally:
        r.hip.set_fused_composite(True, coarse=True)
    # the sequential coarse path, piece by piece on the GPU: coarse MLP samples,
    # composite with weights, sampler
    o, d = O.generate_rays(pose, w, h)
    o, d = o.reshape(-1, 3).contiguous(), d.reshape(-1, 3).contiguous()
    zc = O.uniform_z(nc).expand(n, nc).contiguous()
    _, _, _, w_seq = r.render_rays_z(o, d, zc, use_fine=False, with_weights=True)
    zf_ind = r.importance_sample(zc, w_seq, torch.linspace(0, 1, ni)).cpu()
    assert torch.equal(zf_seq, zf_ind)
    # the sampler's outputs (z in [2, 6]): the two weight forms differ at fp32
    # rounding level, which moves a fine sample by ~1e-7 -- except where a bin's
    # pdf sits at the sampler's denom < 1e-5 switch (rendering.py:86, weights ~0:
    # pdf = 1e-5 / sum), where a rounding-level change of the weight moves the
    # sample within its bin; so the fraction of exact / close samples is asserted
    dz = (zf_fused - zf_seq).abs()
    fe, f6, f5 = float((dz == 0).float().mean()), float((dz <= 1e-6).float().mean()), float((dz <= 1e-5).float().mean())
    print(f"{precision} {res} {nc}+{ni}: fused-coarse vs sequential fine z: exact {fe:.4f}, <= 1e-6 {f6:.4f}, "
          f"<= 1e-5 {f5:.4f}, max {float(dz.max()):.2e}")
    assert f6 >= 0.99 and f5 >= 0.995 and float(dz.max()) < 0.07
    # the fine pass of the (default, fused) render: GPU fine-MLP samples on the
    # render's own fine z, composited by the oracle, against the render's image
    out = torch.empty(n * nf, 4, dtype=torch.float32, device="cuda")
    r.hip.mlp_forward(rt.NERF_NET_FINE, rt.PRECISIONS[precision], o.cuda(), d.cuda(), zf_fused.cuda(), nf, n, nf, out)
    torch.cuda.synchronize()
    out = out.cpu()
    rgb_ref, dep_ref = O.composite(out[:, :1].reshape(n, nf, 1), out[:, 1:].reshape(n, nf, 3), zf_fused, d)
    er, ed = maxabs(rgb_fused.reshape(-1, 3), rgb_ref), maxabs(dep_fused.reshape(-1), dep_ref)
    print(f"{precision} {res} {nc}+{ni}: render vs oracle composite of its fine samples: rgb {er:.2e} depth {ed:.2e}")
    assert er < 1e-5 and ed < 1e-4


def test_last_fine_z_cleared_by_a_render_without_importance(ckpt):
    """A render with n_importance = 0 may reuse the z buffer where the last fine z lived
    (the stratified first-pass z shares it), so nerf_ctx_last_fine_z refuses afterwards
    instead of returning overwritten depths; a copy on another stream is ordered after
    the render that wrote the samples."""
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    r = MI355XRenderer("fp32", n_importance=32)
    r.setup(ckpt)
    pose = _pose(0)
    r.render_image(pose, (16, 8), 32)
    side = torch.cuda.Stream()
    z = torch.empty(16 * 8, 64, dtype=torch.float32, device="cuda")
    r.hip.last_fine_z(16 * 8, 64, z, stream=side)
    side.synchronize()
    assert bool((z[:, 1:] >= z[:, :-1]).all()) and float(z.min()) >= 2.0 and float(z.max()) <= 6.0
    r.n_importance = 0
    r.render_image(pose, (16, 8), 32)
    with pytest.raises(RuntimeError):
        r.hip.last_fine_z(16 * 8, 64, z)
