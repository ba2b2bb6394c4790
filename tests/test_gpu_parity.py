"""GPU parity: the HIP path (through the C ABI) against the reference's golden
vectors and the oracle, on the same inputs.

Tolerances (written here, per SURVEY §8 and BASELINE.json's north star):
  * rays / z tables: bit-exact;
  * fp32 path: RGB and depth max-abs < 1e-4 vs the reference PyTorch-CPU renderer
    (TOL_RENDER); network outputs and compositing to fp32 rounding;
  * bf16 path: error vs fp32 reported, bounded loosely (bf16 has 8 mantissa bits);
  * hierarchical sampler: bit-exact against the oracle on identical inputs.
"""
import os

import numpy as np
import pytest
import torch

from nerf_amd import weights as W

pytestmark = pytest.mark.gpu

TOL_RENDER = 1e-4
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    p = tmp_path_factory.mktemp("ckpt") / "synthetic.pth"
    return W.write_synthetic_checkpoint(str(p), seed=0)


@pytest.fixture(scope="module")
def r32(ckpt):
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    r = MI355XRenderer("fp32")
    r.setup(ckpt)
    return r


@pytest.fixture(scope="module")
def r16(ckpt):
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    r = MI355XRenderer("bf16")
    r.setup(ckpt)
    return r


def maxabs(a, b):
    a = a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)
    return float(np.abs(a - np.asarray(b)).max()) if a.size else 0.0


def test_native_library_is_what_runs(r32):
    import nerf_amd.runtime as rt

    assert rt._lib is not None and os.path.exists(rt.library_path())
    assert "gfx950" in r32.get_device_info()


def test_rays_bit_exact(r32, golden):
    g = golden("rays")
    for k in [k for k in g.files if k.startswith("o_")]:
        tag = k[2:]
        w, h = map(int, tag.split("_")[0].split("x"))
        o, d = r32.generate_rays(torch.from_numpy(g["poses"][int(tag.split("_")[1])]), w, h)
        assert np.array_equal(o.cpu().numpy(), g[k]), tag
        assert np.array_equal(d.cpu().numpy(), g["d_" + tag]), tag


@pytest.mark.parametrize("precision,tol_s,tol_c", [("fp32", 2e-4, 2e-5), ("bf16", 0.5, 0.05)])
def test_query_networks(request, golden, precision, tol_s, tol_c):
    r = request.getfixturevalue("r32" if precision == "fp32" else "r16")
    g = golden("mlp")
    pos, dirs = torch.from_numpy(g["pos"]), torch.from_numpy(g["dirs"])
    for use_fine, tag in ((True, "fine"), (False, "coarse")):
        s, c = r.query_nerf_networks(pos, dirs, use_fine=use_fine)
        es, ec = maxabs(s, g[f"sigma_{tag}"]), maxabs(c, g[f"rgb_{tag}"])
        print(f"{precision} {tag}: sigma err {es:.3e} rgb err {ec:.3e}")
        assert es < tol_s and ec < tol_c


@pytest.mark.parametrize("case", ["rand16", "rand32", "rand64", "rand128", "edge64"])
def test_composite(r32, golden, case):
    g = golden("composite")
    rgb, depth, acc, w = r32.execute_volume_rendering(
        torch.from_numpy(g[f"{case}_sigma"]), torch.from_numpy(g[f"{case}_rgb_in"]),
        torch.from_numpy(g[f"{case}_z"]), torch.from_numpy(g[f"{case}_d"]), with_weights=True)
    assert maxabs(rgb, g[f"{case}_rgb"]) < 2e-6
    assert maxabs(depth, g[f"{case}_depth"]) < 1e-5
    assert maxabs(acc, g[f"{case}_acc"]) < 2e-6
    assert maxabs(w, g[f"{case}_weights"]) < 2e-6


@pytest.mark.parametrize("name", ["render_64x48_s16", "render_37x23_s7", "render_200x150_s32", "render_400x300_s64"])
def test_render_fp32_vs_reference(r32, golden, name):
    g = golden(name)
    w, h, s = int(g["W"]), int(g["H"]), int(g["S"])
    for k in range(len(g["pose_ids"])):
        rgb, depth = r32.render_image(torch.from_numpy(g["poses"][k]), (w, h), s)
        assert tuple(rgb.shape) == (h, w, 3) and tuple(depth.shape) == (h, w)
        er, ed = maxabs(rgb, g[f"rgb_{k}"]), maxabs(depth, g[f"depth_{k}"])
        print(f"{name} view {k}: rgb {er:.3e} depth {ed:.3e}")
        assert er < TOL_RENDER and ed < TOL_RENDER


def test_render_fp32_headline_band(r32, golden):
    g = golden("render_800x600_s128_band")
    r0, r1 = map(int, g["rows"])
    for k in range(2):
        rgb, depth = r32.render_rows(torch.from_numpy(g["poses"][k]), (800, 600), 128, r0, r1)
        er, ed = maxabs(rgb, g[f"rgb_{k}"]), maxabs(depth, g[f"depth_{k}"])
        print(f"800x600x128 band view {k}: rgb {er:.3e} depth {ed:.3e}")
        assert er < TOL_RENDER and ed < TOL_RENDER


def test_render_bf16_error_bounded(r16, golden):
    g = golden("render_200x150_s32")
    for k in range(len(g["pose_ids"])):
        rgb, depth = r16.render_image(torch.from_numpy(g["poses"][k]), (200, 150), 32)
        er, ed = maxabs(rgb, g[f"rgb_{k}"]), maxabs(depth, g[f"depth_{k}"])
        print(f"bf16 200x150x32 view {k}: rgb {er:.3e} depth {ed:.3e}")
        # measured (round 3): rgb 1.6-2.2e-3, depth 4.7-8.7e-3 -- the per-sample kernel is
        # pinned to its MFMA-order restatement in test_gpu_restated.py; this bounds the image
        assert er < 5e-3 and ed < 2.5e-2


def test_importance_sampler_matches_oracle(r32):
    from oracle import nerf_oracle as O

    torch.manual_seed(3)
    n, s, ni = 300, 64, 128
    z = O.uniform_z(s).expand(n, s).contiguous()
    w = torch.rand(n, s) ** 3
    w[5] = 0.0                                   # all-transparent ray
    w[6, 10] = 1.0
    w[6, :10] = 0.0
    for u in (O.default_u(n, ni), torch.sort(torch.rand(n, ni), -1).values):
        ref = O.fine_z(z, w, u)
        got = r32.importance_sample(z, w, u.contiguous())
        assert np.array_equal(got.cpu().numpy(), ref.numpy())


def test_hierarchical_stage_by_stage(r32):
    """64+128-style pipeline checked stage by stage against the oracle, each stage fed
    the oracle's inputs: coarse weights, importance samples (bit-exact), fine image."""
    from oracle import nerf_oracle as O

    c, f = W.synthetic_models(0)
    coarse, fine = O.Net(c), O.Net(f)
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][2])
    o, d = O.generate_rays(pose, 48, 20)
    o, d = o.reshape(-1, 3), d.reshape(-1, 3)
    n, nc, ni = o.shape[0], 64, 128
    zc = O.uniform_z(nc).expand(n, nc).contiguous()
    # coarse pass -> weights
    pts = O.sample_points(o, d, zc)
    s_, c_ = O.nerf_forward(coarse, pts.reshape(-1, 3), d[:, None].expand_as(pts).reshape(-1, 3))
    _, _, _, w_ref = O.composite(s_.reshape(n, nc, 1), c_.reshape(n, nc, 3), zc, d, True)
    _, _, _, w_gpu = r32.render_rays_z(o, d, zc, use_fine=False, with_weights=True)
    ew = maxabs(w_gpu, w_ref.numpy())
    # importance samples from the oracle's weights: bit-exact
    u = O.default_u(n, ni)
    zf_ref = O.fine_z(zc, w_ref, u)
    zf_gpu = r32.importance_sample(zc, w_ref, u.contiguous())
    assert np.array_equal(zf_gpu.cpu().numpy(), zf_ref.numpy())
    # fine pass on the oracle's fine samples
    pts = O.sample_points(o, d, zf_ref)
    s_, c_ = O.nerf_forward(fine, pts.reshape(-1, 3), d[:, None].expand_as(pts).reshape(-1, 3))
    rgb_ref, dep_ref = O.composite(s_.reshape(n, -1, 1), c_.reshape(n, -1, 3), zf_ref, d)
    rgb_gpu, dep_gpu = r32.render_rays_z(o, d, zf_ref)
    er, ed = maxabs(rgb_gpu, rgb_ref.numpy()), maxabs(dep_gpu, dep_ref.numpy())
    print(f"hierarchical stages: coarse weights {ew:.2e}, fine rgb {er:.2e} depth {ed:.2e}")
    assert ew < 1e-4 and er < TOL_RENDER and ed < TOL_RENDER


def test_render_hierarchical_end_to_end(ckpt):
    """Whole 64+128 render at the parity gate: the fine samples are placed by the coarse
    net's weights, so the chain is checked with the GPU's own coarse weights carried
    forward (fp32 summation order moves a fine z by ~1e-6, amplified by the 2^9*pi
    encoding): oracle sampler on them == the render's fine z (bit for bit), then the
    oracle's fine pass on those samples within 1e-4 of the render."""
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer
    from oracle import nerf_oracle as O

    r = MI355XRenderer("fp32", n_importance=128)
    r.setup(ckpt)
    c, f = W.synthetic_models(0)
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][0])
    w, h, nc, ni = 40, 30, 64, 128
    rgb, depth = [t.clone() for t in r.render_image(pose, (w, h), nc)]
    zf_render = torch.empty(w * h, nc + ni, dtype=torch.float32, device="cuda")
    r.hip.last_fine_z(w * h, nc + ni, zf_render)
    o, d = O.generate_rays(pose, w, h)
    o, d = o.reshape(-1, 3), d.reshape(-1, 3)
    zc = O.uniform_z(nc).expand(w * h, nc).contiguous()
    _, _, _, w_gpu = r.render_rays_z(o, d, zc, use_fine=False, with_weights=True)
    zf = O.fine_z(zc, w_gpu.cpu(), O.default_u(w * h, ni))
    assert torch.equal(zf, zf_render.cpu())
    pts = O.sample_points(o, d, zf)
    s_, c_ = O.nerf_forward(O.Net(f), pts.reshape(-1, 3), d[:, None].expand_as(pts).reshape(-1, 3))
    ref_rgb, ref_depth = O.composite(s_.reshape(w * h, -1, 1), c_.reshape(w * h, -1, 3), zf, d)
    er, ed = maxabs(rgb.reshape(-1, 3), ref_rgb.numpy()), maxabs(depth.reshape(-1), ref_depth.numpy())
    print(f"hierarchical end-to-end 40x30 64+128: rgb {er:.3e} depth {ed:.3e}")
    assert er < TOL_RENDER and ed < TOL_RENDER


def test_headline_full_size_properties(r16):
    """800x600x128 bf16 (the benchmark config): finite, in range, deterministic."""
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer  # noqa: F401

    pose = torch.eye(4)
    pose[2, 3] = 4.0
    rgb1, d1 = r16.render_image(pose, (800, 600), 128)
    rgb2, d2 = r16.render_image(pose, (800, 600), 128)
    assert torch.isfinite(rgb1).all() and torch.isfinite(d1).all()
    assert float(rgb1.min()) >= 0.0 and float(rgb1.max()) <= 1.0
    assert float(d1.min()) >= 0.0 and float(d1.max()) <= 6.0
    assert torch.equal(rgb1, rgb2) and torch.equal(d1, d2)


@pytest.mark.parametrize("res,s", [((1, 1), 1), ((7, 3), 2), ((16, 16), 1), ((33, 9), 100)])
def test_edge_shapes_vs_oracle(r32, ckpt, res, s):
    from oracle import nerf_oracle as O

    c, f = W.synthetic_models(0)
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][2])
    rgb, depth = r32.render_image(pose, res, s)
    ref_rgb, ref_depth = O.render_image(O.Net(f), pose, res, s)
    assert maxabs(rgb, ref_rgb.numpy()) < TOL_RENDER and maxabs(depth, ref_depth.numpy()) < TOL_RENDER


# ------------------------------------------------ stratified sampling (a2s) --
def test_sample_points_bit_exact(r32, golden):
    """sample_kernel vs the reference's own VolumeRenderer.sample_points_on_rays
    (perturb=True, captured t_rand) and the benchmark's uniform sampler."""
    from oracle import nerf_oracle as O

    g = golden("stratified")
    o, d = torch.from_numpy(g["rays_o"]), torch.from_numpy(g["rays_d"])
    s = g["t_rand"].shape[1]
    pts, z = r32.sample_points_on_rays(o, d, s, t_rand=torch.from_numpy(g["t_rand"]))
    assert np.array_equal(z.cpu().numpy(), g["z"])
    assert np.array_equal(pts.cpu().numpy(), g["pts"])
    pts, z = r32.sample_points_on_rays(o, d, s)
    z_ref = O.uniform_z(s).expand(o.shape[0], s)
    assert np.array_equal(z.cpu().numpy(), z_ref.numpy())
    assert np.array_equal(pts.cpu().numpy(), O.sample_points(o, d, z_ref).numpy())
    for n_s in (1, 2):                          # degenerate strata
        t = torch.rand(o.shape[0], n_s)
        _, z = r32.sample_points_on_rays(o, d, n_s, t_rand=t)
        assert np.array_equal(z.cpu().numpy(), O.stratified_z(O.uniform_z(n_s), t).numpy())


def test_render_stratified_fp32_vs_oracle(r32):
    from oracle import nerf_oracle as O

    _, f = W.synthetic_models(0)
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][2])
    gen = torch.Generator().manual_seed(0)
    w, h, s = 64, 48, 32
    t_rand = torch.rand(w * h, s, generator=gen)
    rgb, depth = r32.render_rows(pose, (w, h), s, 0, h, t_rand=t_rand)
    ref_rgb, ref_depth = O.render_image(O.Net(f), pose, (w, h), s, t_rand=t_rand)
    er, ed = maxabs(rgb, ref_rgb.numpy()), maxabs(depth, ref_depth.numpy())
    print(f"stratified 64x48x32: rgb {er:.3e} depth {ed:.3e}")
    assert er < TOL_RENDER and ed < TOL_RENDER
    # a row band draws its own rows' t_rand
    rgb_b, _ = r32.render_rows(pose, (w, h), s, 10, 20, t_rand=t_rand[10 * w:20 * w])
    assert torch.equal(rgb_b, rgb[10:20])


def test_render_stratified_hierarchical_stagewise(r32):
    """Stratified coarse samples + per-ray random u: the importance stage is bit-exact
    and the fine image within TOL_RENDER when fed the oracle's coarse weights."""
    from oracle import nerf_oracle as O

    c, _ = W.synthetic_models(0)
    coarse = O.Net(c)
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][2])
    o, d = O.generate_rays(pose, 32, 16)
    o, d = o.reshape(-1, 3), d.reshape(-1, 3)
    n, nc, ni = o.shape[0], 64, 128
    gen = torch.Generator().manual_seed(1)
    t_rand = torch.rand(n, nc, generator=gen)
    u = torch.sort(torch.rand(n, ni, generator=gen), -1).values
    zc = O.stratified_z(O.uniform_z(nc), t_rand)
    _, zc_gpu = r32.sample_points_on_rays(o, d, nc, t_rand=t_rand)
    assert np.array_equal(zc_gpu.cpu().numpy(), zc.numpy())
    pts = O.sample_points(o, d, zc)
    s_, c_ = O.nerf_forward(coarse, pts.reshape(-1, 3), d[:, None].expand_as(pts).reshape(-1, 3))
    _, _, _, w_ref = O.composite(s_.reshape(n, nc, 1), c_.reshape(n, nc, 3), zc, d, True)
    _, _, _, w_gpu = r32.render_rays_z(o, d, zc, use_fine=False, with_weights=True)
    assert maxabs(w_gpu, w_ref.numpy()) < 1e-4
    zf_gpu = r32.importance_sample(zc, w_ref, u.contiguous())
    assert np.array_equal(zf_gpu.cpu().numpy(), O.fine_z(zc, w_ref, u).numpy())


def test_render_stratified_hierarchical_end_to_end(ckpt):
    """Stratified coarse samples (injected t_rand) + per-ray importance draws (injected u):
    the same chain as test_render_hierarchical_end_to_end at the 1e-4 gate."""
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer
    from oracle import nerf_oracle as O

    r = MI355XRenderer("fp32", n_importance=64)
    r.setup(ckpt)
    c, f = W.synthetic_models(0)
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][0])
    w, h, nc, ni = 32, 24, 32, 64
    gen = torch.Generator().manual_seed(2)
    t_rand = torch.rand(w * h, nc, generator=gen)
    u = torch.sort(torch.rand(w * h, ni, generator=gen), -1).values
    rgb, depth = [t.clone() for t in r.render_rows(pose, (w, h), nc, 0, h, t_rand=t_rand, u=u)]
    zf_render = torch.empty(w * h, nc + ni, dtype=torch.float32, device="cuda")
    r.hip.last_fine_z(w * h, nc + ni, zf_render)
    o, d = O.generate_rays(pose, w, h)
    o, d = o.reshape(-1, 3), d.reshape(-1, 3)
    zc = O.stratified_z(O.uniform_z(nc), t_rand).contiguous()
    _, _, _, w_gpu = r.render_rays_z(o, d, zc, use_fine=False, with_weights=True)
    zf = O.fine_z(zc, w_gpu.cpu(), u)
    assert torch.equal(zf, zf_render.cpu())
    pts = O.sample_points(o, d, zf)
    s_, c_ = O.nerf_forward(O.Net(f), pts.reshape(-1, 3), d[:, None].expand_as(pts).reshape(-1, 3))
    ref_rgb, ref_depth = O.composite(s_.reshape(w * h, -1, 1), c_.reshape(w * h, -1, 3), zf, d)
    er, ed = maxabs(rgb.reshape(-1, 3), ref_rgb.numpy()), maxabs(depth.reshape(-1), ref_depth.numpy())
    print(f"stratified hierarchical end-to-end {w}x{h} {nc}+{ni}: rgb {er:.3e} depth {ed:.3e}")
    assert er < TOL_RENDER and ed < TOL_RENDER


# ------------------------------------------------------------ fp8 path (C5) --
@pytest.fixture(scope="module")
def r8(ckpt):
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    r = MI355XRenderer("fp8")
    r.setup(ckpt)
    return r


def test_render_fp8_error_vs_fp32(r8, r32, golden):
    """Config 5: the fp8 image against the fp32 parity path (the reference's own
    compressed renderer is 0.42 RGB max-abs off fp32 on this checkpoint)."""
    g = golden("render_800x600_s128_band")
    pose = torch.from_numpy(g["poses"][0])
    r0, r1 = map(int, g["rows"])
    rgb8, d8 = r8.render_rows(pose, (800, 600), 128, r0, r1)
    rgb32, d32 = r32.render_rows(pose, (800, 600), 128, r0, r1)
    er, ed = maxabs(rgb8, rgb32.cpu().numpy()), maxabs(d8, d32.cpu().numpy())
    mr = float((rgb8 - rgb32).abs().mean())
    print(f"fp8 vs fp32 800x600x128 band: rgb max {er:.3e} mean {mr:.3e}, depth max {ed:.3e}")
    assert torch.isfinite(rgb8).all() and torch.isfinite(d8).all()
    assert er < 5e-2 and mr < 1e-2           # measured (round 3): rgb max 1.4e-2, mean 3.2e-3


def test_fp8_error_below_reference_compressed(r8, r32):
    """Config 5's error baseline: the reference's own compressed (int8, pruned,
    fp16) renderer, restated in the oracle and pinned to its golden vectors.  The
    fp8 path must be closer to fp32 than the reference's compressed path is."""
    from oracle import nerf_oracle as O

    _, f = W.synthetic_models(0)
    pose = torch.eye(4)
    pose[2, 3] = 4.0
    w, h, s = 64, 48, 32
    rgb32, d32 = r32.render_image(pose, (w, h), s)
    rgb8, d8 = r8.render_image(pose, (w, h), s)
    rgbc, dc = O.compressed_render_image(O.compressed_weights(f), pose, (w, h), s)
    e8, ec = maxabs(rgb8, rgb32.cpu().numpy()), maxabs(rgbc, rgb32.cpu().numpy())
    m8 = float((rgb8 - rgb32).abs().mean())
    mc = float((rgbc - rgb32.cpu()).abs().mean())
    print(f"vs fp32 at {w}x{h}x{s}: fp8 rgb max {e8:.3e} mean {m8:.3e}; "
          f"reference int8 compressed rgb max {ec:.3e} mean {mc:.3e}")
    assert e8 < ec and m8 < mc


def test_plain_c_host_matches_python(r32, tmp_path):
    """examples/render_c.c drives the C ABI with no Python in the process; its frame
    equals the Python plugin's bit for bit (same weights, t table and stream order)."""
    import subprocess

    exe = os.path.join(os.path.dirname(GOLDEN), "..", "examples", "render_c")
    assert os.path.exists(exe), "build with `make -C examples` (done by __graft_entry__.build())"
    _, f = W.synthetic_models(0)
    with open(tmp_path / "params.bin", "wb") as fh:
        for name, _, _ in W.LAYER_SPECS:
            for suffix in ("weight", "bias"):
                fh.write(np.ascontiguousarray(f[f"{name}.{suffix}"], np.float32).tobytes())
    w, h, s = 64, 48, 32
    t = torch.linspace(0, 1, s).numpy()
    t.tofile(tmp_path / "t.bin")
    res = subprocess.run([exe, str(tmp_path / "params.bin"), str(w), str(h), str(s), "0", str(tmp_path / "out.bin"),
                          str(tmp_path / "t.bin")], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    out = np.fromfile(tmp_path / "out.bin", np.float32)
    pose = torch.eye(4)
    pose[2, 3] = 4.0
    rgb, depth = r32.render_image(pose, (w, h), s)
    assert np.array_equal(out[: w * h * 3], rgb.cpu().numpy().ravel())
    assert np.array_equal(out[w * h * 3:], depth.cpu().numpy().ravel())


def _torchrun(args, env_extra, timeout=300, nproc=2):
    import socket
    import subprocess
    import sys

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port)] + args
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)


def test_multi_rank_rehearsal_on_one_device():
    """The N>1 path (bands, all-gather, barrier, max-over-ranks timing, one JSON
    line from rank 0) with two ranks sharing this box's one GPU over gloo; the
    driver's multi-GPU bench runs the same code over RCCL."""
    import json as js

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = _torchrun([os.path.join(repo, "tests", "dist_render_check.py")], {"NERF_DIST_BACKEND": "gloo"})
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [js.loads(l) for l in res.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 2 and all(o["world"] == 2 and o["backend"] == "gloo" and o["identical"] for o in lines)
    res = _torchrun([os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--width", "200",
                     "--height", "150", "--spp", "32", "--cpu-seconds", "0", "--no-error-check"],
                    {"NERF_DIST_BACKEND": "gloo"})
    assert res.returncode == 0, res.stderr[-3000:]
    # exactly one JSON line, from rank 0 (gloo's own connection messages aside)
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, res.stdout
    b = js.loads(lines[0])
    assert b["n_gpus"] == 2 and b["value"] > 0 and b["config"]["parallelism"].startswith("row-band x2")
    c4 = b["c4_hierarchical_sharded"]                 # config 4, every rank taking part
    assert c4["n_gpus"] == 2 and c4["rays_per_s"] > 0
    assert b["exchange_ms_per_frame"] > 0 and b["mlp_ms_per_frame_rank_max"] > 0
    t = b["training"]                                 # data-parallel training step, every rank taking part
    assert t["n_gpus"] == 2 and t["rays_per_s"] > 0 and t["parallelism"].startswith("data parallel x2")
    assert t["loss_first_last"][-1] < t["loss_first_last"][0]


@pytest.mark.parametrize("precision", ["bf16", "f16x3"])
def test_rccl_process_group_world1(precision):
    """The nccl branches of nerf_amd.distributed on this one-GPU box: an RCCL process
    group of world size 1 (init_from_env with device_id), the band all-gather, the
    packed-tile gather to the root and the gradient all-reduce, each through RCCL on
    device tensors, the frames bit-identical to a single-call render."""
    import json as js

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = _torchrun([os.path.join(repo, "tests", "dist_render_check.py")],
                    {"NERF_DIST_FORCE_GROUP": "1", "NERF_DIST_BACKEND": "nccl", "NERF_CHECK_PRECISION": precision},
                    nproc=1)
    assert res.returncode == 0, res.stderr[-3000:]
    out = js.loads([l for l in res.stdout.splitlines() if l.startswith("{")][-1])
    assert out["world"] == 1 and out["backend"] == "nccl" and out["identical"] and out["all_reduce_ok"]


def test_bench_single_gpu_json_contract():
    """bench.py at N=1 (reduced frame, bounded CPU sample): one JSON line with the
    driver's keys, a roofline object for the MLP kernel and a cpu_baseline object;
    value = W*H*steps / wall time and roofline.frac = achieved / peak."""
    import json as js
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--steps", "3", "--warmup", "1",
                          "--width", "160", "--height", "120", "--spp", "32", "--cpu-seconds", "0.5",
                          "--no-error-check", "--no-extras"], capture_output=True, text=True, timeout=110)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, res.stdout
    b = js.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in b, k
    assert b["n_gpus"] == 1 and b["steps"] == 3 and b["warmup"] == 1 and b["dtype"] == "bf16"
    assert b["higher_is_better"] is True and b["vs_baseline"] is None and "workload" in b["config"]
    # a step renders both suite views (benchmark_suite.py:188-220): value = W*H / mean view time
    assert b["protocol"]["frames_per_step"] == 2 and b["ms_per_view"] == pytest.approx(b["ms_per_step"] / 2)
    assert b["value"] == pytest.approx(160 * 120 / (b["ms_per_view"] * 1e-3), rel=1e-6)
    rf = b["roofline"]
    assert rf["bound"] == "mfma" and rf["unit"] == "TFLOP/s" and rf["peak"] == 2500.0
    assert 0 < rf["achieved"] and rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"])
    assert rf["flop_per_launch"] == 160 * 120 * 32 * W.FLOPS_PER_SAMPLE
    assert rf["traffic"] is None                      # PMC bytes are quoted for the headline frame only
    cb = b["cpu_baseline"]
    assert cb["kind"] == "port" and cb["unit"] == "rays/s" and cb["value"] > 0 and cb["cores"] >= 1
    t = b["training"]                                 # the training-step leg
    assert t["n_gpus"] == 1 and t["rays_per_s"] == pytest.approx(2048 / (t["ms_per_step"] * 1e-3), rel=1e-6)
    gk = t["gemm_kernels_rank0"]
    for key in ("forward", "backward_data"):
        assert 0 < gk[key]["frac"] < 1 and gk[key]["peak"] == 157.3 and gk[key]["unit"] == "TFLOP/s"
    assert 0 < gk["weight_grad"]["frac"] < 1 and gk["weight_grad"]["peak"] == 8000.0 and gk["weight_grad"]["unit"] == "GB/s"
    assert t["cpu_baseline"]["kind"] == "port" and t["cpu_baseline"]["value"] > 0
    assert t["loss_first_last"][-1] < t["loss_first_last"][0]


# ------------------------------------- compositing fused into the MLP epilogue --
@pytest.mark.parametrize("precision,spp,n_imp", [("bf16", 32, 0), ("bf16", 128, 0), ("bf16", 64, 128),
                                                 ("fp8", 128, 0), ("fp8", 64, 128), ("bf16", 48, 0)])
def test_fused_composite_matches_sequential(ckpt, precision, spp, n_imp):
    """NERF_OPT_FUSED_COMPOSITE: per-32-sample partial integrals chained per ray are
    the sequential composite regrouped, on the same network outputs (fp32 rounding
    level; 1e-5 written here).  spp=48 (not a multiple of 32) keeps the sequential
    kernel, so it must agree bit for bit."""
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    r = MI355XRenderer(precision, n_importance=n_imp)
    r.setup(ckpt)
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][2])
    res = (67, 41)                                  # ragged: the last MLP tile is partial
    r.hip.set_fused_composite(False)
    rgb_s, d_s = [t.clone() for t in r.render_image(pose, res, spp)]
    r.hip.set_fused_composite(True, coarse=False)         # the rendered pass only
    rgb_f, d_f = r.render_image(pose, res, spp)
    er, ed = maxabs(rgb_f, rgb_s.cpu().numpy()), maxabs(d_f, d_s.cpu().numpy())
    print(f"fused vs sequential composite {precision} {spp}+{n_imp}: rgb {er:.2e} depth {ed:.2e}")
    if (spp + n_imp) % 32:
        assert er == 0.0 and ed == 0.0
    else:
        assert er < 1e-5 and ed < 1e-5 * 6.0
    if n_imp:
        # also the coarse pass: its weights move at rounding level, which moves the
        # importance samples slightly (amplified by the 2^9*pi encoding of the fine
        # pass), so the bound is the hierarchical end-to-end one
        r.hip.set_fused_composite(True, coarse=True)
        rgb_c, d_c = r.render_image(pose, res, spp)
        ec, edc = maxabs(rgb_c, rgb_s.cpu().numpy()), maxabs(d_c, d_s.cpu().numpy())
        print(f"  + fused coarse weights: rgb {ec:.2e} depth {edc:.2e}")
        assert ec < 2e-2 and edc < 2e-2


def test_fused_composite_headline_vs_fp32(r16, r32):
    """The benchmark configuration with the fused epilogue stays within the bf16
    error band against the fp32 parity path (which is < 1e-4 vs the reference)."""
    pose = torch.eye(4)
    pose[2, 3] = 4.0
    rgb16, d16 = r16.render_rows(pose, (800, 600), 128, 292, 308)
    rgb32, d32 = r32.render_rows(pose, (800, 600), 128, 292, 308)
    er, ed = maxabs(rgb16, rgb32.cpu().numpy()), maxabs(d16, d32.cpu().numpy())
    print(f"bf16 fused vs fp32, 800x600x128 rows 292-308: rgb {er:.2e} depth {ed:.2e}")
    assert er < 5e-3 and ed < 2e-2


def test_back_to_back_renders_reupload_changed_tables(r16):
    """nerf_render skips re-uploading an unchanged z table / importance draw (no host
    synchronisation between frames); a changed table must still be uploaded."""
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][1])
    a64 = [t.clone() for t in r16.render_image(pose, (40, 30), 64)]
    a96 = [t.clone() for t in r16.render_image(pose, (40, 30), 96)]
    for _ in range(3):                                # queued without waiting in between
        b64 = r16.render_image(pose, (40, 30), 64)
        b96 = r16.render_image(pose, (40, 30), 96)
    torch.cuda.synchronize()
    assert all(torch.equal(x, y) for x, y in zip(a64, b64))
    assert all(torch.equal(x, y) for x, y in zip(a96, b96))
    r16.near = 2.5                                    # same S, different table
    try:
        c64 = r16.render_image(pose, (40, 30), 64)
        assert not torch.equal(c64[1], a64[1])
    finally:
        r16.near = 2.0
    assert all(torch.equal(x, y) for x, y in zip(a64, r16.render_image(pose, (40, 30), 64)))


def test_full_size_band_invariance(r16):
    """800x600x128 bf16 (headline): a row band rendered on its own is
    bit-identical to the same rows of the full frame (rays are independent; the
    multi-GPU split relies on it)."""
    pose = torch.eye(4)
    pose[2, 3] = 4.0
    rgb, depth = r16.render_image(pose, (800, 600), 128)
    brgb, bdep = r16.render_rows(pose, (800, 600), 128, 225, 300)
    assert torch.equal(brgb, rgb[225:300]) and torch.equal(bdep, depth[225:300])


def test_full_size_hierarchical_properties(ckpt):
    """C3 at full size (800x600, 64 coarse + 128 importance, bf16): finite, in
    range, deterministic, and band-invariant."""
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    h = MI355XRenderer("bf16", n_importance=128)
    h.setup(ckpt)
    pose = torch.eye(4)
    pose[2, 3] = 4.0
    rgb, depth = [t.clone() for t in h.render_image(pose, (800, 600), 64)]
    rgb2, depth2 = h.render_image(pose, (800, 600), 64)
    assert torch.equal(rgb, rgb2) and torch.equal(depth, depth2)
    assert torch.isfinite(rgb).all() and torch.isfinite(depth).all()
    assert float(rgb.min()) >= 0.0 and float(rgb.max()) <= 1.0
    assert float(depth.min()) >= 0.0 and float(depth.max()) <= 6.0
    brgb, bdep = h.render_rows(pose, (800, 600), 64, 500, 512)
    assert torch.equal(brgb, rgb[500:512]) and torch.equal(bdep, depth[500:512])


@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp8"])
def test_empty_band_and_single_sample(ckpt, precision):
    """Edge cases the reference's semantics define: an empty row band renders
    nothing (and does not fail); S = 1 renders zeros (pytorch_renderers.py:107-108)."""
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    r = MI355XRenderer(precision)
    r.setup(ckpt)
    pose = torch.eye(4)
    pose[2, 3] = 4.0
    rgb, depth = r.render_rows(pose, (64, 48), 32, 10, 10)
    assert rgb.shape == (0, 64, 3) and depth.shape == (0, 64)
    rgb, depth = r.render_image(pose, (64, 48), 1)
    torch.cuda.synchronize()
    assert float(rgb.abs().max()) == 0.0 and float(depth.abs().max()) == 0.0


def test_repeated_renders_do_not_grow_memory(r16):
    """The reference's memory check (test_system.py:258-287: RSS growth < 500 MB over
    repeated renders), here for host RSS and device memory: the context's scratch is
    allocated once per size and reused, so after a warm-up frame neither grows."""
    import psutil

    pose = torch.eye(4)
    pose[2, 3] = 4.0
    r16.render_image(pose, (800, 600), 128)
    torch.cuda.synchronize()
    rss0 = psutil.Process().memory_info().rss
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(20):
        r16.render_image(pose, (800, 600), 128)
    torch.cuda.synchronize()
    rss_growth = psutil.Process().memory_info().rss - rss0
    dev_growth = free0 - torch.cuda.mem_get_info()[0]
    print(f"20 frames 800x600x128: host RSS +{rss_growth / 2**20:.1f} MiB, device +{dev_growth / 2**20:.1f} MiB")
    assert rss_growth < 500 * 2**20
    assert dev_growth < 64 * 2**20


@pytest.mark.parametrize("s,kind", [(64, "unit"), (7, "unit"), (200, "unit"), (256, "unit"),
                                    (64, "wide"), (200, "wide")])
def test_importance_sampler_exact_paths(r32, s, kind):
    """The sampler's normaliser and cdf are torch-CPU cumsums (sequential double).
    The kernel sums in parallel when that is provably exact (weights in [0, 1], the
    composite's range: kind "unit") and sequentially otherwise (kind "wide": weights
    spanning 1e-30..1e6); both must equal the oracle bit for bit."""
    from oracle import nerf_oracle as O

    torch.manual_seed(11 + s)
    n, ni = 97, 130
    z = torch.sort(torch.rand(n, s) * 4.0 + 2.0, -1).values.contiguous()
    w = torch.rand(n, s) ** 3
    if kind == "wide":
        w = w * torch.pow(10.0, torch.randint(-30, 7, (n, s)).float())
    w[3] = 0.0
    u = torch.sort(torch.rand(n, ni), -1).values.contiguous()
    ref = O.fine_z(z, w, u)
    got = r32.importance_sample(z, w, u)
    assert np.array_equal(got.cpu().numpy(), ref.numpy())


@pytest.mark.parametrize("precision", ["bf16", "fp8"])
@pytest.mark.parametrize("res,s", [((1, 1), 32), ((17, 5), 64), ((33, 9), 100), ((7, 3), 2)])
def test_ragged_shapes_reduced_precision(ckpt, r32, precision, res, s):
    """Partial 256-sample tiles and partial 32-sample segments on the bf16 / fp8
    MLPs (fused compositing when S % 32 == 0, the sequential path otherwise),
    against the fp32 parity path on the same pose, bounded at about three times the
    measured error of each path."""
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    r = MI355XRenderer(precision)
    r.setup(ckpt)
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][2])
    rgb, depth = r.render_image(pose, res, s)
    rgb32, d32 = r32.render_image(pose, res, s)
    assert rgb.shape == (res[1], res[0], 3) and depth.shape == (res[1], res[0])
    assert torch.isfinite(rgb).all() and torch.isfinite(depth).all()
    er, ed = maxabs(rgb, rgb32.cpu().numpy()), maxabs(depth, d32.cpu().numpy())
    mr = float((rgb.cpu() - rgb32.cpu()).abs().mean())
    print(f"{precision} {res}x{s}: rgb max {er:.3e} mean {mr:.3e}, depth max {ed:.3e}")
    # measured (round 3): bf16 rgb <= 1.4e-3, depth <= 1.7e-3; fp8 rgb <= 1.4e-2, depth <= 2.9e-2
    tol_rgb, tol_depth, tol_mean = (5e-3, 1e-2, 1e-3) if precision == "bf16" else (5e-2, 0.1, 1.5e-2)
    assert er < tol_rgb and ed < tol_depth and mr < tol_mean


@pytest.mark.parametrize("precision,spp,n_imp", [("fp32", 32, 0), ("bf16", 128, 0), ("bf16", 64, 128),
                                                 ("fp8", 64, 0), ("bf16", 48, 0), ("f16x3", 128, 0),
                                                 ("bf16x3", 64, 64), ("f16x3", 48, 0)])
def test_render_band_packed_matches_render_rows(ckpt, precision, spp, n_imp):
    """nerf_render_band (the multi-GPU path's packed [rows, W, 4] tile) holds exactly
    render_rows' rgb and depth, for fused and sequential compositing and the
    hierarchical mode; a second band into a larger tile leaves its tail alone."""
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    r = MI355XRenderer(precision, n_importance=n_imp)
    r.setup(ckpt)
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][2])
    res, r0, r1 = (53, 40), 7, 31
    rgb, depth = [t.clone() for t in r.render_rows(pose, res, spp, r0, r1)]
    tile = torch.full((r1 - r0 + 2, res[0], 4), -7.0, device="cuda")
    r.render_band(pose, res, spp, r0, r1, tile)
    torch.cuda.synchronize()
    assert torch.equal(tile[: r1 - r0, :, :3], rgb) and torch.equal(tile[: r1 - r0, :, 3], depth)
    assert bool((tile[r1 - r0:] == -7.0).all())


def test_cli_benchmark_only_on_gpu(tmp_path):
    """main.py --benchmark_only (the reference CLI's benchmark mode, main.py:112-262)
    on a small grid: the CSV with the reference's columns (benchmark_suite.py:244-255),
    sample renders per renderer and the performance plot."""
    import subprocess
    import sys

    import pandas as pd

    from nerf_amd.benchmark.benchmark_suite import CSV_COLUMNS

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "out"
    res = subprocess.run([sys.executable, os.path.join(repo, "nerf-dbr_amd", "main.py"), "--benchmark_only",
                          "--synthetic-checkpoint", "--checkpoint", str(tmp_path / "ckpt.pth"),
                          "--resolutions", "64x48,100x75", "--spp", "16,32", "--views", "2",
                          "--precisions", "fp32,bf16,fp8", "--hierarchical", "64", "--output_dir", str(out)],
                         capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    df = pd.read_csv(out / "benchmark_results.csv")
    assert list(df.columns) == CSV_COLUMNS
    assert len(df) == 4 * 2 * 2                                      # 4 renderers x 2 resolutions x 2 spp
    assert set(df["Resolution"]) == {"64x48", "100x75"} and set(df["Samples/Ray"]) == {16, 32}
    assert (df["Rays/Second"] > 0).all()
    for _, row in df.iterrows():
        w, h = map(int, row["Resolution"].split("x"))
        assert row["Rays/Second"] == pytest.approx(w * h / row["Render Time (s)"], rel=1e-6)
        assert "gfx950" in row["Device Info"]
    for name in df["Method"].unique():
        d = out / "sample_renders" / name.replace(" ", "_")
        for v in (0, 1):
            assert (d / f"view_{v}_rgb.png").exists() and (d / f"view_{v}_depth.png").exists()
    assert (out / "performance_comparison.png").exists()
