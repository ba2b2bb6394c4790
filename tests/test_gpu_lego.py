"""GPU parity on the Lego checkpoint (every BASELINE config says "Lego").

The checkpoint is the reference's bundled original-NeRF Lego networks distilled into
NeRFModel's layout (nerf_amd/checkpoints/lego_distilled.npz, tools/lego/distill.py);
the fixtures are the reference's own PyTorchCPURenderer on it
(tests/golden/make_golden.py --lego).  Tolerances, per the north star:
  * fp32 and the split-fp16 parity path (f16x3): RGB and depth max-abs < 1e-4 on
    every Lego image, the 800x600x128 headline band and the 64+128 hierarchical chain;
  * split-bf16 (bf16x3): within the gate on the synthetic checkpoint, but NOT on Lego
    (measured depth 1.3e-4 - 3.2e-4: the distilled net's high-frequency trunk
    amplifies bf16x3's 2^-17 rounding); its error is measured and bounded at 5e-4;
  * bf16 / fp8 (the throughput paths): error against the fp32 path measured on real
    content and bounded loosely (they are not parity paths).
"""
import os

import numpy as np
import pytest
import torch

from nerf_amd import weights as W

pytestmark = pytest.mark.gpu

TOL_RENDER = 1e-4
GATE = ["fp32", "f16x3"]          # the paths held to the 1e-4 gate on real content
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    return W.write_lego_checkpoint(str(tmp_path_factory.mktemp("ckpt_lego") / "lego.pth"))


_R = {}


def renderer(ckpt, precision, n_importance=0):
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    key = (precision, n_importance)
    if key not in _R:
        r = MI355XRenderer(precision, n_importance=n_importance)
        r.setup(ckpt)
        _R[key] = r
    return _R[key]


def maxabs(a, b):
    a = a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)
    b = b.detach().cpu().numpy() if hasattr(b, "detach") else np.asarray(b)
    return float(np.abs(a - b).max()) if a.size else 0.0


def test_lego_fixture_is_this_checkpoint():
    import json

    meta = json.load(open(os.path.join(GOLDEN, "golden_lego_meta.json")))
    c, f = W.lego_models()
    assert meta["fine_digest"] == W.state_dict_digest(f) and meta["coarse_digest"] == W.state_dict_digest(c)


@pytest.mark.parametrize("precision", GATE)
def test_lego_query_networks(ckpt, golden, precision):
    g = golden("lego_mlp")
    r = renderer(ckpt, precision)
    pos, dirs = torch.from_numpy(g["pos"]), torch.from_numpy(g["dirs"])
    for use_fine, tag in ((True, "fine"), (False, "coarse")):
        s, c = r.query_nerf_networks(pos, dirs, use_fine=use_fine)
        ref_s = g[f"sigma_{tag}"]
        es = float(np.abs(s.cpu().numpy() - ref_s).max() / max(1.0, np.abs(ref_s).max()))
        ec = maxabs(c, g[f"rgb_{tag}"])
        print(f"lego {precision} {tag}: sigma rel err {es:.3e} rgb err {ec:.3e}")
        tol = 1e-5 if precision == "fp32" else 1e-4
        assert es < tol and ec < tol


@pytest.mark.parametrize("precision", GATE)
@pytest.mark.parametrize("name", ["render_lego_200x150_s32", "render_lego_400x300_s64"])
def test_lego_render_vs_reference(ckpt, golden, precision, name):
    g = golden(name)
    w, h, s = int(g["W"]), int(g["H"]), int(g["S"])
    r = renderer(ckpt, precision)
    for k in range(len(g["pose_ids"])):
        rgb, depth = r.render_image(torch.from_numpy(g["poses"][k]), (w, h), s)
        er, ed = maxabs(rgb, g[f"rgb_{k}"]), maxabs(depth, g[f"depth_{k}"])
        print(f"lego {precision} {name} view {int(g['pose_ids'][k])}: rgb {er:.3e} depth {ed:.3e}")
        assert er < TOL_RENDER and ed < TOL_RENDER


@pytest.mark.parametrize("precision", GATE)
def test_lego_headline_band_vs_reference(ckpt, golden, precision):
    g = golden("render_lego_800x600_s128_band")
    r0, r1 = map(int, g["rows"])
    r = renderer(ckpt, precision)
    for k in range(2):
        rgb, depth = r.render_rows(torch.from_numpy(g["poses"][k]), (800, 600), 128, r0, r1)
        er, ed = maxabs(rgb, g[f"rgb_{k}"]), maxabs(depth, g[f"depth_{k}"])
        print(f"lego {precision} 800x600x128 band view {k}: rgb {er:.3e} depth {ed:.3e}")
        assert er < TOL_RENDER and ed < TOL_RENDER


@pytest.mark.parametrize("precision", GATE)
def test_lego_hierarchical_chain_at_gate(ckpt, precision):
    """64+128 on Lego: the GPU's coarse weights -> the oracle's sampler (== the render's
    fine z, bit for bit) -> the oracle's fine pass on those samples, within 1e-4 of the
    render (the hierarchical mode is build-defined)."""
    from oracle import nerf_oracle as O

    ni, nc = 128, 64
    r = renderer(ckpt, precision, n_importance=ni)
    c, f = W.lego_models()
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][2])
    w, h = 40, 30
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
    ref_rgb, ref_dep = O.composite(s_.reshape(w * h, -1, 1), c_.reshape(w * h, -1, 3), zf, d)
    er, ed = maxabs(rgb.reshape(-1, 3), ref_rgb), maxabs(depth.reshape(-1), ref_dep)
    print(f"lego {precision} hierarchical 40x30 64+128 chain: rgb {er:.3e} depth {ed:.3e}")
    assert er < TOL_RENDER and ed < TOL_RENDER


def test_lego_bf16x3_error_measured(ckpt, golden):
    """bf16x3 on real content: reported against the reference, bounded above the gate
    (why f16x3 is the parity-grade fast path; tools/precision_lab.py emulates both).
    Only RGB is bounded: depth can jump by up to `far` on a ray whose last sample's
    sigma is ~0 in fp32, where the reference's 1e10 last distance turns a rounding-
    level sigma into alpha ~1 (measured 5.97 on one 400x300 pixel, RGB there < 1e-4)."""
    worst = 0.0
    r = renderer(ckpt, "bf16x3")
    for name in ("render_lego_200x150_s32", "render_lego_400x300_s64"):
        g = golden(name)
        w, h, s = int(g["W"]), int(g["H"]), int(g["S"])
        for k in range(len(g["pose_ids"])):
            rgb, depth = r.render_image(torch.from_numpy(g["poses"][k]), (w, h), s)
            er, ed = maxabs(rgb, g[f"rgb_{k}"]), maxabs(depth, g[f"depth_{k}"])
            print(f"lego bf16x3 {name} view {int(g['pose_ids'][k])}: rgb {er:.3e} depth {ed:.3e}")
            worst = max(worst, er)
    assert worst < 5e-4


@pytest.mark.parametrize("precision,tol_rgb_mean", [("bf16", 8e-3), ("fp8", 6e-2)])
def test_lego_throughput_paths_error_vs_fp32(ckpt, golden, precision, tol_rgb_mean):
    """bf16 / fp8 on real content, against the fp32 parity path on the same frames
    (measured and reported; the loose bounds only catch a broken kernel)."""
    g = golden("render_lego_200x150_s32")
    r, r32 = renderer(ckpt, precision), renderer(ckpt, "fp32")
    for k in range(len(g["pose_ids"])):
        pose = torch.from_numpy(g["poses"][k])
        rgb, depth = r.render_image(pose, (200, 150), 32)
        rgb32, d32 = r32.render_image(pose, (200, 150), 32)
        er, ed = maxabs(rgb, rgb32), maxabs(depth, d32)
        mr = float((rgb - rgb32).abs().mean())
        print(f"lego {precision} 200x150x32 view {int(g['pose_ids'][k])}: rgb max {er:.3e} mean {mr:.3e} "
              f"depth max {ed:.3e}")
        assert torch.isfinite(rgb).all() and mr < tol_rgb_mean and er < 1.0


@pytest.mark.parametrize("precision", GATE)
def test_lego_stratified_hierarchical_chain_at_gate(ckpt, precision):
    """Stratified coarse samples (injected t_rand, rendering.py:42-47) and per-ray
    importance draws (injected u) on Lego: GPU coarse weights -> oracle sampler == the
    render's fine z -> oracle fine pass within 1e-4 of the render."""
    from oracle import nerf_oracle as O

    nc, ni = 32, 64
    r = renderer(ckpt, precision, n_importance=ni)
    _, f = W.lego_models()
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][0])
    w, h = 32, 24
    gen = torch.Generator().manual_seed(5)
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
    ref_rgb, ref_dep = O.composite(s_.reshape(w * h, -1, 1), c_.reshape(w * h, -1, 3), zf, d)
    er, ed = maxabs(rgb.reshape(-1, 3), ref_rgb), maxabs(depth.reshape(-1), ref_dep)
    print(f"lego {precision} stratified hierarchical {w}x{h} {nc}+{ni}: rgb {er:.3e} depth {ed:.3e}")
    assert er < TOL_RENDER and ed < TOL_RENDER


@pytest.mark.parametrize("res,s", [((1, 1), 1), ((7, 3), 2), ((33, 9), 100), ((131, 3), 32)])
def test_lego_f16x3_edge_shapes_vs_oracle(ckpt, res, s):
    """Partial tiles and segments, S not a multiple of 32 (sequential composite) and of 32
    (fused), on real content, against the oracle's fp32 render."""
    from oracle import nerf_oracle as O

    _, f = W.lego_models()
    r = renderer(ckpt, "f16x3")
    pose = torch.from_numpy(np.load(os.path.join(GOLDEN, "rays.npz"))["poses"][2])
    rgb, depth = r.render_image(pose, res, s)
    ref_rgb, ref_depth = O.render_image(O.Net(f), pose, res, s)
    er, ed = maxabs(rgb, ref_rgb), maxabs(depth, ref_depth)
    print(f"lego f16x3 {res}x{s}: rgb {er:.3e} depth {ed:.3e}")
    assert er < TOL_RENDER and ed < TOL_RENDER


FULL = "render_lego_800x600_s128_full"


@pytest.mark.parametrize("precision", GATE)
def test_lego_headline_full_frames_vs_reference(ckpt, golden, precision):
    """Every pixel of the whole 800x600x128 headline frame, rendered by the reference's own
    PyTorchCPURenderer.render_image (pytorch_renderers.py:127-170) on the Lego checkpoint for
    the suite's views 0 and 1 and the off-axis pose (make_golden.py --lego-full): RGB and
    depth within the 1e-4 gate on all 480,000 pixels of each frame."""
    g = golden(FULL)
    r = renderer(ckpt, precision)
    for k in range(len(g["pose_ids"])):
        rgb, depth = r.render_image(torch.from_numpy(g["poses"][k]), (800, 600), 128)
        er, ed = maxabs(rgb, g[f"rgb_{k}"]), maxabs(depth, g[f"depth_{k}"])
        print(f"lego {precision} 800x600x128 full frame view {int(g['pose_ids'][k])}: rgb {er:.3e} depth {ed:.3e}")
        assert er < TOL_RENDER and ed < TOL_RENDER


# Per view (suite 0, suite 1, off-axis): RGB max, RGB mean and the count of pixels whose depth
# moves by > 1e-2, as measured on the driver's round-5 GPU suite (profiles/round5/r5u/gpu_suite.log);
# each test bound is 1.5x the measurement (+16 on the count) so a regression fails.
FULL_MEASURED = {
    "bf16": [(2.949e-02, 4.765e-04, 9039), (1.302e-03, 1.441e-05, 0), (4.011e-02, 5.802e-04, 13294)],
    "fp8": [(2.043e-01, 3.739e-03, 47309), (3.136e-02, 1.414e-04, 30817), (2.601e-01, 4.312e-03, 68028)],
    "bf16x3": [(5.692e-05, 8.755e-07, 0), (2.258e-06, 2.209e-08, 0), (7.772e-05, 1.009e-06, 1)],
}


def regression_bounds(measured):
    """1.5x a measured (max, mean, count) triple, the count with 16 pixels of slack."""
    m, a, n = measured
    return 1.5 * m, 1.5 * a, int(1.5 * n) + 16


@pytest.mark.parametrize("precision", ["bf16", "fp8", "bf16x3"])
def test_lego_headline_full_frames_error_report(ckpt, golden, precision):
    """The non-gate paths on the same whole frames, against the reference: max and mean RGB
    error and the number of pixels whose depth differs by more than 1e-2 (the single-pixel
    depth flips a row band would miss: a last sample with sigma ~ 0 turns a rounding-level
    sigma into alpha ~ 1 through the reference's 1e10 last distance).  Each is bounded at 1.5x
    its round-5 measurement per view (FULL_MEASURED)."""
    g = golden(FULL)
    r = renderer(ckpt, precision)
    for k in range(len(g["pose_ids"])):
        rgb, depth = r.render_image(torch.from_numpy(g["poses"][k]), (800, 600), 128)
        drgb = np.abs(rgb.cpu().numpy() - g[f"rgb_{k}"])
        ddep = np.abs(depth.cpu().numpy() - g[f"depth_{k}"])
        n_flip = int((ddep > 1e-2).sum())
        b_max, b_mean, b_flip = regression_bounds(FULL_MEASURED[precision][k])
        print(f"lego {precision} 800x600x128 full frame view {int(g['pose_ids'][k])}: rgb max {drgb.max():.3e} "
              f"mean {drgb.mean():.3e}; depth max {ddep.max():.3e}, pixels with depth error > 1e-2: {n_flip} "
              f"of {ddep.size} (bounds {b_max:.3e} / {b_mean:.3e} / {b_flip})")
        assert np.isfinite(drgb).all()
        assert drgb.max() < b_max and drgb.mean() < b_mean and n_flip <= b_flip


def test_lego_fp8_vs_reference_compressed(ckpt, golden):
    """Config 5's bar on Lego at 200x150x32: the fp8 path at least as close to the reference's
    fp32 render as the reference's own int8 compressed renderer (src/benchmark/compressed_renderer.py,
    rendered by it: compressed_lego.npz), in max AND mean RGB, on suite view 0 and the off-axis
    pose (the whole 800x600x128 frames: the test below).  Round 5's kernel keeps L0, L1, C0, the heads and the encodings on the bf16
    MFMA (tools/fp8_mixed_lab.py; the all-fp8 network of rounds 1-4 was 1.9x further off in max)."""
    g, gc = golden("render_lego_200x150_s32"), golden("compressed_lego")
    r = renderer(ckpt, "fp8")
    for kc, kg in ((0, 0), (1, 2)):
        assert np.array_equal(gc["poses"][kc], g["poses"][kg])
        rgb, _ = r.render_image(torch.from_numpy(g["poses"][kg]), (200, 150), 32)
        e8 = np.abs(rgb.cpu().numpy() - g[f"rgb_{kg}"])
        ec = np.abs(gc[f"rgb_{kc}"] - g[f"rgb_{kg}"])
        print(f"lego 200x150x32 view {int(g['pose_ids'][kg])} vs the reference's fp32 render: fp8 rgb max {e8.max():.3e} "
              f"mean {e8.mean():.3e}; reference int8 compressed rgb max {ec.max():.3e} mean {ec.mean():.3e}; "
              f"fp8 closer in max: {bool(e8.max() < ec.max())}, in mean: {bool(e8.mean() < ec.mean())}")
        assert np.isfinite(e8).all()
        assert e8.max() < ec.max() and e8.mean() < ec.mean()


def test_lego_fp8_vs_reference_compressed_full_frames(ckpt, golden):
    """Config 5's bar at config 5's own size: on whole 800x600x128 frames of
    suite view 0 and the off-axis pose, the fp8 path is closer to the reference's fp32 render
    (render_lego_800x600_s128_full.npz) than the reference's own int8 CompressedNeRFRenderer
    (compressed_lego_800x600_s128.npz, rendered by it through its own pieces in 4096-ray chunks,
    make_golden_compressed.py --lego-full; compressed_renderer.py:161-211, 233-269, 311-358), in
    max AND mean RGB."""
    g, gc = golden(FULL), golden("compressed_lego_800x600_s128")
    r = renderer(ckpt, "fp8")
    for kc, pid in enumerate(gc["pose_ids"]):
        kg = int(np.flatnonzero(g["pose_ids"] == pid)[0])
        assert np.array_equal(gc["poses"][kc], g["poses"][kg])
        rgb, depth = r.render_image(torch.from_numpy(g["poses"][kg]), (800, 600), 128)
        e8 = np.abs(rgb.cpu().numpy() - g[f"rgb_{kg}"])
        ec = np.abs(gc[f"rgb_{kc}"] - g[f"rgb_{kg}"])
        d8 = np.abs(depth.cpu().numpy() - g[f"depth_{kg}"])
        dc = np.abs(gc[f"depth_{kc}"] - g[f"depth_{kg}"])
        print(f"lego 800x600x128 view {int(pid)} vs the reference's fp32 render: fp8 rgb max {e8.max():.3e} mean "
              f"{e8.mean():.3e}, depth > 1e-2 on {int((d8 > 1e-2).sum())}; reference int8 compressed rgb max "
              f"{ec.max():.3e} mean {ec.mean():.3e}, depth > 1e-2 on {int((dc > 1e-2).sum())}; fp8 closer in max: "
              f"{bool(e8.max() < ec.max())}, in mean: {bool(e8.mean() < ec.mean())}")
        assert np.isfinite(e8).all()
        assert e8.max() < ec.max() and e8.mean() < ec.mean()
