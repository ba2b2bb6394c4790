"""Pin the oracle (oracle/nerf_oracle.py) to golden vectors produced by the reference.

The fixtures come from tests/golden/make_golden.py, which ran the reference's
own renderer, model and volume-render code on the synthetic checkpoint.  The
oracle must reproduce them bit-for-bit where the arithmetic is deterministic
element-wise work (rays, t/z tables, stratified samples, the whole pipeline on
this host) and to fp32 rounding otherwise (a different host's GEMM kernels may
sum in another order).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
from nerf_amd import weights as W

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TOL = 2e-6     # fp32 rounding slack for GEMM/transcendental kernels of another host


@pytest.fixture(scope="module")
def nets():
    c, f = W.synthetic_models(0)
    return O.Net(c), O.Net(f)


def test_checkpoint_digest_matches_fixtures():
    meta = json.load(open(os.path.join(GOLDEN, "golden_meta.json")))
    c, f = W.synthetic_models(0)
    assert W.state_dict_digest(c) == meta["coarse_digest"]
    assert W.state_dict_digest(f) == meta["fine_digest"]


def test_rays_bit_exact(golden):
    g = golden("rays")
    keys = [k for k in g.files if k.startswith("o_")]
    assert len(keys) == 9
    for k in keys:
        tag = k[2:]
        w, h = map(int, tag.split("_")[0].split("x"))
        pi = int(tag.split("_")[1])
        o, d = O.generate_rays(g["poses"][pi], w, h)
        assert np.array_equal(o.numpy(), g[k]), tag
        assert np.array_equal(d.numpy(), g["d_" + tag]), tag


@pytest.mark.parametrize("s", [1, 2, 3, 16, 32, 64, 128, 192, 256])
def test_tvals_and_z_bit_exact(golden, s):
    g = golden("tvals")
    assert np.array_equal(O.t_vals(s).numpy(), g[f"t_{s}"])
    assert np.array_equal(O.uniform_z(s).numpy(), g[f"z_{s}"])


def test_stratified_samples_bit_exact(golden):
    g = golden("stratified")
    z = O.stratified_z(O.uniform_z(32), torch.from_numpy(g["t_rand"]))
    assert np.array_equal(z.numpy(), g["z"])
    pts = O.sample_points(torch.from_numpy(g["rays_o"]), torch.from_numpy(g["rays_d"]), z)
    assert np.array_equal(pts.numpy(), g["pts"])


def test_positional_encoding(golden):
    g = golden("pe")
    x = torch.from_numpy(g["x"])
    for L, key in ((10, "pe10"), (4, "pe4")):
        pe = O.positional_encoding(x, L).numpy()
        assert pe.shape == g[key].shape == (x.shape[0], 3 + 6 * L)
        np.testing.assert_allclose(pe, g[key], rtol=0, atol=TOL)


def test_mlp_forward(golden, nets):
    g = golden("mlp")
    coarse, fine = nets
    for net, tag in ((fine, "fine"), (coarse, "coarse")):
        s, rgb = O.nerf_forward(net, torch.from_numpy(g["pos"]), torch.from_numpy(g["dirs"]))
        np.testing.assert_allclose(s.numpy(), g[f"sigma_{tag}"], rtol=1e-6, atol=1e-5)
        np.testing.assert_allclose(rgb.numpy(), g[f"rgb_{tag}"], rtol=0, atol=TOL)


@pytest.mark.parametrize("case", ["rand16", "rand32", "rand64", "rand128", "edge64"])
def test_composite(golden, case):
    g = golden("composite")
    rgb, depth, acc, w = O.composite(g[f"{case}_sigma"], g[f"{case}_rgb_in"], g[f"{case}_z"], g[f"{case}_d"], True)
    np.testing.assert_allclose(rgb.numpy(), g[f"{case}_rgb"], rtol=0, atol=TOL)
    np.testing.assert_allclose(depth.numpy(), g[f"{case}_depth"], rtol=0, atol=4 * TOL)
    np.testing.assert_allclose(acc.numpy(), g[f"{case}_acc"], rtol=0, atol=TOL)
    np.testing.assert_allclose(w.numpy(), g[f"{case}_weights"], rtol=0, atol=TOL)


@pytest.mark.parametrize("name", ["render_64x48_s16", "render_37x23_s7", "render_200x150_s32"])
def test_full_render(golden, nets, name):
    g = golden(name)
    _, fine = nets
    w, h, s = int(g["W"]), int(g["H"]), int(g["S"])
    for k in range(len(g["pose_ids"])):
        rgb, depth = O.render_image(fine, g["poses"][k], (w, h), s)
        np.testing.assert_allclose(rgb.numpy(), g[f"rgb_{k}"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(depth.numpy(), g[f"depth_{k}"], rtol=0, atol=1e-5)


def test_headline_band(golden, nets):
    """Rows 296..303 of the 800x600x128 headline image (reference's chunked path)."""
    g = golden("render_800x600_s128_band")
    _, fine = nets
    r0, r1 = map(int, g["rows"])
    for k in range(2):
        rgb, depth = O.render_image(fine, g["poses"][k], (800, 600), 128, rows=(r0, r1))
        np.testing.assert_allclose(rgb.numpy(), g[f"rgb_{k}"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(depth.numpy(), g[f"depth_{k}"], rtol=0, atol=1e-5)


def test_importance_sample_properties():
    """Build-defined hierarchical sampler (reference crashes): parity unpinned
    beyond these properties -- sorted union, coarse z preserved, samples inside [near, far]."""
    torch.manual_seed(0)
    n, s, ni = 64, 64, 128
    z = O.uniform_z(s).expand(n, s).contiguous()
    w = torch.rand(n, s) ** 4
    u = O.default_u(n, ni)
    zi = O.importance_sample(z, w, u)
    assert zi.shape == (n, ni)
    assert torch.all(zi[:, 1:] >= zi[:, :-1])           # monotone in ascending u
    assert torch.all((zi >= 2.0) & (zi <= 6.0))
    zf = O.fine_z(z, w, u)
    assert zf.shape == (n, s + ni)
    assert torch.all(zf[:, 1:] >= zf[:, :-1])
    # every coarse sample survives the merge
    for r in range(0, n, 16):
        assert set(z[r].tolist()) <= set(zf[r].tolist())


def test_compressed_restatement_matches_reference(golden):
    """The reference's int8 compressed renderer (fp8 path's error baseline)."""
    g = golden("compressed")
    _, f = W.synthetic_models(0)
    cw = O.compressed_weights(f)
    s, c = O.compressed_query(cw, torch.from_numpy(g["pos"]), torch.from_numpy(g["dirs"]))
    assert np.array_equal(s.numpy(), g["sigma"]) and np.array_equal(c.numpy(), g["rgb"])
    rgb, depth = O.compressed_render_image(cw, torch.from_numpy(g["pose"]), (32, 24), 16)
    assert np.array_equal(rgb.numpy(), g["image"]) and np.array_equal(depth.numpy(), g["depth"])


# ---- the Lego checkpoint: reference renders on real content ----------
@pytest.fixture(scope="module")
def lego_nets():
    c, f = W.lego_models()
    return O.Net(c), O.Net(f)


def test_lego_checkpoint_digest_matches_fixtures():
    meta = json.load(open(os.path.join(GOLDEN, "golden_lego_meta.json")))
    c, f = W.lego_models()
    assert W.state_dict_digest(c) == meta["coarse_digest"] and W.state_dict_digest(f) == meta["fine_digest"]


def test_lego_mlp_forward(golden, lego_nets):
    g = golden("lego_mlp")
    coarse, fine = lego_nets
    for net, tag in ((fine, "fine"), (coarse, "coarse")):
        s, rgb = O.nerf_forward(net, torch.from_numpy(g["pos"]), torch.from_numpy(g["dirs"]))
        np.testing.assert_allclose(s.numpy(), g[f"sigma_{tag}"], rtol=1e-5, atol=1e-4)
        np.testing.assert_allclose(rgb.numpy(), g[f"rgb_{tag}"], rtol=0, atol=TOL)


def test_lego_full_render_and_band(golden, lego_nets):
    _, fine = lego_nets
    g = golden("render_lego_200x150_s32")
    for k in range(len(g["pose_ids"])):
        rgb, depth = O.render_image(fine, g["poses"][k], (200, 150), 32)
        np.testing.assert_allclose(rgb.numpy(), g[f"rgb_{k}"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(depth.numpy(), g[f"depth_{k}"], rtol=0, atol=1e-5)
    g = golden("render_lego_800x600_s128_band")
    r0, r1 = map(int, g["rows"])
    rgb, depth = O.render_image(fine, g["poses"][1], (800, 600), 128, rows=(r0, r1))
    np.testing.assert_allclose(rgb.numpy(), g["rgb_1"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(depth.numpy(), g["depth_1"], rtol=0, atol=1e-5)


def test_lego_headline_full_frames_sampled_rows(golden, lego_nets):
    """The whole-frame 800x600x128 fixtures (make_golden.py --lego-full, the reference's own
    render_image on views 0, 1 and the off-axis pose): the oracle reproduces rows from the
    top, the middle and the bottom of every frame; consistent with the headline band fixture
    where they overlap."""
    _, fine = lego_nets
    g = golden("render_lego_800x600_s128_full")
    assert (int(g["W"]), int(g["H"]), int(g["S"])) == (800, 600, 128)
    for k in range(len(g["pose_ids"])):
        assert g[f"rgb_{k}"].shape == (600, 800, 3) and g[f"depth_{k}"].shape == (600, 800)
        for r0 in (0, 297, 599):
            rgb, depth = O.render_image(fine, g["poses"][k], (800, 600), 128, rows=(r0, r0 + 1))
            np.testing.assert_allclose(rgb.numpy(), g[f"rgb_{k}"][r0:r0 + 1], rtol=0, atol=1e-5)
            np.testing.assert_allclose(depth.numpy(), g[f"depth_{k}"][r0:r0 + 1], rtol=0, atol=1e-5)
    band = golden("render_lego_800x600_s128_band")
    b0, b1 = map(int, band["rows"])
    for kb, kf in ((0, 0), (1, 2)):                    # band views: suite view 0, off-axis
        np.testing.assert_array_equal(band[f"rgb_{kb}"], g[f"rgb_{kf}"][b0:b1])
        np.testing.assert_array_equal(band[f"depth_{kb}"], g[f"depth_{kf}"][b0:b1])


def test_compressed_restatement_on_lego(golden):
    """Config 5's error baseline on Lego: the oracle's restatement of the reference's int8
    compressed renderer reproduces the reference's own render (make_golden_compressed.py
    --lego) of the distilled checkpoint at 200x150x32, bit for bit."""
    g = golden("compressed_lego")
    _, f = W.lego_models()
    cw = O.compressed_weights(f)
    for k in range(len(g["pose_ids"])):
        rgb, depth = O.compressed_render_image(cw, torch.from_numpy(g["poses"][k]), (200, 150), 32)
        np.testing.assert_array_equal(rgb.numpy(), g[f"rgb_{k}"])
        np.testing.assert_array_equal(depth.numpy(), g[f"depth_{k}"])


def test_c3_truth_fixtures_consistent():
    """The float64 C3 truth (make_golden.py --lego-c3-fp64) and the fp32 CPU spread record
    (tools/c3_truth_spread.py, c3_truth_spread.json) describe the same frames: same poses, and
    the reference fp32 chain's distance to the truth recomputed here equals the recorded one."""
    import json

    g = np.load(os.path.join(GOLDEN, "render_lego_800x600_c3_full.npz"))
    t = np.load(os.path.join(GOLDEN, "render_lego_800x600_c3_fp64.npz"))
    spread = json.load(open(os.path.join(GOLDEN, "c3_truth_spread.json")))
    assert t["rgb_0"].dtype == np.float64 and np.array_equal(g["poses"], t["poses"])
    for k, pid in enumerate(g["pose_ids"]):
        e_rgb = np.abs(g[f"rgb_{k}"].astype(np.float64) - t[f"rgb_{k}"]).max(-1)
        e_dep = np.abs(g[f"depth_{k}"].astype(np.float64) - t[f"depth_{k}"])
        rec = next(v for v in spread["views"] if v["pose_id"] == int(pid))["reference_fp32_chain"]
        assert int(((e_rgb >= 1e-4) | (e_dep >= 1e-4)).sum()) == rec["over_1e-4"]
        assert abs(float(e_rgb.max()) - rec["rgb_max"]) < 1e-12 and abs(float(e_dep.max()) - rec["depth_max"]) < 1e-12
