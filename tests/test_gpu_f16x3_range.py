"""NERF_F16X3's fp16 range contract (include/nerf_mi355x.h, mlp_x3.h).

The split-fp16 parity path rounds every weight and activation to fp16 halves, so a value
at or above 65520 would overflow.  Weights are checked when the network is loaded (the
precision is then refused for that network); activations and encoding inputs are checked
on the device per sample (an overflowed hi = +inf turns the next layer's column into NaN,
which the kernel detects) and reported as NerfRangeError: the plugin never returns an
image with inf or NaN, and below the boundary the path matches fp32.  Reference: the
forward it restates computes in fp32 (src/models/nerf.py:107-129); there is no reference
counterpart of the range error.
"""
import numpy as np
import pytest
import torch

from nerf_amd import runtime as rt
from nerf_amd import weights as W

pytestmark = pytest.mark.gpu


def _renderer(path, precision):
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    r = MI355XRenderer(precision)
    r.setup(path)
    return r


def _points(n=4096, seed=3, scale=4.0):
    rng = np.random.default_rng(seed)
    return (torch.from_numpy(rng.uniform(-scale, scale, (n, 3)).astype(np.float32)),
            torch.from_numpy(rng.uniform(-1.2, 1.2, (n, 3)).astype(np.float32)))


def _max_activation(sd, pos):
    """Largest post-ReLU trunk activation (float64 forward of the eight trunk layers)."""
    from oracle import nerf_oracle as O

    pe = O.positional_encoding(pos, 10).numpy().astype(np.float64).T
    h, m = pe, 0.0
    for i in range(8):
        if i == 4:
            h = np.concatenate([h, pe])
        h = np.maximum(sd[f"layers.{i}.weight"].astype(np.float64) @ h + sd[f"layers.{i}.bias"][:, None], 0)
        m = max(m, float(h.max()))
    return m


def _scaled(sd, factor):
    out = dict(sd)
    out["layers.2.weight"] = (sd["layers.2.weight"] * np.float32(factor)).astype(np.float32)
    out["layers.2.bias"] = (sd["layers.2.bias"] * np.float32(factor)).astype(np.float32)
    return out


@pytest.fixture(scope="module")
def nets(tmp_path_factory):
    """Three versions of one low-gain network: layer 2 scaled so that the largest activation
    lands at ~2e4 (inside fp16's range), and at ~1.5e5 (outside it; the weights still fit)."""
    base = W.synthetic_state_dict(21, conditioned=False)
    pos, _ = _points()
    m0 = _max_activation(base, pos)
    d = tmp_path_factory.mktemp("f16range")
    out = {}
    for tag, target in (("inside", 2.0e4), ("outside", 1.5e5)):   # layer 2's weights stay inside fp16
        # the largest activation is not linear in the factor (layers 0-1 are unscaled, biases
        # follow), so a few fixed-point steps land it near the target
        f = target / m0
        for _ in range(6):
            sd = _scaled(base, f)
            m = _max_activation(sd, pos)
            f *= target / m
        p = str(d / f"{tag}.pth")
        W.save_checkpoint(p, sd, sd)
        out[tag] = (p, m)
    return out


def test_f16x3_inside_range_matches_fp32(nets):
    path, m = nets["inside"]
    assert 5e3 < m < 6.5e4, m
    pos, dirs = _points()
    r16, r32 = _renderer(path, "f16x3"), _renderer(path, "fp32")
    s, c = r16.query_nerf_networks(pos, dirs)
    s32, c32 = r32.query_nerf_networks(pos, dirs)
    es = float(((s - s32).abs() / s32.abs().clamp_min(1.0)).max())
    ec = float((c - c32).abs().max())
    print(f"f16x3 with activations up to {m:.3g}: sigma rel {es:.2e}, rgb {ec:.2e} vs fp32")
    assert torch.isfinite(s).all() and torch.isfinite(c).all()
    # sigma relative to its size; RGB is a sigmoid of logits ~1e4 here, so an fp32-level
    # relative difference of the logits (~2^-22) is what the absolute bound allows
    assert es < 1e-4 and ec < 1e-3
    rgb, dep = r16.render_image(torch.eye(4), (48, 32), 32)
    assert torch.isfinite(rgb).all() and torch.isfinite(dep).all()


def test_f16x3_outside_range_raises_and_recovers(nets):
    path, m = nets["outside"]
    assert m > 1e5, m
    pos, dirs = _points()
    r = _renderer(path, "f16x3")
    with pytest.raises(rt.NerfRangeError):
        r.query_nerf_networks(pos, dirs)
    pose = torch.eye(4)
    pose[2, 3] = 4.0
    with pytest.raises(rt.NerfRangeError):
        r.render_image(pose, (64, 48), 32)          # fused-composite render pass
    with pytest.raises(rt.NerfRangeError):
        r.render_image(pose, (64, 48), 20)          # sequential composite (S % 32 != 0)
    # the other precisions run the same network
    s32, _ = _renderer(path, "fp32").query_nerf_networks(pos, dirs)
    assert torch.isfinite(s32).all()
    # the flag was cleared by the report: a network inside the range renders again
    r.setup(nets["inside"][0])
    rgb, _ = r.render_image(pose, (64, 48), 32)
    assert torch.isfinite(rgb).all()


def test_f16x3_encoding_input_outside_range_raises(nets):
    """A sample coordinate itself beyond fp16's range (the raw x of the encoding)."""
    r = _renderer(nets["inside"][0], "f16x3")
    pos, dirs = _points(256)
    pos[17, 1] = 7.0e4
    with pytest.raises(rt.NerfRangeError):
        r.query_nerf_networks(pos, dirs)
    pos[17, 1] = 0.5
    s, _ = r.query_nerf_networks(pos, dirs)
    assert torch.isfinite(s).all()


def test_f16x3_refused_for_out_of_range_weights(tmp_path):
    """A weight above 65504: loading succeeds (every other precision works), NERF_F16X3 is
    refused with a message naming the range, and the load leaves no stale error behind."""
    sd = W.synthetic_state_dict(4, conditioned=False)
    big = dict(sd)
    big["layers.1.weight"] = sd["layers.1.weight"].copy()
    big["layers.1.weight"][0, 0] = np.float32(1e5)
    p_big, p_ok = str(tmp_path / "big.pth"), str(tmp_path / "ok.pth")
    W.save_checkpoint(p_big, big, big)
    W.save_checkpoint(p_ok, sd, sd)
    pos, dirs = _points(128)
    r = _renderer(p_ok, "f16x3")
    r.query_nerf_networks(pos, dirs)
    before = rt.load_library().nerf_last_error().decode()
    r.setup(p_big)                                   # reload over a valid net
    assert rt.load_library().nerf_last_error().decode() == before   # the probe's refusal is not the load's error
    with pytest.raises(rt.NerfError, match="fp16"):
        r.query_nerf_networks(pos, dirs)
    for prec in ("fp32", "bf16", "bf16x3"):
        s, _ = _renderer(p_big, prec).query_nerf_networks(pos, dirs)
        assert torch.isfinite(s).all()
