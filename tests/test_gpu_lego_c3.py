"""BASELINE config 3 on whole Lego frames: 800x600, 64 coarse + 128 importance samples.

The fixture (tests/golden/render_lego_800x600_c3_full.npz, ``make_golden.py --lego-c3``) is
the reference's intended hierarchical chain run by the reference's own pieces -- rays, the 64
uniform coarse samples, the coarse ``NeRFModel`` and ``VolumeRenderer.volume_render``
(src/benchmark/base_renderer.py:165-281, src/utils/rendering.py:102-143) -- with the
oracle's fixed-gather sampler between them (the reference's ``importance_sample``,
rendering.py:54-100, crashes at its gather: build-defined), for suite view 0 and
the off-axis pose.  It also records a digest of each ray's 192 fine depths, so a test can
tell which rays the GPU rendered on the very samples the reference chain used.

  (i)   over all 480,000 rays, the render's fine depths equal the oracle's sampler fed the
        GPU's own coarse weights, bit for bit;
  (ii)  fp32 and f16x3: every pixel whose ray was rendered on the reference chain's own fine
        samples is within the 1e-4 gate of the fixture.  A pixel outside it must be a ray
        whose fine samples differ from the reference chain's, and there the GPU's render is
        within 1e-4 of the oracle's fine pass on the GPU's own samples: the difference is
        upstream of the fine pass, the coarse weights' last-bit differences (GPU MFMA vs the
        reference's CPU GEMM summation order) moved by the sampler.  Each such ray is listed
        with the sampler step that moved it (a ``denom < 1e-5`` switch, rendering.py:93, or an
        interpolation t = (u - cdf) / denom in a low-probability bin);
  (iii) bf16 and fp8 report max / mean RGB and the pixels whose depth moves by > 1e-2,
        bounded at 1.5x their round-5 measurement;
  (iv)  the truth: the same chain in float64 (render_lego_800x600_c3_fp64.npz,
        ``make_golden.py --lego-c3-fp64``).  The hierarchical chain is ill-conditioned at a few
        thousand rays per frame (a last-bit change of a coarse weight moves a fine sample), so
        no fp32 implementation can match another one there; what is asserted is that the GPU's
        fp32 render (and f16x3 with an fp32 coarse pass) is no further from the float64 truth
        than two fp32 CPU implementations of the chain are (c3_truth_spread.json).
"""
import os

import numpy as np
import pytest
import torch

from nerf_amd import weights as W

pytestmark = pytest.mark.gpu

TOL = 1e-4
C3 = "render_lego_800x600_c3_full"
C3_FP64 = "render_lego_800x600_c3_fp64"
NC, NI = 64, 128
MAX_DW = 1e-5                   # coarse weights GPU vs the oracle's CPU pass on the over-gate rays
_R = {}


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    return W.write_lego_checkpoint(str(tmp_path_factory.mktemp("ckpt_lego_c3") / "lego.pth"))


def renderer(ckpt, precision, coarse=None):
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    if (precision, coarse) not in _R:
        r = MI355XRenderer(precision, n_importance=NI, coarse_precision=coarse)
        r.setup(ckpt)
        _R[(precision, coarse)] = r
    return _R[(precision, coarse)]


def sampler_steps(z, w, u):
    """Per importance sample, the oracle sampler's bin (below), its raw denominator and
    whether the ``denom < 1e-5`` switch took it (rendering.py:86-93, gather fixed)."""
    w = w + 1e-5
    total = torch.cumsum(w, -1)[..., -1:]
    cdf = torch.cat([torch.zeros_like(w[..., :1]), torch.cumsum(w / total, -1)], -1)
    idx = torch.searchsorted(cdf.contiguous(), u.contiguous(), right=True)
    below, above = torch.clamp(idx - 1, 0, z.shape[-1] - 1), torch.clamp(idx, 0, z.shape[-1] - 1)
    denom = torch.gather(cdf, -1, above) - torch.gather(cdf, -1, below)
    return below, denom, denom < 1e-5


@pytest.mark.parametrize("precision", ["fp32", "f16x3"])
def test_lego_c3_full_frames_vs_reference(ckpt, golden, precision):
    from oracle import nerf_oracle as O

    g = golden(C3)
    w, h = int(g["W"]), int(g["H"])
    n = w * h
    r = renderer(ckpt, precision)
    _, fine = W.lego_models()
    coarse_net, fine_net = O.Net(W.lego_models()[0]), O.Net(fine)
    u = O.default_u(n, NI)
    for k in range(len(g["pose_ids"])):
        view = int(g["pose_ids"][k])
        pose = torch.from_numpy(g["poses"][k])
        rgb, depth = [t.clone() for t in r.render_image(pose, (w, h), NC)]
        zf = torch.empty(n, NC + NI, dtype=torch.float32, device="cuda")
        r.hip.last_fine_z(n, NC + NI, zf)
        zf = zf.cpu()
        # (i) the whole frame's fine samples are the oracle sampler on the GPU's coarse weights
        o, d = O.generate_rays(pose, w, h)
        o, d = o.reshape(-1, 3), d.reshape(-1, 3)
        zc = O.uniform_z(NC).expand(n, NC).contiguous()
        _, _, _, w_gpu = r.render_rays_z(o, d, zc, use_fine=False, with_weights=True)
        w_gpu = w_gpu.cpu()
        assert torch.equal(O.fine_z(zc, w_gpu, u), zf), "fine samples differ from the oracle sampler"
        # (ii) against the reference chain's pixels
        same = O.z_row_digest(zf) == g[f"zf_digest_{k}"].reshape(-1)
        e_rgb = np.abs(rgb.cpu().numpy().reshape(-1, 3) - g[f"rgb_{k}"].reshape(-1, 3)).max(-1)
        e_dep = np.abs(depth.cpu().numpy().reshape(-1) - g[f"depth_{k}"].reshape(-1))
        over = (e_rgb >= TOL) | (e_dep >= TOL)
        print(f"lego C3 {precision} view {view}: rays on the reference chain's own fine samples {int(same.sum())} "
              f"of {n}; rgb max {e_rgb.max():.3e} depth max {e_dep.max():.3e}; on the same samples rgb "
              f"{e_rgb[same].max() if same.any() else 0:.3e} depth {e_dep[same].max() if same.any() else 0:.3e}; "
              f"pixels over {TOL}: {int(over.sum())} (on the same samples: {int((over & same).sum())})")
        assert not (over & same).any(), "a ray rendered on the reference chain's samples is outside the gate"
        bad = np.flatnonzero(over)
        if bad.size == 0:
            continue
        # the oracle's fine pass on the GPU's own fine samples, for every pixel over the gate
        sel = torch.from_numpy(bad)
        ob, db, zb = o[sel], d[sel], zf[sel]
        pts = O.sample_points(ob, db, zb)
        s_, c_ = O.nerf_forward(fine_net, pts.reshape(-1, 3), db[:, None].expand_as(pts).reshape(-1, 3))
        ref_rgb, ref_dep = O.composite(s_.reshape(bad.size, -1, 1), c_.reshape(bad.size, -1, 3), zb, db)
        f_rgb = float((rgb.reshape(-1, 3)[sel.cuda()].cpu() - ref_rgb).abs().max())
        f_dep = float((depth.reshape(-1)[sel.cuda()].cpu() - ref_dep).abs().max())
        # the oracle's own coarse pass on those rays (the reference's arithmetic on the CPU): its
        # weights, its samples, and what moved them
        ps = O.sample_points(ob, db, zc[sel])
        sc, cc = O.nerf_forward(coarse_net, ps.reshape(-1, 3), db[:, None].expand_as(ps).reshape(-1, 3))
        _, _, _, w_cpu = O.composite(sc.reshape(bad.size, NC, 1), cc.reshape(bad.size, NC, 3), zc[sel], db, True)
        z_cpu = O.fine_z(zc[sel], w_cpu, u[sel])
        reproduces = O.z_row_digest(z_cpu) == g[f"zf_digest_{k}"].reshape(-1)[bad]
        b_g, den_g, sw_g = sampler_steps(zc[sel], w_gpu[sel], u[sel])
        b_c, den_c, sw_c = sampler_steps(zc[sel], w_cpu, u[sel])
        switch = (sw_g != sw_c).any(-1).numpy()
        bin_moved = (b_g != b_c).any(-1).numpy() & ~switch
        interp = ~switch & ~bin_moved
        min_denom = torch.where(sw_g, torch.ones_like(den_g), den_g).min(-1).values.numpy()
        dw = float((w_gpu[sel] - w_cpu).abs().max())
        dz = float((zf[sel] - z_cpu).abs().max())
        print(f"  {bad.size} pixels over the gate: GPU render vs the oracle's fine pass on the GPU's samples rgb "
              f"{f_rgb:.3e} depth {f_dep:.3e}; coarse weights GPU vs oracle max {dw:.2e}, fine depths max {dz:.2e}; "
              f"the oracle's coarse pass reproduces the reference chain's samples on {int(reproduces.sum())}; "
              f"cause: denom<1e-5 switch flipped {int(switch.sum())}, a sample changed bins {int(bin_moved.sum())}, "
              f"interpolation in a bin of denom >= 1e-5 {int(interp.sum())} (min denom median "
              f"{np.median(min_denom):.2e})")
        for i in bad[:12]:
            j = int(np.flatnonzero(bad == i)[0])
            print(f"    pixel ({i // w}, {i % w}): rgb err {e_rgb[i]:.2e} depth err {e_dep[i]:.2e}; switch "
                  f"{bool(switch[j])} bin {bool(bin_moved[j])} min denom {min_denom[j]:.2e}")
        assert f_rgb < TOL and f_dep < TOL, "the fine pass on the GPU's own samples is outside the gate"
        assert dw < MAX_DW, "the coarse weights differ by more than last bits"
        assert not same[bad].any()


def truth_stats(rgb, depth, t_rgb, t_dep):
    """Error of one frame against the float64 truth: max / mean RGB, max depth, and the pixels
    whose RGB (any channel) or depth is off by 1e-4 or more."""
    e_rgb = np.abs(np.asarray(rgb, np.float64).reshape(-1, 3) - t_rgb.reshape(-1, 3)).max(-1)
    e_dep = np.abs(np.asarray(depth, np.float64).reshape(-1) - t_dep.reshape(-1))
    return {"rgb_max": float(e_rgb.max()), "rgb_mean": float(e_rgb.mean()), "depth_max": float(e_dep.max()),
            "over": int(((e_rgb >= TOL) | (e_dep >= TOL)).sum())}


def fp32_envelope(spread, pose_id, ref):
    """The worse of two fp32 CPU implementations of the chain against the float64 truth: the
    reference's own pieces (the fixture) and the oracle's restatement run on a GPU box's host CPU,
    whose GEMM kernels sum in another order (tests/golden/c3_truth_spread.json)."""
    o = next(v for v in spread["views"] if v["pose_id"] == pose_id)["oracle_fp32_chain"]
    return {"over": max(ref["over"], o["over_1e-4"]), "rgb_max": max(ref["rgb_max"], o["rgb_max"]),
            "rgb_mean": max(ref["rgb_mean"], o["rgb_mean"]), "depth_max": max(ref["depth_max"], o["depth_max"])}


@pytest.mark.parametrize("precision,coarse", [("fp32", None), ("f16x3", "fp32"), ("f16x3", None)])
def test_lego_c3_no_further_from_fp64_than_reference(ckpt, golden, precision, coarse):
    """(iv) against the float64 run of the same chain (rendering.py:72-143 with the gather fixed,
    base_renderer.py:165-281, nerf.py:92-131 in float64).  Two fp32 CPU implementations -- the
    reference's own pieces and the oracle on another host CPU -- are 3,432-3,450 (view 0) and
    5,660-5,690 (off-axis) pixels over 1e-4 from it, with RGB max 5.7e-3-8.9e-3: in this chain a
    last-bit change of a coarse weight moves fine samples, so no fp32 implementation is closer.
    The GPU's fp32 path, and f16x3 with its coarse pass in fp32 (NERF_OPT_COARSE_PRECISION),
    have no more pixels over 1e-4 than the worse of the two CPU implementations, a mean error
    within 5 % of it, and max RGB / depth errors (single-pixel statistics) within 25 % of its.
    f16x3 with its own split-fp16 coarse pass (2^-22 operands against fp32's 2^-24) is further:
    its count stays within 5 % of the envelope and its mean within 10 % (the max is reported)."""
    g, t, spread = golden(C3), golden(C3_FP64), golden("c3_truth_spread.json")
    w, h = int(g["W"]), int(g["H"])
    r = renderer(ckpt, precision, coarse)
    for k in range(len(g["pose_ids"])):
        assert np.array_equal(g["poses"][k], t["poses"][k])
        rgb, depth = r.render_image(torch.from_numpy(g["poses"][k]), (w, h), NC)
        ref = truth_stats(g[f"rgb_{k}"], g[f"depth_{k}"], t[f"rgb_{k}"], t[f"depth_{k}"])
        env = fp32_envelope(spread, int(g["pose_ids"][k]), ref)
        gpu = truth_stats(rgb.cpu().numpy(), depth.cpu().numpy(), t[f"rgb_{k}"], t[f"depth_{k}"])
        print(f"lego C3 view {int(g['pose_ids'][k])} vs float64: reference fp32 chain rgb max {ref['rgb_max']:.3e} "
              f"mean {ref['rgb_mean']:.3e} depth max {ref['depth_max']:.3e} over {TOL}: {ref['over']}; fp32 CPU "
              f"envelope rgb max {env['rgb_max']:.3e} over {env['over']}; GPU {precision}"
              f"{'' if coarse is None else ' (' + coarse + ' coarse)'} rgb max {gpu['rgb_max']:.3e} mean "
              f"{gpu['rgb_mean']:.3e} depth max {gpu['depth_max']:.3e} over: {gpu['over']}")
        if precision == "fp32" or coarse == "fp32":
            assert gpu["over"] <= env["over"]
            assert gpu["rgb_mean"] <= 1.05 * env["rgb_mean"]
            assert gpu["rgb_max"] <= 1.25 * env["rgb_max"] and gpu["depth_max"] <= 1.25 * env["depth_max"]
        else:
            assert gpu["over"] <= 1.05 * env["over"] and gpu["rgb_mean"] <= 1.10 * env["rgb_mean"]


# Per view (suite 0, off-axis): RGB max, RGB mean and pixels with depth moved by > 1e-2 against
# the fp32 fixture, measured on the driver's round-5 GPU suite (profiles/round5/r5u/gpu_suite.log);
# bounded at 1.5x (+16 on the count; RGB max only where 1.5x stays below 1).
C3_MEASURED = {
    "bf16": [(4.858e-01, 1.153e-03, 20432), (6.551e-01, 6.226e-04, 12441)],
    "fp8": [(5.155e-01, 4.539e-03, 66700), (9.073e-01, 3.428e-03, 71941)],
}


@pytest.mark.parametrize("precision", ["bf16", "fp8"])
def test_lego_c3_full_frames_error_report(ckpt, golden, precision):
    """(iii) the throughput paths on the same whole C3 frames, bounded at 1.5x their round-5
    measurement per view so that a regression fails."""
    g = golden(C3)
    w, h = int(g["W"]), int(g["H"])
    r = renderer(ckpt, precision)
    for k in range(len(g["pose_ids"])):
        rgb, depth = r.render_image(torch.from_numpy(g["poses"][k]), (w, h), NC)
        e_rgb = np.abs(rgb.cpu().numpy() - g[f"rgb_{k}"])
        e_dep = np.abs(depth.cpu().numpy() - g[f"depth_{k}"])
        n_flip = int((e_dep > 1e-2).sum())
        m, a, n = C3_MEASURED[precision][k]
        b_max, b_mean, b_flip = 1.5 * m, 1.5 * a, int(1.5 * n) + 16
        print(f"lego C3 {precision} view {int(g['pose_ids'][k])}: rgb max {e_rgb.max():.3e} mean {e_rgb.mean():.3e}; "
              f"depth max {e_dep.max():.3e}, pixels with depth error > 1e-2: {n_flip} of {e_dep.size} "
              f"(bounds {min(b_max, 1.0):.3e} / {b_mean:.3e} / {b_flip})")
        assert np.isfinite(e_rgb).all() and e_rgb.mean() < b_mean and n_flip <= b_flip
        if b_max < 1.0:
            assert e_rgb.max() < b_max


def test_coarse_precision_option_samples_like_that_precision(ckpt, golden):
    """NERF_OPT_COARSE_PRECISION: an f16x3 render whose coarse pass runs in fp32 takes its fine
    samples from the fp32 coarse weights -- bit for bit the fp32 render's fine depths -- and its
    image stays within the gate of the fp32 render (only the fine pass differs)."""
    g = golden(C3)
    pose = torch.from_numpy(g["poses"][1])
    w, h = 200, 150
    a, b = renderer(ckpt, "f16x3", "fp32"), renderer(ckpt, "fp32")
    zs, imgs = [], []
    for r in (a, b):
        rgb, depth = [x.clone() for x in r.render_image(pose, (w, h), NC)]
        z = torch.empty(w * h, NC + NI, dtype=torch.float32, device="cuda")
        r.hip.last_fine_z(w * h, NC + NI, z)
        zs.append(z.cpu())
        imgs.append((rgb.cpu(), depth.cpu()))
    er = float((imgs[0][0] - imgs[1][0]).abs().max())
    ed = float((imgs[0][1] - imgs[1][1]).abs().max())
    print(f"f16x3 with fp32 coarse vs fp32, {w}x{h} 64+128: fine z equal {bool(torch.equal(zs[0], zs[1]))}; "
          f"rgb {er:.3e} depth {ed:.3e}")
    assert torch.equal(zs[0], zs[1])
    assert er < TOL and ed < TOL


def test_coarse_precision_option_rejects_bad_values(ckpt):
    """NERF_OPT_COARSE_PRECISION takes -1 or a precision (NERF_E_INVALID otherwise), and a
    renderer built with an unknown coarse precision is refused before any device call."""
    from nerf_amd import runtime as rt
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    r = renderer(ckpt, "f16x3", "fp32")
    for bad in (-2, 5, 99):
        with pytest.raises(rt.NerfError, match="NERF_OPT_COARSE_PRECISION"):
            r.hip.set_coarse_precision(bad)
    r.hip.set_coarse_precision(rt.NERF_FP32)       # restore the cached renderer's setting
    with pytest.raises(ValueError):
        MI355XRenderer("f16x3", n_importance=NI, coarse_precision="fp16")
