"""The reference's own Lego networks on the GPU: the original NeRF implementation's layout
("optionally a second original-NeRF weight-layout loader in the MLP kernel";
include/nerf_mi355x.h NERF_LAYOUT_ORIGINAL_NERF), rendered by the fp32 kernel.

The arrays are the reference's bundled data/lego_example_weights/model{,_fine}_200000.npy, read
by the static parser (tools/lego/npy_static.py) and exported by __graft_entry__.build() into
tools/lego/_teacher_{coarse,fine}.npz for the GPU box, which has no reference checkout.  The CPU
side is tools/lego/teacher.Teacher (the original network restated in PyTorch: encodings without
pi, skip cat([pe, h]) into layer 5, normalised view directions, the feature layer) composited by
the oracle's execute_volume_rendering restatement (pytorch_renderers.py:105-125) -- the
reference's renderer semantics with the original networks.  No reference code runs these arrays
(SURVEY F5), so the parity anchor is that restatement, not a reference output.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 1e-4
_R = {}


def arrays(which):
    from tools.lego import teacher as T

    cache = os.path.join(REPO, "tools", "lego", f"_teacher_{which}.npz")
    if not (os.path.isdir(T.LEGO_DIR) or os.path.exists(cache)):
        pytest.fail(f"{cache} missing: run __graft_entry__.build() where the reference checkout is present")
    return T.load_arrays(which)


def renderer(precision="fp32", n_importance=0):
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    if (precision, n_importance) not in _R:
        r = MI355XRenderer(precision, n_importance=n_importance)
        r.setup_original_nerf(arrays("coarse"), arrays("fine"))
        _R[(precision, n_importance)] = r
    return _R[(precision, n_importance)]


def teacher(which):
    from tools.lego import teacher as T

    return T.Teacher(arrays(which)).eval()


def cpu_render(net, pose, w, h, spp, rows):
    """The reference renderer's uniform path (base_renderer.py:223-281, pytorch_renderers.py:
    105-170) with the original network as the MLP, on rows [r0, r1)."""
    from oracle import nerf_oracle as O

    o, d = O.generate_rays(pose, w, h)
    o, d = o[rows[0]:rows[1]].reshape(-1, 3), d[rows[0]:rows[1]].reshape(-1, 3)
    z = O.uniform_z(spp).expand(o.shape[0], spp)
    pts = O.sample_points(o, d, z)
    with torch.no_grad():
        s, c = net(pts.reshape(-1, 3), d[:, None].expand_as(pts).reshape(-1, 3))
    rgb, dep = O.composite(s.reshape(o.shape[0], spp, 1), c.reshape(o.shape[0], spp, 3), z, d)
    return rgb.reshape(rows[1] - rows[0], w, 3), dep.reshape(rows[1] - rows[0], w)


@pytest.mark.parametrize("precision", ["fp32", "f16x3"])
def test_original_nerf_query_matches_teacher(precision):
    """nerf_query (explicit points) with the original fine network against its restatement."""
    r = renderer(precision)
    g = np.load(os.path.join(REPO, "tests", "golden", "lego_mlp.npz"))
    pos, dirs = torch.from_numpy(g["pos"][:4096]), torch.from_numpy(g["dirs"][:4096])
    sigma, rgb = r.query_nerf_networks(pos.cuda(), dirs.cuda(), use_fine=True)
    with torch.no_grad():
        s_ref, c_ref = teacher("fine")(pos, dirs)
    es = float(((sigma.cpu() - s_ref).abs() / (s_ref.abs() + 1.0)).max())
    ec = float((rgb.cpu() - c_ref).abs().max())
    print(f"original-NeRF fine query {precision}: sigma rel max {es:.3e} (sigma up to {float(s_ref.max()):.1f}), "
          f"rgb max {ec:.3e}")
    assert es < 1e-4 and ec < 1e-5


@pytest.mark.parametrize("precision", ["fp32", "f16x3"])
@pytest.mark.parametrize("res,spp,rows", [((200, 150), 32, (0, 150)), ((800, 600), 128, (296, 304))])
def test_original_nerf_render_at_gate(res, spp, rows, precision):
    """Whole 200x150x32 frames and a band of the 800x600x128 headline frame, suite view 0 and
    the off-axis pose, within the 1e-4 gate of the CPU render with the same networks."""
    from nerf_amd.benchmark.benchmark_suite import generate_test_poses

    off_axis = np.load(os.path.join(REPO, "tests", "golden", "render_lego_200x150_s32.npz"))["poses"][2]
    poses = [generate_test_poses(2)[0], torch.from_numpy(off_axis)]
    r = renderer(precision)
    net = teacher("fine")
    w, h = res
    for k, pose in enumerate(poses):
        rgb, dep = r.render_rows(pose, (w, h), spp, rows[0], rows[1])
        ref_rgb, ref_dep = cpu_render(net, pose, w, h, spp, rows)
        er = float((rgb.cpu() - ref_rgb).abs().max())
        ed = float((dep.cpu() - ref_dep).abs().max())
        r.check_range()
        print(f"original-NeRF Lego {precision} {w}x{h}x{spp} rows {rows} view {k}: rgb {er:.3e} depth {ed:.3e} "
              f"(mean rgb {float(ref_rgb.mean()):.3f})")
        assert float(ref_rgb.max()) > 0.1                         # the object is in the frame
        assert er < TOL and ed < TOL


def test_original_nerf_hierarchical_runs_and_other_precisions_refused():
    """64 + 128 hierarchical with both original networks: finite, inside [0, 1]; and a net in
    the original layout refuses every precision but fp32 and f16x3 (NERF_E_INVALID)."""
    from nerf_amd import runtime as rt
    from nerf_amd.benchmark.benchmark_suite import generate_test_poses

    r = renderer("fp32", 128)
    rgb, dep = r.render_image(generate_test_poses(2)[0], (80, 60), 64)
    rgb = rgb.cpu()
    assert torch.isfinite(rgb).all() and float(rgb.min()) >= 0.0 and float(rgb.max()) <= 1.0 + 1e-6
    assert float(rgb.max()) > 0.1
    pos = torch.zeros(32, 3, device="cuda")
    out = torch.empty(32, 4, device="cuda")
    with pytest.raises(rt.NerfError, match="original-NeRF layout"):
        r.hip.query(rt.NERF_NET_FINE, rt.NERF_BF16, pos, pos + 1.0, out)


def test_original_nerf_hierarchical_f16x3_with_fp32_coarse_samples_like_fp32():
    """The original networks, 64 + 128: f16x3 with its coarse pass in fp32 takes the fp32 render's
    fine samples bit for bit, and its image is within the gate of the fp32 render."""
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer
    from nerf_amd.benchmark.benchmark_suite import generate_test_poses

    pose = generate_test_poses(2)[0]
    w, h = 120, 90
    a = MI355XRenderer("f16x3", n_importance=128, coarse_precision="fp32")
    a.setup_original_nerf(arrays("coarse"), arrays("fine"))
    b = renderer("fp32", 128)
    zs, imgs = [], []
    for r in (a, b):
        rgb, dep = [t.clone() for t in r.render_image(pose, (w, h), 64)]
        z = torch.empty(w * h, 192, dtype=torch.float32, device="cuda")
        r.hip.last_fine_z(w * h, 192, z)
        zs.append(z.cpu())
        imgs.append((rgb.cpu(), dep.cpu()))
    er = float((imgs[0][0] - imgs[1][0]).abs().max())
    ed = float((imgs[0][1] - imgs[1][1]).abs().max())
    print(f"original-NeRF 64+128 {w}x{h}: f16x3 (fp32 coarse) vs fp32: fine z equal {bool(torch.equal(zs[0], zs[1]))}, "
          f"rgb {er:.3e} depth {ed:.3e}")
    assert torch.equal(zs[0], zs[1]) and er < TOL and ed < TOL
