"""The largest launches: more than 2^32 samples in one render.

Every sample index in the render path is 64-bit; below 2^32 samples the kernels divide sample
indices in 32 bits (fetch_render_sample's idx32), above it in 64.  A 4096x2160 frame at 512
samples per ray is 4.53e9 samples (the MLP scratch alone is 72 GB of the 288 GB): its first
and last row bands must equal the same bands rendered as launches of their own, bit for bit
(a ray's result does not depend on where in the launch its samples sit).  The reference has
no such test (its CPU renderer is far too slow for a frame this size); the property is the
repo's own.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

W_, H_, SPP = 4096, 2160, 512
BAND = 8


@pytest.fixture(scope="module")
def lego_ckpt(tmp_path_factory):
    from nerf_amd import weights as W

    return W.write_lego_checkpoint(str(tmp_path_factory.mktemp("maxsize") / "lego.pth"))


@pytest.mark.parametrize("precision", ["bf16", "fp8", "f16x3"])
def test_render_beyond_2p32_samples(lego_ckpt, precision):
    from nerf_amd.benchmark.benchmark_suite import generate_test_poses
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    assert W_ * H_ * SPP > 2 ** 32
    free, _ = torch.cuda.mem_get_info()
    if free < 100 * 2 ** 30:
        pytest.skip(f"needs ~80 GB of device memory, {free / 2 ** 30:.0f} GB free")
    r = MI355XRenderer(precision)
    r.setup(lego_ckpt)
    try:
        pose = generate_test_poses(2)[0]
        rgb, dep = r.render_rows(pose, (W_, H_), SPP, 0, H_)
        r.check_range()
        torch.cuda.synchronize()
        assert bool(torch.isfinite(rgb).all()) and bool(torch.isfinite(dep).all())
        for r0 in (0, H_ // 2 - BAND // 2, H_ - BAND):
            b_rgb, b_dep = r.render_rows(pose, (W_, H_), SPP, r0, r0 + BAND)
            torch.cuda.synchronize()
            assert torch.equal(b_rgb, rgb[r0:r0 + BAND]) and torch.equal(b_dep, dep[r0:r0 + BAND]), (
                f"{precision}: rows [{r0}, {r0 + BAND}) of the 4.53e9-sample launch differ from their own launch")
        # the image is not blank: the Lego object covers part of the centre rows
        centre = rgb[H_ // 2 - BAND // 2:H_ // 2 + BAND // 2].cpu().numpy()
        assert float(np.abs(centre - centre.mean()).max()) > 1e-3
    finally:
        del r
        torch.cuda.empty_cache()
