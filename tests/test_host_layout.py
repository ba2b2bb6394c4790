"""Host-side checks of the C ABI library -- no GPU needed.

* the library loads and exports every symbol include/nerf_mi355x.h declares;
* the z table helper reproduces the reference's z values bit for bit;
* the weight packer (the same C++ code nerf_ctx_load_weights runs) produces
  fragment blobs that, pushed through a numpy emulation of the kernels'
  MFMA lane maps, compute exactly the NeRF MLP.  This pins the packing and the
  k-order permutations on CPU; the GPU tests then pin the kernels themselves.
"""
import os
import re

import numpy as np
import pytest
import torch

from nerf_amd import runtime as rt
from nerf_amd import weights as W
from oracle import nerf_oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "nerf_mi355x.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nerf_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding():
    assert declared_functions() == sorted(rt.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = rt.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.nerf_abi_version() == 6


def test_uniform_z_bit_exact(golden):
    g = golden("tvals")
    for s in [1, 2, 3, 16, 32, 64, 128, 192, 256]:
        assert np.array_equal(rt.uniform_z(g[f"t_{s}"], 2.0, 6.0), g[f"z_{s}"]), s


def test_linspace01_matches_torch():
    import torch

    for n in list(range(1, 300)) + [511, 512, 513, 1000, 1023, 1024, 2048]:
        assert np.array_equal(rt.linspace01(n), torch.linspace(0, 1, n).numpy()), n


def test_pack_rejects_bad_input():
    sd = W.synthetic_state_dict(3)
    bad = dict(sd)
    bad["layers.4.weight"] = np.zeros((256, 318), np.float32)
    with pytest.raises(ValueError):
        rt.pack_weights(bad)


# ---------------------------------------------------------------- layout spec --
# Python statement of nerf_layout.h (the kernels' register maps).
def acc_row(r, h):
    return (r & 3) + 8 * (r >> 2) + 4 * h


def pe_slot_feature(h, q):
    if q < 30:
        return 3 + 6 * (5 * h + q // 6) + (q % 6)
    if h == 0:
        return q - 30
    return 2 if q == 30 else -1


def dpe_slot_feature(h, q):
    if q < 12:
        return 3 + 6 * (2 * h + q // 6) + (q % 6)
    if h == 0:
        return q - 12 if q < 14 else -1
    return 2 if q == 12 else -1


LAYERS = [  # (spec prefix, out, hidden, extra)
    ("layers.0", 256, 0, "pos"), ("layers.1", 256, 256, None), ("layers.2", 256, 256, None),
    ("layers.3", 256, 256, None), ("layers.4", 256, 256, "pos"), ("layers.5", 256, 256, None),
    ("layers.6", 256, 256, None), ("layers.7", 256, 256, None), ("color_layers.0", 128, 256, "dir"),
]


def bf16_to_f32(u16):
    return (u16.astype(np.uint32) << 16).view(np.float32)


def round_bf16(x):
    return bf16_to_f32((torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(torch.bfloat16)
                        .view(torch.int16).numpy().view(np.uint16)))


def slot_values(feats, h, n_slots, slot_fn):
    """[n_slots, ncols] values lane half h supplies (0 for padding)."""
    out = np.zeros((n_slots, feats.shape[1]))
    for q in range(n_slots):
        f = slot_fn(h, q)
        if f >= 0:
            out[q] = feats[f]
    return out


def unpack_bias(prm, layer, nt):
    b = np.zeros(32 * nt)
    for o in range(nt):
        for h in range(2):
            for r in range(16):
                b[32 * o + acc_row(r, h)] = prm[256 * layer + (o * 2 + h) * 16 + r]
    return b


def heads(prm, x, hcol):
    """density and colour heads from the packed param blob (fp32 VALU path)."""
    sig_w, c1_w = np.zeros(256), np.zeros((3, 128))
    for h in range(2):
        for t in range(8):
            for r in range(16):
                sig_w[32 * t + acc_row(r, h)] = prm[2304 + (h * 8 + t) * 16 + r]
        for c in range(3):
            for t in range(4):
                for r in range(16):
                    c1_w[c, 32 * t + acc_row(r, h)] = prm[2564 + ((c * 2 + h) * 4 + t) * 16 + r]
    sigma = np.maximum(sig_w @ x + prm[2560], 0)
    rgb = 1 / (1 + np.exp(-(c1_w @ hcol + prm[2948:2951, None])))
    return sigma, rgb


# the original NeRF implementation's trunk (NERF_LAYOUT_ORIGINAL_NERF): the encoding re-enters at layer 5
LAYERS_ORIG = LAYERS[:4] + [("layers.4", 256, 256, None), ("layers.5", 256, 256, "pos")] + LAYERS[6:]


def emulate(f32_blob, bf16_blob, prm, pe, dpe, precision, layers=LAYERS):
    """Run the packed network the way the kernels' lane maps do.  pe [63, n], dpe [27, n]."""
    n = pe.shape[1]
    x = None
    off_f32, off_bf16 = 0, 0
    for li, (_, out, hidden, extra) in enumerate(layers):
        nt = out // 32
        n_ext = {"pos": 32, "dir": 16, None: 0}[extra]
        ext = [None, None]
        if extra:
            feats, fn = (pe, pe_slot_feature) if extra == "pos" else (dpe, dpe_slot_feature)
            ext = [slot_values(feats, h, n_ext, fn) for h in range(2)]
        acc = np.tile(unpack_bias(prm, li, nt)[:, None], (1, n))
        if precision == "fp32":
            ku = hidden // 2 + n_ext
            a = f32_blob[off_f32: off_f32 + ku * nt * 64].reshape(ku // 4, nt, 2, 32, 4)
            off_f32 += ku * nt * 64
            a = a.transpose(0, 4, 1, 2, 3).reshape(ku, nt, 2, 32)          # [u, o, k(h), i]
            for u in range(ku):
                for h in range(2):
                    if u < hidden // 2:
                        b = x[32 * (u >> 4) + acc_row(u & 15, h)]
                    else:
                        b = ext[h][u - hidden // 2]
                    acc += np.einsum("oi,j->oij", a[u, :, h], b).reshape(32 * nt, n)
        else:
            ku = hidden // 16 + n_ext // 8
            raw = bf16_blob[off_bf16: off_bf16 + ku * nt * 512]
            off_bf16 += ku * nt * 512
            # stream order [quarter q][u][tile-in-quarter][lane][8] -> [u, o, h, i, j]
            a = bf16_to_f32(raw).reshape(nt // 2, ku, 2, 2, 32, 8).transpose(1, 0, 2, 3, 4, 5)
            a = a.reshape(ku, nt, 2, 32, 8)
            xr = None if x is None else round_bf16(x)
            for u in range(ku):
                for h in range(2):
                    for j in range(8):
                        if u < hidden // 16:
                            b = xr[32 * (u >> 1) + 16 * (u & 1) + 8 * (j >> 2) + 4 * h + (j & 3)]
                        else:
                            b = round_bf16(ext[h][8 * (u - hidden // 16) + j])
                        acc += np.einsum("oi,j->oij", a[u, :, h, :, j], b).reshape(32 * nt, n)
        acc = np.maximum(acc, 0)
        if li == 7:
            x7 = acc
        x = acc
    if precision == "fp32":
        return heads(prm, x7, x)
    # bf16: the heads run as one MFMA tile from the head units (nerf_layout.h)
    raw = bf16_blob[516 * 1024: (516 + 12) * 1024]
    a = bf16_to_f32(raw).reshape(24, 2, 32, 8)                      # [k-step][half][row][j]
    x7r, xr = round_bf16(x7), round_bf16(x)
    out = np.zeros((4, n))
    for u in range(24):
        for h in range(2):
            for j in range(8):
                if u < 16:
                    b = x7r[32 * (u >> 1) + 16 * (u & 1) + 8 * (j >> 2) + 4 * h + (j & 3)]
                else:
                    v = u - 16
                    b = xr[32 * (v >> 1) + 16 * (v & 1) + 8 * (j >> 2) + 4 * h + (j & 3)]
                out += np.outer(a[u, h, :4, j], b)
    sigma = np.maximum(out[3] + prm[2560], 0)
    rgb = 1 / (1 + np.exp(-(out[:3] + prm[2948:2951, None])))
    return sigma, rgb


def direct(sd, pe, dpe, rnd):
    """Plain restatement with the precision's rounding applied at MFMA inputs."""
    x = pe
    for i in range(8):
        if i == 4:
            x = np.concatenate([x, pe])
        x = np.maximum(rnd(sd[f"layers.{i}.weight"]).astype(np.float64) @ rnd(x) + sd[f"layers.{i}.bias"][:, None], 0)
    sigma = np.maximum(rnd(sd["density_head.weight"]).astype(np.float64) @ rnd(x) + sd["density_head.bias"][:, None], 0)[0]
    hcol = np.maximum(rnd(sd["color_layers.0.weight"]).astype(np.float64) @ rnd(np.concatenate([x, dpe]))
                      + sd["color_layers.0.bias"][:, None], 0)
    rgb = 1 / (1 + np.exp(-(rnd(sd["color_layers.1.weight"]).astype(np.float64) @ rnd(hcol)
                            + sd["color_layers.1.bias"][:, None])))
    return sigma, rgb


@pytest.fixture(scope="module")
def packed():
    sd = W.synthetic_state_dict(1)
    return sd, rt.pack_weights(sd)


@pytest.fixture(scope="module")
def samples(golden):
    g = golden("mlp")
    idx = np.linspace(0, g["pos"].shape[0] - 1, 24).astype(int)
    pos, dirs = torch.from_numpy(g["pos"][idx]), torch.from_numpy(g["dirs"][idx])
    return (O.positional_encoding(pos, 10).numpy().T.astype(np.float64),
            O.positional_encoding(dirs, 4).numpy().T.astype(np.float64), g, idx)


def test_packed_sizes():
    sd = W.synthetic_state_dict(1)
    f32, bf, prm = rt.pack_weights(sd)
    assert f32.size * 4 == 8 * 0 + sum(((h // 2 + {"pos": 32, "dir": 16, None: 0}[e]) * (o // 32) * 64 * 4)
                                       for _, o, h, e in LAYERS)
    assert bf.size * 2 == 544 * 2048          # 516 units padded to a multiple of 32
    assert prm.size == 2952


def test_fp32_packing_computes_the_mlp(packed, samples):
    sd, (f32, bf, prm) = packed
    pe, dpe, _, _ = samples
    s_emu, rgb_emu = emulate(f32, bf, prm, pe, dpe, "fp32")
    s_dir, rgb_dir = direct(sd, pe, dpe, lambda a: np.asarray(a, np.float64))
    np.testing.assert_allclose(s_emu, s_dir, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(rgb_emu, rgb_dir, rtol=1e-9, atol=1e-9)


def test_bf16_packing_computes_the_mlp(packed, samples):
    sd, (f32, bf, prm) = packed
    pe, dpe, _, _ = samples
    s_emu, rgb_emu = emulate(f32, bf, prm, pe, dpe, "bf16")
    s_dir, rgb_dir = direct(sd, pe, dpe, lambda a: round_bf16(a).astype(np.float64))
    np.testing.assert_allclose(s_emu, s_dir, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(rgb_emu, rgb_dir, rtol=1e-6, atol=1e-6)


def test_fp32_emulation_matches_reference_golden(samples):
    """The packed fine net through the emulated lane maps reproduces the reference's outputs."""
    pe, dpe, g, idx = samples
    c, f = W.synthetic_models(0)
    f32, bf, prm = rt.pack_weights(f)
    s_emu, rgb_emu = emulate(f32, bf, prm, pe, dpe, "fp32")
    np.testing.assert_allclose(s_emu, g["sigma_fine"][idx, 0], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(rgb_emu.T, g["rgb_fine"][idx], rtol=0, atol=1e-6)


# ------------------------------------------------------------------ fp8 path --
def e4m3_round(x):
    """torch's f32 -> float8_e4m3fn (RNE) and back."""
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(torch.float8_e4m3fn).float().numpy().astype(np.float64)


def e4m3_decode(codes):
    return torch.from_numpy(np.ascontiguousarray(codes, np.uint8)).view(torch.float8_e4m3fn).float().numpy()


def test_f32_to_e4m3_matches_torch():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(20000) * s for s in (1e-3, 0.05, 1, 30, 150)]).astype(np.float32)
    x = np.concatenate([x, [0.0, -0.0, 448.0, -448.0, 2.0 ** -9, 2.0 ** -10, 3 * 2.0 ** -10, 2.0 ** -6, 1.0625,
                            1.1875, 240.0, 232.0, 447.9]]).astype(np.float32)
    x = np.clip(x, -448, 448)
    ours = rt.f32_to_e4m3(x)
    ref = torch.from_numpy(x).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    assert np.array_equal(ours, ref)


def test_fp8_activation_round_saturates():
    """The fp8 activation contract (mlp_fp8.hip convert_tile, oracle.fp8_activation_round):
    ReLU and a clamp at 448 (v_med3_f32), then e4m3 RNE at scale 1 -- never NaN."""
    x = np.array([-3.0, -0.0, 0.0, 2.0 ** -10, 3 * 2.0 ** -10, 0.3, 1.0625, 447.9, 448.0, 464.0, 1e4, 3e38],
                 np.float32)
    got = O.fp8_activation_round(x)
    assert np.isfinite(got).all()
    assert np.array_equal(got, [0.0, 0.0, 0.0, 0.0, 2.0 ** -8, 0.3125, 1.0, 448.0, 448.0, 448.0, 448.0, 448.0])


FP8_UNITS, FP8_LAYER_UNITS = 168, 162          # nerf_layout.h kMixUnits, kMixLayerUnits
FP8_BF16 = {0, 1, 8}                           # L0, L1, C0 on the bf16 MFMA (mlp_fp8.hip, round 5)


def hid_bf16(u, h, j):
    return 32 * (u >> 1) + 16 * (u & 1) + 8 * (j >> 2) + 4 * h + (j & 3)


def emulate_fp8(blob, prm, pe, dpe):
    """Kernel lane maps of the mixed fp8 path (nerf_layout.h "fp8, mixed"), float64
    accumulation: per layer and quarter the fp8 units ([o2][p][lane][16 B] e4m3, the row's
    E8M0 scale), then the bf16 units ([s][o2][lane][8 bf16], two k-steps), then the six head
    units ([k][lane][8 bf16])."""
    n = pe.shape[1]
    scales = blob[FP8_UNITS * 4096:].view(np.uint32).reshape(10, 4, 64, 2)
    units = blob[:FP8_UNITS * 4096].reshape(FP8_UNITS, 4096)
    ext_all = {"pos": [round_bf16(slot_values(pe, h, 32, pe_slot_feature)) for h in range(2)],
               "dir": [round_bf16(slot_values(dpe, h, 16, dpe_slot_feature)) for h in range(2)]}
    nu = 0
    x = x7 = None
    for li, (_, out, hidden, extra) in enumerate(LAYERS):
        nt, nq = out // 32, out // 64
        bf = li in FP8_BF16
        n_ext = {"pos": 4, "dir": 2, None: 0}[extra]
        nf = 0 if bf else hidden // 64
        nb = (hidden // 16 + n_ext) // 2 if bf else n_ext // 2
        kh = hidden // 16
        acc = np.tile(unpack_bias(prm, li, nt)[:, None], (1, n))
        xq = None if x is None else O.fp8_activation_round(x)
        xb = None if x is None else round_bf16(np.maximum(x, 0))
        for q in range(nq):
            for u in range(nf):
                a = e4m3_decode(units[nu]).reshape(2, 2, 64, 16).transpose(0, 2, 1, 3).reshape(2, 64, 32)
                nu += 1
                for o2 in range(2):
                    for lane in range(64):
                        r, h = lane & 31, lane >> 5
                        sc = np.ldexp(1.0, int(scales[li, q, lane, o2] & 0xFF) - 127)
                        b = xq[[32 * (2 * u + (j >> 4)) + acc_row(j & 15, h) for j in range(32)]]
                        acc[32 * (2 * q + o2) + r] += sc * (a[o2, lane].astype(np.float64) @ b)
            for ub in range(nb):
                a = bf16_to_f32(units[nu].view(np.uint16)).reshape(2, 2, 64, 8)          # [s][o2][lane][j]
                nu += 1
                for sk in range(2):
                    ks = (0 if bf else kh) + 2 * ub + sk
                    for lane in range(64):
                        r, h = lane & 31, lane >> 5
                        if ks < kh:
                            b = xb[[hid_bf16(ks, h, j) for j in range(8)]]
                        else:
                            e = ks - kh
                            b = ext_all[extra][h][8 * e: 8 * e + 8]
                        for o2 in range(2):
                            acc[32 * (2 * q + o2) + r] += a[sk, o2, lane].astype(np.float64) @ b
        x = acc
        if li == 7:
            x7 = acc
    assert nu == FP8_LAYER_UNITS
    # heads: one bf16 tile, k-steps 0..15 density over L7's output, 16..23 colour over C0's
    a = bf16_to_f32(units[FP8_LAYER_UNITS:].view(np.uint16)).reshape(24, 64, 8)          # [k-step][lane][j]
    x7b, xcb = round_bf16(np.maximum(x7, 0)), round_bf16(np.maximum(x, 0))
    out = np.zeros((4, n))
    for u in range(24):
        src, v = (x7b, u) if u < 16 else (xcb, u - 16)
        for lane in range(64):
            r, h = lane & 31, lane >> 5
            if r < 4:
                out[r] += a[u, lane].astype(np.float64) @ src[[hid_bf16(v, h, j) for j in range(8)]]
    return np.maximum(out[3] + prm[2560], 0), 1 / (1 + np.exp(-(out[:3] + prm[2948:2951, None])))


def test_fp8_packing_computes_the_mlp(samples):
    pe, dpe, _, _ = samples
    sd = W.synthetic_state_dict(1)
    blob = rt.pack_weights_fp8(sd)
    _, _, prm = rt.pack_weights(sd)
    assert blob.size == FP8_UNITS * 4096 + 10 * 4 * 64 * 2 * 4
    s_emu, rgb_emu = emulate_fp8(blob, prm, pe[:, :6], dpe[:, :6])
    s_dir, rgb_dir = O.fp8_mlp_restated(sd, pe[:, :6], dpe[:, :6], chain=False)
    np.testing.assert_allclose(s_emu, s_dir, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(rgb_emu, rgb_dir, rtol=1e-6, atol=1e-6)


# ---------------------------------------------------------- split-bf16 path --
def test_bf16x3_packing_splits_the_bf16_stream():
    """nerf_pack_weights_bf16x3: unit n of the split blob is the bf16 blob's unit n
    rounded (W_hi, bit-identical to the bf16 packing) followed by the rounded
    remainder (W_lo = bf16(W - W_hi)); hi + lo carries W to 2^-16 relative."""
    sd = W.synthetic_state_dict(2)
    _, bf, _ = rt.pack_weights(sd)
    x3 = rt.pack_weights_bf16x3(sd)
    unit = 1024                                        # bf16 elements per 2 KiB unit
    n_units = bf.size // unit
    assert x3.size == 2 * bf.size
    u3 = x3.reshape(n_units, 2, unit)
    assert np.array_equal(u3[:, 0], bf.reshape(n_units, unit))
    hi, lo = bf16_to_f32(u3[:, 0]), bf16_to_f32(u3[:, 1])
    # the fp32 values of the stream, from the fp32 packing of the same weights
    # through the hi/lo identity: |W - (hi + lo)| <= 2^-17 |W| (lo is RNE of an exact remainder)
    w_rec = hi.astype(np.float64) + lo
    nz = hi != 0
    rel = np.abs(lo[nz] / hi[nz])
    assert rel.max() <= 2.0 ** -8 + 1e-12                # a remainder is below half a bf16 ulp of hi
    assert np.all(np.isfinite(w_rec))
    # every non-padding weight of the network appears with its split in the blob
    flat = np.concatenate([sd[f"layers.{i}.weight"].ravel() for i in range(8)])
    hi_w = round_bf16(flat).astype(np.float64)
    lo_w = round_bf16((flat.astype(np.float64) - hi_w).astype(np.float32))
    recon = set(np.round((hi_w + lo_w) * 2 ** 30).astype(np.int64).tolist())
    got = set(np.round(w_rec[nz] * 2 ** 30).astype(np.int64).tolist())
    assert recon <= got | {0}


def test_f16x3_packing_splits_and_refuses_out_of_range():
    """nerf_pack_weights_f16x3: the same unit layout as the split-bf16 blob with fp16 halves,
    hi = f16(w), lo = f16(w - hi), so hi + lo carries w to ~2^-22; a weight outside fp16's
    range (65504) is refused with NERF_E_INVALID (the loader then leaves NERF_F16X3
    unavailable for that network)."""
    sd = W.synthetic_state_dict(2)
    x3 = rt.pack_weights_f16x3(sd)
    unit = 1024
    n_units = x3.size // (2 * unit)
    u3 = x3.reshape(n_units, 2, unit)
    hi = u3[:, 0].view(np.float16).astype(np.float64)
    lo = u3[:, 1].view(np.float16).astype(np.float64)
    assert np.all(np.isfinite(hi)) and np.all(np.isfinite(lo))
    nz = hi != 0
    assert np.abs(lo[nz] / hi[nz]).max() <= 2.0 ** -11 + 1e-12     # below half an fp16 ulp of hi
    # every layer weight is reproduced by hi + lo to fp16x2 precision
    flat = np.concatenate([sd[f"layers.{i}.weight"].ravel() for i in range(8)]).astype(np.float64)
    rec = np.sort((hi + lo)[nz].ravel())
    idx = np.clip(np.searchsorted(rec, flat), 1, rec.size - 1)
    near = np.minimum(np.abs(rec[idx] - flat), np.abs(rec[idx - 1] - flat))
    assert near.max() <= 2.0 ** -22 * np.abs(flat).max()
    # out of range: refused, and the message says why
    bad = dict(sd)
    bad["layers.3.weight"] = sd["layers.3.weight"].copy()
    bad["layers.3.weight"][5, 7] = np.float32(7e4)
    with pytest.raises(rt.NerfError, match="fp16 range"):
        rt.pack_weights_f16x3(bad)


def synthetic_original_nerf(seed=0):
    """24 arrays in the original NeRF implementation's layout ([in, out] kernels; SURVEY §8f
    row 1), He-scaled so activations stay O(1)."""
    rng = np.random.default_rng(seed)
    shapes = ([(63, 256)] + [(256, 256)] * 4 + [(319, 256)] + [(256, 256)] * 2
              + [(256, 256), (283, 128), (128, 3), (256, 1)])
    out = []
    for fan_in, fan_out in shapes:
        out += [rng.normal(0, np.sqrt(2.0 / fan_in), (fan_in, fan_out)), rng.normal(0, 0.05, fan_out)]
    return [a.astype(np.float32) for a in out]


def original_nerf_direct(a, x, d):
    """The original network in float64 (the restatement of tools/lego/teacher.py): encodings
    sin(2^k x) without pi, skip cat([pe, h]) into layer 5, normalised view directions, a linear
    feature layer before the views layer.  x, d [n, 3] -> sigma [n], rgb [3, n]."""
    a = [np.asarray(v, np.float64) for v in a]

    def embed(v, L):
        return np.concatenate([v] + [f(v * 2.0 ** k) for k in range(L) for f in (np.sin, np.cos)], -1)

    pe = embed(x, 10)
    ve = embed(d / np.linalg.norm(d, axis=-1, keepdims=True), 4)
    h = pe
    for i in range(8):
        h = np.maximum(h @ a[2 * i] + a[2 * i + 1], 0)
        if i == 4:
            h = np.concatenate([pe, h], -1)
    sigma = np.maximum(h @ a[22] + a[23], 0)[:, 0]
    feat = h @ a[16] + a[17]
    h2 = np.maximum(np.concatenate([feat, ve], -1) @ a[18] + a[19], 0)
    return sigma, (1 / (1 + np.exp(-(h2 @ a[20] + a[21])))).T


def test_original_nerf_layout_packing_computes_the_network():
    """NERF_LAYOUT_ORIGINAL_NERF (the optional second weight layout): the host
    transform (layer 5's columns re-ordered to [h, pe], the feature layer folded into colour 0 in
    float64) and the packer's skip-at-layer-5 f32 blob, pushed through the fp32 kernel's lane maps
    with the no-pi encodings of normalised directions, compute the original network."""
    arrays = synthetic_original_nerf(3)
    f32, prm = rt.pack_weights_original_nerf(arrays)
    rng = np.random.default_rng(4)
    x = rng.uniform(-1.2, 1.2, (20, 3))
    d = rng.normal(0, 1, (20, 3)) * rng.uniform(0.5, 2.0, (20, 1))      # raw, unnormalised rays_d

    def embed(v, L):
        return np.concatenate([v] + [f(v * 2.0 ** k) for k in range(L) for f in (np.sin, np.cos)], -1)

    pe = embed(x, 10).T
    dpe = embed(d / np.linalg.norm(d, axis=-1, keepdims=True), 4).T
    s_emu, rgb_emu = emulate(f32, None, prm, pe, dpe, "fp32", LAYERS_ORIG)
    s_dir, rgb_dir = original_nerf_direct(arrays, x, d)
    assert np.abs(s_dir).max() > 1e-2 and rgb_dir.std() > 1e-3              # a non-degenerate network
    np.testing.assert_allclose(s_emu, s_dir, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(rgb_emu, rgb_dir, rtol=1e-5, atol=1e-5)
    # the NeRFModel layout of the same blob sizes: the two layouts differ exactly in layers 4 and 5
    assert f32.size == rt.pack_weights(W.synthetic_state_dict(1))[0].size
