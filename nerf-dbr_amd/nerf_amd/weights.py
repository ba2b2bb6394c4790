"""NeRF weight schema, checkpoint I/O and the deterministic synthetic checkpoint.

The network is the reference's ``NeRFModel`` (``src/models/nerf.py:48-131``):
eight 256-wide trunk layers with the positional encoding re-injected before
layer 4 (``nerf.py:107-110``), a 1-wide density head (``nerf.py:84,114``) and a
two-layer colour head fed with ``[x, PE4(d)]`` (``nerf.py:87-90,117-129``).
Weights are stored exactly as ``nn.Linear`` stores them: ``weight`` is
``[out, in]`` row-major fp32, ``bias`` is ``[out]``.

Checkpoints use the reference trainer's dict layout
(``src/training/trainer.py:376-384``): ``{'coarse_model': state_dict,
'fine_model': state_dict, ...}``; renderers only read the two model entries
(``src/benchmark/base_renderer.py:42-48``).  Unlike the reference
(``base_renderer.py:42``, ``weights_only=False``) checkpoints are loaded with
``torch.load(weights_only=True)``: nothing in a checkpoint file is executed.

The reference ships no trained checkpoint in this layout, and a randomly
initialised net renders an all-black image.  Two checkpoints are provided: the
Lego checkpoint (``lego_models``: the reference's bundled original-NeRF Lego
networks distilled into this layout, see ``LEGO_NPZ``), and ``synthetic_state_dict``, a
*conditioned* random net instead: ``nn.Linear``'s default
init distribution (U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for weight and bias) drawn
from numpy's legacy ``RandomState`` (a stream numpy keeps stable across
releases), then trunk weights x2, density weight x30, density bias = 0.2 and
the last colour weight x8, so images have real structure and depth.
"""
from __future__ import annotations

import hashlib
import os
from typing import Dict, List, Mapping, Tuple

import numpy as np

POS_L = 10            # nerf.py:50 (pos_L default)
DIR_L = 4             # nerf.py:50 (dir_L default)
HIDDEN = 256          # nerf.py:50 (hidden_dim default)
POS_DIM = 3 + 3 * 2 * POS_L   # 63 (nerf.py:64 comment says 60; it is 63)
DIR_DIM = 3 + 3 * 2 * DIR_L   # 27
SKIP_LAYER = 4                # nerf.py:108 (`if i == 4`)

# (state-dict prefix, out_features, in_features) in forward order (nerf.py:72-90)
LAYER_SPECS: List[Tuple[str, int, int]] = (
    [("layers.0", HIDDEN, POS_DIM)]
    + [(f"layers.{i}", HIDDEN, HIDDEN) for i in (1, 2, 3)]
    + [("layers.4", HIDDEN, HIDDEN + POS_DIM)]
    + [(f"layers.{i}", HIDDEN, HIDDEN) for i in (5, 6, 7)]
    + [("density_head", 1, HIDDEN),
       ("color_layers.0", HIDDEN // 2, HIDDEN + DIR_DIM),
       ("color_layers.1", 3, HIDDEN // 2)]
)

N_PARAMS = sum(o * i + o for _, o, i in LAYER_SPECS)          # 530,052
# multiply-accumulates per sample: every Linear, unpadded
MACS_PER_SAMPLE = sum(o * i for _, o, i in LAYER_SPECS)       # 527,872
FLOPS_PER_SAMPLE = 2 * MACS_PER_SAMPLE                        # 1,055,744

StateDict = Dict[str, np.ndarray]


def expected_shapes() -> Dict[str, Tuple[int, ...]]:
    out: Dict[str, Tuple[int, ...]] = {}
    for name, o, i in LAYER_SPECS:
        out[f"{name}.weight"] = (o, i)
        out[f"{name}.bias"] = (o,)
    return out


def validate_state_dict(sd: Mapping[str, np.ndarray]) -> None:
    """Strict key/shape check, the same contract as ``load_state_dict(strict=True)``."""
    exp = expected_shapes()
    missing = sorted(set(exp) - set(sd))
    unexpected = sorted(set(sd) - set(exp))
    if missing or unexpected:
        raise KeyError(f"state_dict mismatch: missing={missing} unexpected={unexpected}")
    for k, shape in exp.items():
        if tuple(sd[k].shape) != shape:
            raise ValueError(f"state_dict[{k!r}] has shape {tuple(sd[k].shape)}, expected {shape}")


def synthetic_state_dict(seed: int, conditioned: bool = True) -> StateDict:
    """Deterministic NeRFModel weights (see module docstring)."""
    rng = np.random.RandomState(seed)
    sd: StateDict = {}
    for name, o, i in LAYER_SPECS:
        bound = 1.0 / np.sqrt(i)
        sd[f"{name}.weight"] = rng.uniform(-bound, bound, size=(o, i)).astype(np.float32)
        sd[f"{name}.bias"] = rng.uniform(-bound, bound, size=(o,)).astype(np.float32)
    if conditioned:
        for li in range(8):
            sd[f"layers.{li}.weight"] *= np.float32(2.0)
        sd["density_head.weight"] *= np.float32(30.0)
        sd["density_head.bias"][:] = np.float32(0.2)
        sd["color_layers.1.weight"] *= np.float32(8.0)
    return sd


def synthetic_models(seed: int = 0, conditioned: bool = True) -> Tuple[StateDict, StateDict]:
    """(coarse, fine) state dicts: coarse from ``seed``, fine from ``seed + 1``."""
    return synthetic_state_dict(seed, conditioned), synthetic_state_dict(seed + 1, conditioned)


def state_dict_digest(sd: Mapping[str, np.ndarray]) -> str:
    h = hashlib.sha256()
    for name, _, _ in LAYER_SPECS:
        for suffix in ("weight", "bias"):
            h.update(np.ascontiguousarray(sd[f"{name}.{suffix}"], dtype=np.float32).tobytes())
    return h.hexdigest()


def _to_numpy(sd) -> StateDict:
    out: StateDict = {}
    for k, v in sd.items():
        if hasattr(v, "detach"):
            v = v.detach().cpu().numpy()
        out[k] = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
    return out


def save_checkpoint(path: str, coarse: Mapping[str, np.ndarray], fine: Mapping[str, np.ndarray]) -> str:
    """Write a reference-format checkpoint (``trainer.py:376-384``, model entries only)."""
    import torch

    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    ckpt = {
        "coarse_model": {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in coarse.items()},
        "fine_model": {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in fine.items()},
    }
    torch.save(ckpt, path)
    return path


def torch_load_weights_only(path: str):
    """``torch.load(path, weights_only=True)`` that also admits numpy scalars.

    The reference trainer stores its loss histories as ``np.float64`` values (they
    come from ``np.mean``, ``src/training/trainer.py:336-345``), which the plain
    weights-only unpickler refuses.  The scalar constructor and the float / int
    dtype classes are added to its allowlist, under both the numpy-2 module path
    and the ``numpy.core`` path older numpy writes; this admits data only, nothing
    that executes."""
    import torch

    try:
        import numpy._core.multiarray as ma
    except ImportError:                                   # numpy < 2
        import numpy.core.multiarray as ma
    safe = [ma.scalar, (ma.scalar, "numpy.core.multiarray.scalar"), np.dtype]
    for name in ("Float64DType", "Float32DType", "Int64DType", "Int32DType"):
        cls = getattr(getattr(np, "dtypes", None), name, None)
        if cls is not None:
            safe.append(cls)
    with torch.serialization.safe_globals(safe):
        return torch.load(path, map_location="cpu", weights_only=True)


def load_checkpoint(path: str) -> Tuple[StateDict, StateDict]:
    """Load ``(coarse, fine)`` from a reference-format checkpoint.

    Raises ``FileNotFoundError`` when the file is missing: unlike the reference
    (``base_renderer.py:62-76``) there is no silent random-weight fallback.
    """
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    if path.endswith(".npz"):              # the raw-array form (lego_distilled.npz)
        return lego_models(path)
    ckpt = torch_load_weights_only(path)
    coarse, fine = _to_numpy(ckpt["coarse_model"]), _to_numpy(ckpt["fine_model"])
    validate_state_dict(coarse)
    validate_state_dict(fine)
    return coarse, fine


def write_synthetic_checkpoint(path: str, seed: int = 0) -> str:
    coarse, fine = synthetic_models(seed)
    return save_checkpoint(path, coarse, fine)


# The Lego checkpoint: the reference's bundled original-NeRF Lego networks
# (data/lego_example_weights/model{_fine,}_200000.npy) distilled into this layout by
# tools/lego/distill.py (recipe, held-out PSNR vs the teacher: lego_distilled.json beside
# it).  Raw fp32 arrays, no pickle: keys "coarse/<param>" and "fine/<param>".
LEGO_NPZ = os.path.join(os.path.dirname(os.path.abspath(__file__)), "checkpoints", "lego_distilled.npz")


def lego_models(path: str = LEGO_NPZ) -> Tuple[StateDict, StateDict]:
    """(coarse, fine) state dicts of the distilled Lego checkpoint."""
    z = np.load(path, allow_pickle=False)
    out = []
    for net in ("coarse", "fine"):
        sd = {k.split("/", 1)[1]: np.ascontiguousarray(z[k], dtype=np.float32) for k in z.files
              if k.startswith(net + "/")}
        validate_state_dict(sd)
        out.append(sd)
    return out[0], out[1]


def write_lego_checkpoint(path: str) -> str:
    """The distilled Lego checkpoint in the reference trainer's format (model entries)."""
    coarse, fine = lego_models()
    return save_checkpoint(path, coarse, fine)


# ------------------------------------------------ the original NeRF layout --
def original_nerf_tensors(arrays) -> List[np.ndarray]:
    """The 24 arrays of the original NeRF implementation's network (the reference's bundled
    Lego weights, ``data/lego_example_weights/model*_200000.npy``, read by
    ``tools/lego/npy_static.py``) -> the 22 tensors
    ``nerf_ctx_load_weights_layout(..., NERF_LAYOUT_ORIGINAL_NERF, ...)`` takes
    (include/nerf_mi355x.h), in NeRFModel's order and ``[out, in]`` orientation:

    * trunk layer i: ``arrays[2i].T``, ``arrays[2i+1]`` -- layer 4 is [256, 256] and layer 5,
      whose input is ``cat([pe, h])`` in the original, is [256, 319] with its columns
      re-ordered to ``[h, pe]`` (exact);
    * the density head: ``arrays[22].T``, ``arrays[23]`` (alpha, ReLU'd by the renderer);
    * colour 0: the views layer with the feature layer (linear, no activation) folded in,
      ``[W_v[:, :256] @ W_f | W_v[:, 256:]]`` and ``W_v[:, :256] @ b_f + b_v`` computed in
      float64 and rounded once;
    * colour 1: the rgb layer ``arrays[20].T``, ``arrays[21]``."""
    a = [np.asarray(x, dtype=np.float64) for x in arrays]
    if len(a) != 24 or a[10].shape != (HIDDEN + POS_DIM, HIDDEN) or a[22].shape != (HIDDEN, 1):
        raise ValueError("not the original-NeRF 8x256 layout (24 arrays, skip into layer 5)")
    out: List[np.ndarray] = []
    for i in range(8):
        w = a[2 * i].T
        if i == 5:   # [pe(63), h(256)] -> [h, pe]
            w = np.concatenate([w[:, POS_DIM:], w[:, :POS_DIM]], axis=1)
        out += [w, a[2 * i + 1]]
    out += [a[22].T, a[23]]
    w_f, b_f, w_v, b_v = a[16].T, a[17], a[18].T, a[19]
    out += [np.concatenate([w_v[:, :HIDDEN] @ w_f, w_v[:, HIDDEN:]], axis=1), w_v[:, :HIDDEN] @ b_f + b_v]
    out += [a[20].T, a[21]]
    return [np.ascontiguousarray(x, dtype=np.float32) for x in out]
