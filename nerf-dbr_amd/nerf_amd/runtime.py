"""ctypes binding of libnerf_mi355x.so (C ABI: include/nerf_mi355x.h).

The library is built in-tree (``nerf-dbr_amd/csrc/Makefile`` ->
``nerf_amd/_lib/libnerf_mi355x.so``).  There is no CPU or PyTorch fallback:
if the library is missing or no gfx950 device is present, constructing a
``Device`` raises ``RuntimeError`` (the exception type the reference's suite
probes renderers with, ``src/benchmark/benchmark_suite.py:80-92``).

Tensors cross the boundary as raw device pointers (``tensor.data_ptr()``) and
the HIP stream as ``torch.cuda.current_stream().cuda_stream``; PyTorch is only
the device-memory and stream plumbing here.
"""
from __future__ import annotations

import ctypes
import os
from typing import Mapping, Optional, Sequence

import numpy as np

from .weights import LAYER_SPECS, validate_state_dict

LIB_NAME = "libnerf_mi355x.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", LIB_NAME)

NERF_OK = 0
NERF_FP32, NERF_BF16, NERF_FP8, NERF_BF16X3, NERF_F16X3 = 0, 1, 2, 3, 4
NERF_NET_COARSE, NERF_NET_FINE = 0, 1
NERF_N_PARAMS = 22
NERF_N_STAGES = 5
NERF_OPT_FUSED_COMPOSITE = 1
NERF_OPT_COARSE_PRECISION = 2
NERF_LAYOUT_NERFMODEL, NERF_LAYOUT_ORIGINAL_NERF = 0, 1
STAGES = ("rays", "coarse_mlp", "importance", "fine_mlp", "composite")

PRECISIONS = {"fp32": NERF_FP32, "bf16": NERF_BF16, "fp8": NERF_FP8, "bf16x3": NERF_BF16X3, "f16x3": NERF_F16X3}

# Every symbol include/nerf_mi355x.h declares, with its ctypes signature.
_c = ctypes
_P = _c.c_void_p
_FP = _c.POINTER(_c.c_float)
SIGNATURES = {
    "nerf_abi_version": (_c.c_int, []),
    "nerf_last_error": (_c.c_char_p, []),
    "nerf_ctx_create": (_c.c_int, [_c.c_int, _c.POINTER(_P)]),
    "nerf_ctx_destroy": (None, [_P]),
    "nerf_device_name": (_c.c_int, [_c.c_int, _c.c_char_p, _c.c_int]),
    "nerf_ctx_load_weights": (_c.c_int, [_P, _c.c_int, _c.POINTER(_FP), _c.c_int]),
    "nerf_ctx_load_weights_layout": (_c.c_int, [_P, _c.c_int, _c.c_int, _c.POINTER(_FP), _c.c_int]),
    "nerf_pack_weights_layout": (_c.c_int, [_c.POINTER(_FP), _c.c_int, _c.c_int, _P, _P, _P]),
    "nerf_packed_sizes": (None, [_c.POINTER(_c.c_size_t)] * 3),
    "nerf_pack_weights": (_c.c_int, [_c.POINTER(_FP), _c.c_int, _P, _P, _P]),
    "nerf_uniform_z": (None, [_FP, _c.c_int, _c.c_float, _c.c_float, _FP]),
    "nerf_fp8_blob_bytes": (_c.c_size_t, []),
    "nerf_pack_weights_fp8": (_c.c_int, [_c.POINTER(_FP), _c.c_int, _P]),
    "nerf_f32_to_e4m3": (None, [_FP, _c.c_int, _P]),
    "nerf_generate_rays": (_c.c_int, [_P, _FP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_float, _P, _P, _P]),
    "nerf_mlp_forward": (_c.c_int, [_P, _c.c_int, _c.c_int, _P, _P, _P, _c.c_int, _c.c_int, _c.c_int, _P, _P]),
    "nerf_query": (_c.c_int, [_P, _c.c_int, _c.c_int, _P, _P, _c.c_int, _P, _P]),
    "nerf_composite": (_c.c_int, [_P, _c.c_int, _P, _c.c_int, _P, _c.c_int, _P, _c.c_int, _c.c_int,
                                  _P, _P, _P, _P, _P]),
    "nerf_importance_sample": (_c.c_int, [_P, _c.c_int, _P, _P, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P, _P]),
    "nerf_render": (_c.c_int, [_P, _FP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_float, _c.c_float,
                               _c.c_float, _FP, _c.c_int, _c.c_int, _FP, _c.c_int, _P, _P, _P]),
    "nerf_render_sampled": (_c.c_int, [_P, _FP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_float, _c.c_float,
                                       _c.c_float, _FP, _c.c_int, _c.c_int, _FP, _P, _P, _c.c_int, _P, _P, _P]),
    "nerf_sample_points": (_c.c_int, [_P, _P, _P, _c.c_int, _FP, _c.c_int, _c.c_float, _c.c_float, _P, _P, _P,
                                      _P]),
    "nerf_ctx_set_profiling": (_c.c_int, [_P, _c.c_int]),
    "nerf_ctx_stage_ms": (_c.c_int, [_P, _FP]),
    "nerf_ctx_set_option": (_c.c_int, [_P, _c.c_int, _c.c_int]),
    "nerf_ctx_stage_ms_history": (_c.c_int, [_P, _c.c_int, _FP]),
    "nerf_render_band": (_c.c_int, [_P, _FP, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_float, _c.c_float,
                                    _c.c_float, _FP, _c.c_int, _c.c_int, _FP, _c.c_int, _P, _P]),
    "nerf_ctx_last_fine_z": (_c.c_int, [_P, _c.c_long, _c.c_int, _P, _P]),
    "nerf_ctx_range_status": (_c.c_int, [_P, _P]),
    "nerf_positional_encoding": (_c.c_int, [_c.c_int, _P, _c.c_long, _c.c_int, _P, _P]),
    "nerf_bf16x3_blob_bytes": (_c.c_size_t, []),
    "nerf_pack_weights_bf16x3": (_c.c_int, [_c.POINTER(_FP), _c.c_int, _P]),
    "nerf_pack_weights_f16x3": (_c.c_int, [_c.POINTER(_FP), _c.c_int, _P]),
    "nerf_linspace01": (None, [_c.c_int, _FP]),
    "nerf_trainer_create": (_c.c_int, [_c.c_int, _P, _c.POINTER(_FP), _c.POINTER(_FP), _c.c_int, _c.POINTER(_P)]),
    "nerf_trainer_destroy": (None, [_P]),
    "nerf_train_step": (_c.c_int, [_P, _P, _c.c_int, _c.c_int, _c.c_float, _FP, _P, _c.c_int, _P, _c.c_int, _P,
                                   _P]),
    "nerf_train_backward": (_c.c_int, [_P, _P, _c.c_int, _c.c_int, _c.c_float, _FP, _P, _c.c_int, _c.c_int, _P,
                                       _P, _P]),
    "nerf_trainer_set_grad_buffer": (_c.c_int, [_P, _P]),
    "nerf_trainer_read": (_c.c_int, [_P, _c.c_int, _c.c_int, _c.POINTER(_FP), _c.c_int]),
    "nerf_trainer_write_grads": (_c.c_int, [_P, _c.c_int, _c.POINTER(_FP), _c.c_int]),
    "nerf_trainer_write": (_c.c_int, [_P, _c.c_int, _c.c_int, _c.POINTER(_FP), _c.c_int]),
    "nerf_trainer_set_schedule": (_c.c_int, [_P, _c.c_long, _c.c_double]),
    "nerf_trainer_set_precision": (_c.c_int, [_P, _c.c_int]),
    "nerf_trainer_update": (_c.c_int, [_P, _P]),
    "nerf_trainer_lr": (_c.c_double, [_P]),
    "nerf_trainer_steps": (_c.c_long, [_P]),
    "nerf_trainer_set_profiling": (_c.c_int, [_P, _c.c_int]),
    "nerf_trainer_stage_ms": (_c.c_int, [_P, _FP]),
    "nerf_trainer_gemm_flops": (_c.c_double, [_P]),
}


class TrainConfig(_c.Structure):
    """nerf_train_config (include/nerf_mi355x.h)."""
    _fields_ = [("lr", _c.c_double), ("beta1", _c.c_double), ("beta2", _c.c_double), ("eps", _c.c_double),
                ("weight_decay", _c.c_double), ("lr_gamma", _c.c_double), ("grad_clip", _c.c_double),
                ("n_coarse", _c.c_int), ("n_fine", _c.c_int), ("near_", _c.c_float), ("far_", _c.c_float)]


NERF_TRAIN_NO_UPDATE = 1
NERF_TRAIN_NET_FLOATS = 530052
NERF_TR_PARAMS, NERF_TR_GRADS, NERF_TR_EXP_AVG, NERF_TR_EXP_AVG_SQ = 0, 1, 2, 3
NERF_TRAIN_N_STAGES = 6
TRAIN_STAGES = ("rays_encode", "forward_gemm", "render_heads", "backward_data_gemm", "weight_grad_gemm",
                "reduce_update")

_lib: Optional[ctypes.CDLL] = None


class NerfError(RuntimeError):
    pass


class NerfRangeError(NerfError, ArithmeticError):
    """NERF_E_RANGE: an NERF_F16X3 launch met an activation outside fp16's range."""


def library_path() -> str:
    return os.environ.get("NERF_MI355X_LIB", LIB_PATH)


def load_library() -> ctypes.CDLL:
    """Load and type the shared library (no device needed).  RuntimeError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not os.path.exists(path):
        raise NerfError(f"{LIB_NAME} not built at {path}; run `make -C nerf-dbr_amd/csrc` "
                        f"or __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


NERF_E_RANGE = -5


def _check(rc: int) -> None:
    if rc != NERF_OK:
        msg = load_library().nerf_last_error().decode(errors="replace")
        raise (NerfRangeError if rc == NERF_E_RANGE else NerfError)(f"libnerf_mi355x error {rc}: {msg}")


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(_FP)


def _param_list(sd: Mapping[str, np.ndarray]):
    validate_state_dict(sd)
    arrs = []
    for name, _, _ in LAYER_SPECS:
        for suffix in ("weight", "bias"):
            arrs.append(np.ascontiguousarray(sd[f"{name}.{suffix}"], dtype=np.float32))
    ptrs = (_FP * NERF_N_PARAMS)(*[_fptr(a) for a in arrs])
    return arrs, ptrs


def pack_weights(sd: Mapping[str, np.ndarray]):
    """Host-only packing (the same code the loader runs): (f32 blob, bf16 blob as uint16, params)."""
    lib = load_library()
    sizes = [ctypes.c_size_t() for _ in range(3)]
    lib.nerf_packed_sizes(*[ctypes.byref(s) for s in sizes])
    f32 = np.zeros(sizes[0].value // 4, np.float32)
    bf = np.zeros(sizes[1].value // 2, np.uint16)
    prm = np.zeros(sizes[2].value // 4, np.float32)
    keep, ptrs = _param_list(sd)
    _check(lib.nerf_pack_weights(ptrs, NERF_N_PARAMS, f32.ctypes.data_as(_P), bf.ctypes.data_as(_P),
                                 prm.ctypes.data_as(_P)))
    del keep
    return f32, bf, prm


def pack_weights_original_nerf(arrays):
    """Host-only packing of the original NeRF implementation's 24 arrays
    (NERF_LAYOUT_ORIGINAL_NERF, weights.original_nerf_tensors): (f32 blob, params)."""
    from . import weights as W

    lib = load_library()
    sizes = [ctypes.c_size_t() for _ in range(3)]
    lib.nerf_packed_sizes(*[ctypes.byref(s) for s in sizes])
    f32 = np.zeros(sizes[0].value // 4, np.float32)
    prm = np.zeros(sizes[2].value // 4, np.float32)
    arrs = W.original_nerf_tensors(arrays)
    ptrs = (_FP * NERF_N_PARAMS)(*[_fptr(a) for a in arrs])
    _check(lib.nerf_pack_weights_layout(ptrs, NERF_N_PARAMS, NERF_LAYOUT_ORIGINAL_NERF, f32.ctypes.data_as(_P),
                                        prm.ctypes.data_as(_P), None))
    del arrs
    return f32, prm


def pack_weights_fp8(sd: Mapping[str, np.ndarray]) -> np.ndarray:
    """Host-only fp8 packing (e4m3 fragments + E8M0 row scales), as the loader runs it."""
    lib = load_library()
    blob = np.zeros(lib.nerf_fp8_blob_bytes(), np.uint8)
    keep, ptrs = _param_list(sd)
    _check(lib.nerf_pack_weights_fp8(ptrs, NERF_N_PARAMS, blob.ctypes.data_as(_P)))
    del keep
    return blob


def pack_weights_f16x3(sd: Mapping[str, np.ndarray]) -> np.ndarray:
    """Host-only split-fp16 packing (fp16 W_hi and W_lo units, uint16), as the loader runs it."""
    lib = load_library()
    blob = np.zeros(lib.nerf_bf16x3_blob_bytes() // 2, np.uint16)
    keep, ptrs = _param_list(sd)
    _check(lib.nerf_pack_weights_f16x3(ptrs, NERF_N_PARAMS, blob.ctypes.data_as(_P)))
    del keep
    return blob


def pack_weights_bf16x3(sd: Mapping[str, np.ndarray]) -> np.ndarray:
    """Host-only split-bf16 packing (W_hi and W_lo units, uint16), as the loader runs it."""
    lib = load_library()
    blob = np.zeros(lib.nerf_bf16x3_blob_bytes() // 2, np.uint16)
    keep, ptrs = _param_list(sd)
    _check(lib.nerf_pack_weights_bf16x3(ptrs, NERF_N_PARAMS, blob.ctypes.data_as(_P)))
    del keep
    return blob


def f32_to_e4m3(x: np.ndarray) -> np.ndarray:
    """The library's f32 -> e4m3fn rounding (uint8 codes)."""
    lib = load_library()
    a = np.ascontiguousarray(x, dtype=np.float32).ravel()
    out = np.zeros(a.size, np.uint8)
    lib.nerf_f32_to_e4m3(_fptr(a), a.size, out.ctypes.data_as(_P))
    return out.reshape(np.shape(x))


def linspace01(n: int) -> np.ndarray:
    """torch.linspace(0, 1, n) as the library computes it (host helper)."""
    out = np.zeros(n, np.float32)
    load_library().nerf_linspace01(n, _fptr(out))
    return out


def uniform_z(t_vals: np.ndarray, near: float, far: float) -> np.ndarray:
    lib = load_library()
    t = np.ascontiguousarray(t_vals, dtype=np.float32)
    z = np.empty_like(t)
    lib.nerf_uniform_z(_fptr(t), t.size, near, far, _fptr(z))
    return z


def _ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def torch_float32():
    import torch

    return torch.float32


def _stream(stream) -> int:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


class Device:
    """One library context on one GPU (weights resident, scratch reused)."""

    def __init__(self, device_index: int = 0):
        lib = load_library()
        self.lib = lib
        self.index = device_index
        ctx = ctypes.c_void_p()
        _check(lib.nerf_ctx_create(device_index, ctypes.byref(ctx)))
        self._ctx = ctx
        self.loaded = set()

    def close(self) -> None:
        if getattr(self, "_ctx", None) and self._ctx.value:
            self.lib.nerf_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def name(self) -> str:
        buf = ctypes.create_string_buffer(256)
        _check(self.lib.nerf_device_name(self.index, buf, 256))
        return buf.value.decode()

    def load_weights(self, net: int, sd: Mapping[str, np.ndarray]) -> None:
        keep, ptrs = _param_list(sd)
        _check(self.lib.nerf_ctx_load_weights(self._ctx, net, ptrs, NERF_N_PARAMS))
        del keep
        self.loaded.add(net)

    def load_original_nerf(self, net: int, arrays) -> None:
        """The original NeRF implementation's 24 arrays (weights.original_nerf_tensors), rendered
        on NERF_FP32 or NERF_F16X3 (NERF_LAYOUT_ORIGINAL_NERF)."""
        from . import weights as W

        arrs = W.original_nerf_tensors(arrays)
        ptrs = (_FP * NERF_N_PARAMS)(*[_fptr(a) for a in arrs])
        _check(self.lib.nerf_ctx_load_weights_layout(self._ctx, net, NERF_LAYOUT_ORIGINAL_NERF, ptrs, NERF_N_PARAMS))
        del arrs
        self.loaded.add(net)

    # ---- granular device calls (torch CUDA tensors in, results written in place) ----
    def generate_rays(self, c2w: np.ndarray, width: int, height: int, row0: int, row1: int, focal: float,
                      rays_o, rays_d, stream=None) -> None:
        pose = np.ascontiguousarray(np.asarray(c2w, dtype=np.float32).reshape(4, 4))
        _check(self.lib.nerf_generate_rays(self._ctx, _fptr(pose), width, height, row0, row1, focal,
                                           _ptr(rays_o), _ptr(rays_d), _stream(stream)))

    def mlp_forward(self, net: int, precision: int, rays_o, rays_d, z, z_ray_stride: int, n_rays: int,
                    n_samples: int, out, stream=None) -> None:
        _check(self.lib.nerf_mlp_forward(self._ctx, net, precision, _ptr(rays_o), _ptr(rays_d), _ptr(z),
                                         z_ray_stride, n_rays, n_samples, _ptr(out), _stream(stream)))

    def query(self, net: int, precision: int, positions, directions, out, stream=None) -> None:
        _check(self.lib.nerf_query(self._ctx, net, precision, _ptr(positions), _ptr(directions),
                                   positions.shape[0], _ptr(out), _stream(stream)))

    def composite(self, sigma, sigma_stride: int, rgb, rgb_stride: int, z, z_ray_stride: int, rays_d,
                  n_rays: int, n_samples: int, rgb_out, depth_out, acc_out=None, weights_out=None,
                  stream=None) -> None:
        _check(self.lib.nerf_composite(_ptr(sigma), sigma_stride, _ptr(rgb), rgb_stride, _ptr(z), z_ray_stride,
                                       _ptr(rays_d), n_rays, n_samples, _ptr(rgb_out), _ptr(depth_out),
                                       _ptr(acc_out), _ptr(weights_out), _stream(stream)))

    def importance_sample(self, z_coarse, z_ray_stride: int, weights, u, u_ray_stride: int, n_rays: int,
                          n_coarse: int, n_importance: int, z_fine, stream=None) -> None:
        _check(self.lib.nerf_importance_sample(_ptr(z_coarse), z_ray_stride, _ptr(weights), _ptr(u), u_ray_stride,
                                               n_rays, n_coarse, n_importance, _ptr(z_fine), _stream(stream)))

    def render(self, c2w: np.ndarray, width: int, height: int, row0: int, row1: int, focal: float, near: float,
               far: float, t_vals: np.ndarray, n_importance: int, u: Optional[np.ndarray], precision: int,
               rgb_out, depth_out, stream=None, t_rand=None, u_rays=None) -> None:
        """t_rand [rays, S] / u_rays [rays, N]: optional per-ray draws (device tensors)."""
        pose = np.ascontiguousarray(np.asarray(c2w, dtype=np.float32).reshape(4, 4))
        t = np.ascontiguousarray(t_vals, dtype=np.float32)
        uu = None if u is None else np.ascontiguousarray(u, dtype=np.float32)
        n_rays = (row1 - row0) * width
        if t_rand is not None and tuple(t_rand.shape) != (n_rays, t.size):
            raise ValueError(f"t_rand must be [{n_rays}, {t.size}], got {tuple(t_rand.shape)}")
        if u_rays is not None and tuple(u_rays.shape) != (n_rays, n_importance):
            raise ValueError(f"u_rays must be [{n_rays}, {n_importance}], got {tuple(u_rays.shape)}")
        for name, a in (("t_rand", t_rand), ("u_rays", u_rays)):
            if a is not None and not (a.is_cuda and a.dtype == torch_float32() and a.is_contiguous()):
                raise ValueError(f"{name} must be a contiguous float32 device tensor")
        _check(self.lib.nerf_render_sampled(self._ctx, _fptr(pose), width, height, row0, row1, focal, near, far,
                                            _fptr(t), t.size, n_importance, None if uu is None else _fptr(uu),
                                            _ptr(t_rand), _ptr(u_rays), precision, _ptr(rgb_out), _ptr(depth_out),
                                            _stream(stream)))

    def render_band(self, c2w: np.ndarray, width: int, height: int, row0: int, row1: int, focal: float,
                    near: float, far: float, t_vals: np.ndarray, n_importance: int, u: Optional[np.ndarray],
                    precision: int, rgbd_out, stream=None) -> None:
        """Rows [row0, row1) into the packed [rows, W, 4] (r, g, b, depth) device tensor rgbd_out."""
        pose = np.ascontiguousarray(np.asarray(c2w, dtype=np.float32).reshape(4, 4))
        t = np.ascontiguousarray(t_vals, dtype=np.float32)
        uu = None if u is None else np.ascontiguousarray(u, dtype=np.float32)
        n = (row1 - row0) * width
        if rgbd_out.numel() < 4 * n or not rgbd_out.is_contiguous() or rgbd_out.dtype != torch_float32():
            raise ValueError(f"rgbd_out must be a contiguous float32 tensor of >= {4 * n} elements")
        _check(self.lib.nerf_render_band(self._ctx, _fptr(pose), width, height, row0, row1, focal, near, far,
                                         _fptr(t), t.size, n_importance, None if uu is None else _fptr(uu),
                                         precision, _ptr(rgbd_out), _stream(stream)))

    def range_status(self, stream=None) -> None:
        """Synchronize the stream; NerfRangeError if an f16x3 launch since the last call met an
        activation outside fp16's range (nerf_ctx_range_status)."""
        _check(self.lib.nerf_ctx_range_status(self._ctx, _stream(stream)))

    def last_fine_z(self, n_rays: int, per_ray: int, out, stream=None) -> None:
        """The last hierarchical render's fine-pass sample depths [n_rays, per_ray] into out."""
        if out.numel() < n_rays * per_ray or not out.is_contiguous():
            raise ValueError("out too small or not contiguous")
        _check(self.lib.nerf_ctx_last_fine_z(self._ctx, n_rays, per_ray, _ptr(out), _stream(stream)))

    def sample_points(self, rays_o, rays_d, t_vals: np.ndarray, near: float, far: float, z_out, points_out=None,
                      t_rand=None, stream=None) -> None:
        t = np.ascontiguousarray(t_vals, dtype=np.float32)
        n = z_out.shape[0]
        _check(self.lib.nerf_sample_points(self._ctx, _ptr(rays_o), _ptr(rays_d), n, _fptr(t), t.size, near, far,
                                           _ptr(t_rand), _ptr(z_out), _ptr(points_out), _stream(stream)))

    def set_profiling(self, enable: bool) -> None:
        _check(self.lib.nerf_ctx_set_profiling(self._ctx, 1 if enable else 0))

    def set_fused_composite(self, enable, coarse: bool = True) -> None:
        """NERF_OPT_FUSED_COMPOSITE: compositing in the bf16 / fp8 / split MLP epilogue (default on),
        for the rendered pass and (``coarse``) the hierarchical coarse pass's weights."""
        _check(self.lib.nerf_ctx_set_option(self._ctx, NERF_OPT_FUSED_COMPOSITE,
                                            (1 if enable else 0) | (2 if enable and coarse else 0)))

    def set_coarse_precision(self, precision: Optional[int]) -> None:
        """NERF_OPT_COARSE_PRECISION: the hierarchical coarse pass's precision (None: the render's)."""
        _check(self.lib.nerf_ctx_set_option(self._ctx, NERF_OPT_COARSE_PRECISION,
                                            -1 if precision is None else int(precision)))

    def stage_ms_history(self, n: int) -> list:
        """Per-stage device ms of each of the last n renders (n <= 64), oldest first."""
        ms = (ctypes.c_float * (n * NERF_N_STAGES))()
        _check(self.lib.nerf_ctx_stage_ms_history(self._ctx, n, ms))
        return [dict(zip(STAGES, [float(v) for v in ms[k * NERF_N_STAGES:(k + 1) * NERF_N_STAGES]]))
                for k in range(n)]

    def stage_ms(self) -> dict:
        ms = (ctypes.c_float * NERF_N_STAGES)()
        _check(self.lib.nerf_ctx_stage_ms(self._ctx, ms))
        return dict(zip(STAGES, [float(v) for v in ms]))


def positional_encoding(precision: int, x, n_freqs: int, out, stream=None) -> None:
    """nerf_positional_encoding: x device [n, 3] -> out device [n, 3 + 6 n_freqs] (no context needed)."""
    lib = load_library()
    n = x.shape[0]
    if tuple(out.shape) != (n, 3 + 6 * n_freqs) or not (x.is_contiguous() and out.is_contiguous()):
        raise ValueError("x [n, 3] and out [n, 3 + 6*n_freqs], contiguous")
    _check(lib.nerf_positional_encoding(precision, _ptr(x), n, n_freqs, _ptr(out), _stream(stream)))


def exported_symbols() -> Sequence[str]:
    return tuple(SIGNATURES)
