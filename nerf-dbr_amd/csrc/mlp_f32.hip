// fp32 NeRF MLP on gfx950 f32-input MFMA (v_mfma_f32_32x32x2_f32): the parity path.
//
// Replaces NeRFModel.forward (src/models/nerf.py:92-131) fused with
// sample_points_on_rays (src/benchmark/base_renderer.py:260-281) and the
// positional encoding (nerf.py:24-45).  Every product is an exact fp32 fma
// chain (the MFMA's documented numerics), so results differ from the
// reference's oneDNN GEMM only by summation order.
//
// Geometry: 256-thread workgroups (4 waves, one per SIMD), 32 samples per wave.
// Per lane: 8 output tiles x 16 accumulator registers for the layer being
// computed plus the previous layer's 128 (its B operand) -- hence one wave per
// SIMD.  The A operand (weights, pre-packed as one float4 per lane per four
// k-steps) is read straight from L2: at the f32 MFMA rate a CU consumes only
// ~16 B/clk of weights.
#include "nerf_device.h"
#include "nerf_internal.h"

namespace nerf {
namespace {

constexpr int kWavesF32 = 4;

template <int L, int kSkip>
constexpr int f32_layer_offset() {   // in floats
  int off = 0;
  for (int l = 0; l < L; ++l) off += f32_layer_floats(l, kSkip);
  return off;
}

// One MFMA layer: acc[0..NT) = bias + W . [prev | ext]; kSkip: the layer that takes the
// position encoding again (nerf_layout.h)
template <int L, int NT, int NEXT, int kSkip>
__device__ __forceinline__ void layer_f32(f32x16 (&acc)[8], const f32x16 (&prev)[8], const float (&ext)[NEXT],
                                          const f32x4* __restrict__ blob, const float* __restrict__ prm,
                                          int lane, int h) {
  constexpr LayerShape sh = layer_shape(L, kSkip);
  constexpr int KH = sh.hidden / 2;         // hidden k-steps
  constexpr int KU = ksteps_f32(L, kSkip);
  static_assert(KU == KH + (sh.extra == kNone ? 0 : NEXT), "layer/ext mismatch");
  load_bias<NT>(acc, prm, L, h);
  const f32x4* a_base = blob + f32_layer_offset<L, kSkip>() / 4 + lane;
#pragma unroll
  for (int ug = 0; ug < KU / 4; ++ug) {
    f32x4 a[NT];
#pragma unroll
    for (int o = 0; o < NT; ++o) a[o] = a_base[(ug * NT + o) * 64];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = 4 * ug + i;
      float b;
      if (u < KH) b = prev[u >> 4][u & 15];
      else b = ext[u - KH];
#pragma unroll
      for (int o = 0; o < NT; ++o) acc[o] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[o][i], b, acc[o], 0, 0, 0);
    }
  }
}

// kOrig: the original NeRF implementation's network (nerf_ctx_load_weights_layout, layout 1):
// the position encoding re-enters at layer 5, the encodings have no pi, and the view
// directions are normalised before their encoding; its feature layer (linear, no activation)
// arrives folded into C0 by the host.  Otherwise NeRFModel (nerf.py:92-131).
template <bool kExplicit, bool kOrig = false>
__global__ __launch_bounds__(256, 1) void mlp_f32_kernel(const f32x4* __restrict__ blob,
                                                         const float* __restrict__ prm, SampleSrc src,
                                                         long n_points, f32x4* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int h = lane >> 5;
  const long p = (long(blockIdx.x) * kWavesF32 + wave) * kSamplesPerWave + (lane & 31);
  const bool valid = p < n_points;
  const long pc = valid ? p : n_points - 1;

  float x[3], d[3];
  fetch_sample<kExplicit>(src, pc, x, d);
  float pe[32], de[16];
  constexpr int S = kOrig ? kSkipOriginal : kSkipNeRFModel;
  pos_encode<false, false, kOrig>(x[0], x[1], x[2], h, pe);
  if (kOrig) {   // the original's viewdirs = rays_d / |rays_d| (its encoding input)
    const float n = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(d[0], d[0]), __fmul_rn(d[1], d[1])), __fmul_rn(d[2], d[2])));
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = __fdiv_rn(d[c], n);
  }
  dir_encode<false, false, kOrig>(d[0], d[1], d[2], h, de);

  f32x16 a[8], b[8];
  layer_f32<L0, 8, 32, S>(a, b, pe, blob, prm, lane, h);   // b unused (no hidden input)
  relu_tiles<8>(a);
  layer_f32<L1, 8, 32, S>(b, a, pe, blob, prm, lane, h);
  relu_tiles<8>(b);
  layer_f32<L2, 8, 32, S>(a, b, pe, blob, prm, lane, h);
  relu_tiles<8>(a);
  layer_f32<L3, 8, 32, S>(b, a, pe, blob, prm, lane, h);
  relu_tiles<8>(b);
  layer_f32<L4, 8, 32, S>(a, b, pe, blob, prm, lane, h);   // NeRFModel's skip: [x, pe] (nerf.py:109-110)
  relu_tiles<8>(a);
  layer_f32<L5, 8, 32, S>(b, a, pe, blob, prm, lane, h);   // the original's skip ([pe, h], re-ordered)
  relu_tiles<8>(b);
  layer_f32<L6, 8, 32, S>(a, b, pe, blob, prm, lane, h);
  relu_tiles<8>(a);
  layer_f32<L7, 8, 32, S>(b, a, pe, blob, prm, lane, h);
  relu_tiles<8>(b);
  const float sigma = density_head(b, prm, h);
  layer_f32<C0, 4, 16, S>(a, b, de, blob, prm, lane, h);   // [x, PE4(d)] (nerf.py:117-121)
  relu_tiles<4>(a);
  float rgb[3];
  color_head(a, prm, h, rgb);
  if (valid && h == 0) out[p] = f32x4{sigma, rgb[0], rgb[1], rgb[2]};
}

}  // namespace

hipError_t launch_mlp_f32(const float* blob, const float* params, const SampleSrc& src, long n_points,
                          float* out, bool explicit_points, hipStream_t stream, int layout) {
  if (n_points <= 0) return hipSuccess;
  const long per_block = long(kWavesF32) * kSamplesPerWave;
  const long blocks = (n_points + per_block - 1) / per_block;
  if (blocks > 0x7FFFFFFFL) return hipErrorInvalidValue;
  const dim3 grid{unsigned(blocks), 1, 1}, block{64 * kWavesF32, 1, 1};
  if (layout != 0 && layout != 1) return hipErrorInvalidValue;
  if (explicit_points && layout == 1)
    hipLaunchKernelGGL((mlp_f32_kernel<true, true>), grid, block, 0, stream, (const f32x4*)blob, params, src, n_points,
                       (f32x4*)out);
  else if (explicit_points)
    hipLaunchKernelGGL(mlp_f32_kernel<true>, grid, block, 0, stream, (const f32x4*)blob, params, src, n_points,
                       (f32x4*)out);
  else if (layout == 1)
    hipLaunchKernelGGL((mlp_f32_kernel<false, true>), grid, block, 0, stream, (const f32x4*)blob, params, src,
                       n_points, (f32x4*)out);
  else
    hipLaunchKernelGGL(mlp_f32_kernel<false>, grid, block, 0, stream, (const f32x4*)blob, params, src, n_points,
                       (f32x4*)out);
  return hipGetLastError();
}

}  // namespace nerf
