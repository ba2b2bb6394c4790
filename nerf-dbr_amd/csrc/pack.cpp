// Host-side weight packing: nn.Linear [out, in] fp32 tensors -> the fragment
// layouts of nerf_layout.h.  Pure host code (no HIP calls); exported through
// the C ABI so layout tests can run it without a GPU.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "nerf_layout.h"
#include "nerf_mi355x.h"
#include "nerf_internal.h"

using namespace nerf;

namespace {

// state-dict index (in NERF_N_PARAMS order) of each MFMA layer's weight
constexpr int kSpecOfLayer[kNumMfmaLayers] = {0, 1, 2, 3, 4, 5, 6, 7, 9};
constexpr int kSpecDensity = 8, kSpecColor1 = 10;
constexpr int kSpecOut[11] = {256, 256, 256, 256, 256, 256, 256, 256, 1, 128, 3};
constexpr int kSpecIn[11] = {63, 256, 256, 256, 319, 256, 256, 256, 256, 283, 128};

uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return uint16_t((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7FFFu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}

}  // namespace

extern "C" void nerf_packed_sizes(size_t* f32_blob, size_t* bf16_blob, size_t* param_blob) {
  if (f32_blob) *f32_blob = size_t(f32_blob_floats()) * sizeof(float);
  if (bf16_blob) *bf16_blob = size_t(kBf16BlobBytes);
  if (param_blob) *param_blob = size_t(kParamFloats) * sizeof(float);
}

extern "C" int nerf_pack_weights(const float* const* params, int n_params, float* f32_blob,
                                 uint16_t* bf16_blob, float* param_blob) {
  if (!params || n_params != NERF_N_PARAMS) return set_error(NERF_E_INVALID, "nerf_pack_weights: need %d tensors, got %d", NERF_N_PARAMS, n_params);
  for (int i = 0; i < NERF_N_PARAMS; ++i)
    if (!params[i]) return set_error(NERF_E_INVALID, "nerf_pack_weights: tensor %d is NULL", i);
  auto W = [&](int spec, int o, int k) { return params[2 * spec][size_t(o) * kSpecIn[spec] + k]; };
  auto B = [&](int spec, int o) { return params[2 * spec + 1][o]; };

  if (f32_blob) {
    float* dst = f32_blob;
    for (int l = 0; l < kNumMfmaLayers; ++l) {
      const int spec = kSpecOfLayer[l], nt = out_tiles(l), ku = ksteps_f32(l);
      for (int ug = 0; ug < ku / 4; ++ug)
        for (int o = 0; o < nt; ++o)
          for (int lane = 0; lane < 64; ++lane)
            for (int i = 0; i < 4; ++i) {
              const int col = f32_k_col(l, 4 * ug + i, lane >> 5);
              *dst++ = col < 0 ? 0.0f : W(spec, 32 * o + (lane & 31), col);
            }
    }
  }
  if (bf16_blob) {
    uint16_t* dst = bf16_blob;
    for (int l = 0; l < kNumMfmaLayers; ++l) {
      const int spec = kSpecOfLayer[l], nq = out_tiles(l) / 2, ku = ksteps_bf16(l);
      for (int q = 0; q < nq; ++q)
        for (int u = 0; u < ku; ++u)
          for (int o2 = 0; o2 < 2; ++o2)
            for (int lane = 0; lane < 64; ++lane)
              for (int j = 0; j < 8; ++j) {
                const int col = bf16_k_col(l, u, lane >> 5, j);
                const int row = 32 * (2 * q + o2) + (lane & 31);
                *dst++ = col < 0 ? uint16_t(0) : f32_to_bf16_rne(W(spec, row, col));
              }
    }
    uint16_t* end = bf16_blob + size_t(kBf16BlobBytes) / 2;
    while (dst < end) *dst++ = 0;
  }
  if (param_blob) {
    std::memset(param_blob, 0, sizeof(float) * kParamFloats);
    for (int l = 0; l < kNumMfmaLayers; ++l) {
      const int spec = kSpecOfLayer[l];
      for (int o = 0; o < out_tiles(l); ++o)
        for (int h = 0; h < 2; ++h)
          for (int r = 0; r < 16; ++r)
            param_blob[kBiasOff + 256 * l + (o * 2 + h) * 16 + r] = B(spec, 32 * o + acc_row(r, h));
    }
    for (int h = 0; h < 2; ++h)
      for (int t = 0; t < 8; ++t)
        for (int r = 0; r < 16; ++r) param_blob[kSigW + (h * 8 + t) * 16 + r] = W(kSpecDensity, 0, 32 * t + acc_row(r, h));
    param_blob[kSigB] = B(kSpecDensity, 0);
    for (int c = 0; c < 3; ++c) {
      for (int h = 0; h < 2; ++h)
        for (int t = 0; t < 4; ++t)
          for (int r = 0; r < 16; ++r)
            param_blob[kC1W + ((c * 2 + h) * 4 + t) * 16 + r] = W(kSpecColor1, c, 32 * t + acc_row(r, h));
      param_blob[kC1B + c] = B(kSpecColor1, c);
    }
  }
  (void)kSpecOut;
  return NERF_OK;
}

extern "C" void nerf_uniform_z(const float* t_vals, int n, float near_, float far_, float* z_out) {
  // base_renderer.py:275  z = near*(1-t) + far*t ; compiled with -ffp-contract=off
  for (int i = 0; i < n; ++i) {
    volatile float one_minus = 1.0f - t_vals[i];
    volatile float a = near_ * one_minus;
    volatile float b = far_ * t_vals[i];
    z_out[i] = a + b;
  }
}
