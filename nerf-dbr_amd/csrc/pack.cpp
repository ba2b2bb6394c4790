// Host-side weight packing: nn.Linear [out, in] fp32 tensors -> the fragment
// layouts of nerf_layout.h.  Pure host code (no HIP calls); exported through
// the C ABI so layout tests can run it without a GPU.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

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
// the original NeRF implementation's trunk (NERF_LAYOUT_ORIGINAL_NERF): the skip input on layer 5
constexpr int kSpecInOrig[11] = {63, 256, 256, 256, 256, 319, 256, 256, 256, 283, 128};

uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return uint16_t((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7FFFu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}

// f32 -> OCP e4m3fn, round to nearest even; |v| <= 448 is the caller's contract
// (the packer picks power-of-two scales that guarantee it).  Subnormals: 2^-9 steps.
uint8_t f32_to_e4m3_rne(float v) {
  uint32_t u;
  std::memcpy(&u, &v, 4);
  const uint8_t sign = uint8_t((u >> 24) & 0x80u);
  float a = std::fabs(v);
  if (!(a == a)) return 0x7F;                          // NaN
  if (a == 0.0f) return sign;
  int e;
  std::frexp(a, &e);                                   // a = m * 2^e, m in [0.5, 1)
  int ex = e - 1;                                      // a in [2^ex, 2^(ex+1))
  if (ex < -6) ex = -6;                                // subnormal range shares 2^-9 steps
  const float step = std::ldexp(1.0f, ex - 3);         // 3 mantissa bits
  float q = std::nearbyint(a / step) * step;           // default rounding mode: nearest even
  if (q == 0.0f) return sign;
  std::frexp(q, &e);
  ex = e - 1;
  if (ex < -6) return uint8_t(sign | uint8_t(q / std::ldexp(1.0f, -9)));           // subnormal: mantissa only
  const int mant = int(q / std::ldexp(1.0f, ex - 3)) - 8;                          // 0..7
  return uint8_t(sign | uint8_t((ex + 7) << 3) | uint8_t(mant));
}

// E8M0 exponent e (value 2^e) so that max|row| / 2^e <= 448
int row_scale_exp(float max_abs) {
  if (!(max_abs > 0.0f)) return 0;
  int e = int(std::ceil(std::log2(double(max_abs) / double(kFp8Max))));
  while (std::ldexp(double(max_abs), -e) > kFp8Max) ++e;
  while (std::ldexp(double(max_abs), -(e - 1)) <= kFp8Max) --e;
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}

// The bf16 blob's values before rounding (fp32), in stream order: per layer
// [quarter][k-step][tile-in-quarter][lane][8], then the heads' tile
// (nerf_layout.h); padding slots are 0.
void bf16_stream_values(const float* const* params, std::vector<float>& out, int skip = kSkipNeRFModel) {
  const int* in = skip == kSkipOriginal ? kSpecInOrig : kSpecIn;
  auto W = [&](int spec, int o, int k) { return params[2 * spec][size_t(o) * in[spec] + k]; };
  out.clear();
  out.reserve(size_t(kBf16BlobBytes) / 2);
  for (int l = 0; l < kNumMfmaLayers; ++l) {
    const int spec = kSpecOfLayer[l], nq = out_tiles(l) / 2, ku = ksteps_bf16(l, skip);
    for (int q = 0; q < nq; ++q)
      for (int u = 0; u < ku; ++u)
        for (int o2 = 0; o2 < 2; ++o2)
          for (int lane = 0; lane < 64; ++lane)
            for (int j = 0; j < 8; ++j) {
              const int col = bf16_k_col(l, u, lane >> 5, j, skip);
              const int row = 32 * (2 * q + o2) + (lane & 31);
              out.push_back(col < 0 ? 0.0f : W(spec, row, col));
            }
  }
  for (int u = 0; u < kHeadKsteps; ++u)
    for (int lane = 0; lane < 64; ++lane)
      for (int j = 0; j < 8; ++j) {
        int dens = 0;
        const int row = lane & 31;
        const int f = head_k_row_col(u, row, lane >> 5, j, &dens);
        out.push_back(f < 0 ? 0.0f : (dens ? W(kSpecDensity, 0, f) : W(kSpecColor1, row, f)));
      }
}

}  // namespace

extern "C" size_t nerf_bf16x3_blob_bytes(void) { return size_t(kBf16x3BlobBytes); }

extern "C" int nerf_pack_weights_bf16x3(const float* const* params, int n_params, uint16_t* blob) {
  if (!params || n_params != NERF_N_PARAMS || !blob)
    return set_error(NERF_E_INVALID, "nerf_pack_weights_bf16x3: need %d tensors and a blob", NERF_N_PARAMS);
  for (int i = 0; i < NERF_N_PARAMS; ++i)
    if (!params[i]) return set_error(NERF_E_INVALID, "nerf_pack_weights_bf16x3: tensor %d is NULL", i);
  std::vector<float> vals;
  bf16_stream_values(params, vals);
  constexpr size_t kUnit = size_t(kUnitBytes) / 2;          // bf16 elements per bf16 unit
  std::memset(blob, 0, size_t(kBf16x3BlobBytes));
  for (size_t i = 0; i < vals.size(); ++i) {
    const uint16_t hi = f32_to_bf16_rne(vals[i]);
    uint32_t hb = uint32_t(hi) << 16;
    float hf;
    std::memcpy(&hf, &hb, 4);
    const uint16_t lo = f32_to_bf16_rne(vals[i] - hf);     // exact in fp32
    const size_t unit = i / kUnit, off = i % kUnit;
    blob[(2 * unit) * kUnit + off] = hi;
    blob[(2 * unit + 1) * kUnit + off] = lo;
  }
  return NERF_OK;
}

namespace {
int pack_f16x3(const float* const* params, int skip, uint16_t* blob) {
  std::vector<float> vals;
  bf16_stream_values(params, vals, skip);
  constexpr size_t kUnit = size_t(kUnitBytes) / 2;          // 16-bit elements per unit
  std::memset(blob, 0, size_t(kBf16x3BlobBytes));
  for (size_t i = 0; i < vals.size(); ++i) {
    if (!(std::fabs(vals[i]) <= 65504.0f))
      return set_error(NERF_E_INVALID, "nerf_pack_weights_f16x3: weight %g is outside the fp16 range", double(vals[i]));
    const _Float16 hi = _Float16(vals[i]);                  // round to nearest even
    const _Float16 lo = _Float16(vals[i] - float(hi));      // the difference is exact in fp32
    const size_t unit = i / kUnit, off = i % kUnit;
    std::memcpy(&blob[(2 * unit) * kUnit + off], &hi, 2);
    std::memcpy(&blob[(2 * unit + 1) * kUnit + off], &lo, 2);
  }
  return NERF_OK;
}
}  // namespace

extern "C" int nerf_pack_weights_f16x3(const float* const* params, int n_params, uint16_t* blob) {
  if (!params || n_params != NERF_N_PARAMS || !blob)
    return set_error(NERF_E_INVALID, "nerf_pack_weights_f16x3: need %d tensors and a blob", NERF_N_PARAMS);
  for (int i = 0; i < NERF_N_PARAMS; ++i)
    if (!params[i]) return set_error(NERF_E_INVALID, "nerf_pack_weights_f16x3: tensor %d is NULL", i);
  return pack_f16x3(params, kSkipNeRFModel, blob);
}

extern "C" size_t nerf_fp8_blob_bytes(void) { return size_t(kFp8BlobBytes); }

extern "C" void nerf_f32_to_e4m3(const float* x, int n, uint8_t* out) {
  for (int i = 0; i < n; ++i) out[i] = f32_to_e4m3_rne(x[i]);
}

extern "C" int nerf_pack_weights_fp8(const float* const* params, int n_params, uint8_t* blob) {
  if (!params || n_params != NERF_N_PARAMS || !blob)
    return set_error(NERF_E_INVALID, "nerf_pack_weights_fp8: need %d tensors and a blob", NERF_N_PARAMS);
  for (int i = 0; i < NERF_N_PARAMS; ++i)
    if (!params[i]) return set_error(NERF_E_INVALID, "nerf_pack_weights_fp8: tensor %d is NULL", i);
  auto W = [&](int spec, int o, int k) { return params[2 * spec][size_t(o) * kSpecIn[spec] + k]; };
  std::memset(blob, 0, size_t(kFp8BlobBytes));
  uint32_t* scales = reinterpret_cast<uint32_t*>(blob + kFp8ScaleOff);
  for (int i = 0; i < kFp8ScaleBytes / 4; ++i) scales[i] = 127u;
  // the mixed stream (nerf_layout.h): per layer [quarter][fp8 units, then bf16 units]
  for (int l = 0; l < kNumMfmaLayers; ++l) {
    const int spec = kSpecOfLayer[l], nt = out_tiles(l), nq = nt / 2, nf = mix_f8_units(l), nb = mix_b_units(l);
    const int hid = layer_shape(l).hidden;
    int exps[256] = {};
    if (nf > 0) {   // row scales over the columns the fp8 k-steps carry (the hidden inputs)
      for (int row = 0; row < 32 * nt; ++row) {
        float m = 0.0f;
        for (int k = 0; k < hid; ++k) m = std::fmax(m, std::fabs(W(spec, row, k)));
        exps[row] = row_scale_exp(m);
      }
      for (int q = 0; q < 4; ++q)
        for (int lane = 0; lane < 64; ++lane)
          for (int o2 = 0; o2 < 2; ++o2) {
            const int tile = 2 * q + o2;
            scales[((l * 4 + q) * 64 + lane) * 2 + o2] = tile < nt ? uint32_t(127 + exps[32 * tile + (lane & 31)]) : 127u;
          }
    }
    for (int q = 0; q < nq; ++q) {
      const int unit0 = mix_unit_base(l) + q * mix_units_per_quarter(l);
      for (int u = 0; u < nf; ++u) {
        uint8_t* dst = blob + size_t(unit0 + u) * kFp8UnitBytes;
        for (int o2 = 0; o2 < 2; ++o2)
          for (int p = 0; p < 2; ++p)
            for (int lane = 0; lane < 64; ++lane)
              for (int jj = 0; jj < 16; ++jj) {
                const int col = fp8_k_col(l, u, lane >> 5, 16 * p + jj);
                const int row = 32 * (2 * q + o2) + (lane & 31);
                *dst++ = col < 0 ? uint8_t(0) : f32_to_e4m3_rne(std::ldexp(W(spec, row, col), -exps[row]));
              }
      }
      for (int b = 0; b < nb; ++b) {
        uint16_t* dst = reinterpret_cast<uint16_t*>(blob + size_t(unit0 + nf + b) * kFp8UnitBytes);
        for (int sk = 0; sk < 2; ++sk)
          for (int o2 = 0; o2 < 2; ++o2)
            for (int lane = 0; lane < 64; ++lane)
              for (int j = 0; j < 8; ++j) {
                const int col = bf16_k_col(l, mix_b_kstep(l, b, sk), lane >> 5, j);
                const int row = 32 * (2 * q + o2) + (lane & 31);
                *dst++ = col < 0 ? uint16_t(0) : f32_to_bf16_rne(W(spec, row, col));
              }
      }
    }
  }
  // the heads: the bf16 kernel's head tile (nerf_layout.h kHeadKsteps), four k-steps a unit
  uint16_t* hd = reinterpret_cast<uint16_t*>(blob + size_t(kMixLayerUnits) * kFp8UnitBytes);
  for (int u = 0; u < kHeadKsteps; ++u)
    for (int lane = 0; lane < 64; ++lane)
      for (int j = 0; j < 8; ++j) {
        int dens = 0;
        const int row = lane & 31;
        const int f = head_k_row_col(u, row, lane >> 5, j, &dens);
        *hd++ = f < 0 ? uint16_t(0) : f32_to_bf16_rne(dens ? W(kSpecDensity, 0, f) : W(kSpecColor1, row, f));
      }
  return NERF_OK;
}

extern "C" void nerf_packed_sizes(size_t* f32_blob, size_t* bf16_blob, size_t* param_blob) {
  if (f32_blob) *f32_blob = size_t(f32_blob_floats()) * sizeof(float);
  if (bf16_blob) *bf16_blob = size_t(kBf16BlobBytes);
  if (param_blob) *param_blob = size_t(kParamFloats) * sizeof(float);
}

namespace {

// f32 A blob (nerf_layout.h) and the params blob of either network layout
void pack_f32(const float* const* params, int skip, float* f32_blob) {
  const int* in = skip == kSkipOriginal ? kSpecInOrig : kSpecIn;
  auto W = [&](int spec, int o, int k) { return params[2 * spec][size_t(o) * in[spec] + k]; };
  float* dst = f32_blob;
  for (int l = 0; l < kNumMfmaLayers; ++l) {
    const int spec = kSpecOfLayer[l], nt = out_tiles(l), ku = ksteps_f32(l, skip);
    for (int ug = 0; ug < ku / 4; ++ug)
      for (int o = 0; o < nt; ++o)
        for (int lane = 0; lane < 64; ++lane)
          for (int i = 0; i < 4; ++i) {
            const int col = f32_k_col(l, 4 * ug + i, lane >> 5, skip);
            *dst++ = col < 0 ? 0.0f : W(spec, 32 * o + (lane & 31), col);
          }
  }
}

}  // namespace

extern "C" int nerf_pack_weights_layout(const float* const* params, int n_params, int layout, float* f32_blob,
                                        float* param_blob, uint16_t* f16x3_blob) {
  if (layout != NERF_LAYOUT_NERFMODEL && layout != NERF_LAYOUT_ORIGINAL_NERF)
    return set_error(NERF_E_INVALID, "nerf_pack_weights_layout: unknown layout %d", layout);
  if (layout == NERF_LAYOUT_NERFMODEL) {
    const int rc = nerf_pack_weights(params, n_params, f32_blob, nullptr, param_blob);
    return rc != NERF_OK || !f16x3_blob ? rc : nerf_pack_weights_f16x3(params, n_params, f16x3_blob);
  }
  if (!params || n_params != NERF_N_PARAMS)
    return set_error(NERF_E_INVALID, "nerf_pack_weights_layout: need %d tensors, got %d", NERF_N_PARAMS, n_params);
  for (int i = 0; i < NERF_N_PARAMS; ++i)
    if (!params[i]) return set_error(NERF_E_INVALID, "nerf_pack_weights_layout: tensor %d is NULL", i);
  if (f32_blob) pack_f32(params, kSkipOriginal, f32_blob);
  if (f16x3_blob) {
    const int rc = pack_f16x3(params, kSkipOriginal, f16x3_blob);
    if (rc != NERF_OK) return rc;
  }
  // the params blob reads only biases, the density head and colour-1: the same in both layouts
  return param_blob ? nerf_pack_weights(params, n_params, nullptr, nullptr, param_blob) : NERF_OK;
}

extern "C" int nerf_pack_weights(const float* const* params, int n_params, float* f32_blob,
                                 uint16_t* bf16_blob, float* param_blob) {
  if (!params || n_params != NERF_N_PARAMS) return set_error(NERF_E_INVALID, "nerf_pack_weights: need %d tensors, got %d", NERF_N_PARAMS, n_params);
  for (int i = 0; i < NERF_N_PARAMS; ++i)
    if (!params[i]) return set_error(NERF_E_INVALID, "nerf_pack_weights: tensor %d is NULL", i);
  auto W = [&](int spec, int o, int k) { return params[2 * spec][size_t(o) * kSpecIn[spec] + k]; };
  auto B = [&](int spec, int o) { return params[2 * spec + 1][o]; };

  if (f32_blob) pack_f32(params, kSkipNeRFModel, f32_blob);
  if (bf16_blob) {
    std::vector<float> vals;
    bf16_stream_values(params, vals);
    for (size_t i = 0; i < vals.size(); ++i) bf16_blob[i] = f32_to_bf16_rne(vals[i]);
    for (size_t i = vals.size(); i < size_t(kBf16BlobBytes) / 2; ++i) bf16_blob[i] = 0;
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

extern "C" void nerf_linspace01(int n, float* out) {
  // torch.linspace(0, 1, n) on the CPU (ATen linspace_kernel): step = (1 - 0) / (n - 1)
  // in fp32; the first half is start + step*i, the second end - step*(n-1-i), each a
  // single rounding of the exact value (a fused multiply-add in ATen's build)
  if (n <= 0) return;
  if (n == 1) {
    out[0] = 0.0f;
    return;
  }
  const float step = 1.0f / float(n - 1);
  const int half = n / 2;
  for (int i = 0; i < n; ++i)
    out[i] = i < half ? std::fma(step, float(i), 0.0f) : std::fma(-step, float(n - 1 - i), 1.0f);
}
