// Device helpers shared by the gfx950 NeRF kernels: exact-order sampling,
// positional encoding into per-lane-half slots, and the VALU heads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nerf_layout.h"

namespace nerf {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// fl32(2^k * pi): `freq * torch.pi` with freq = 2.0**k as fp32 (nerf.py:22,42);
// a power-of-two multiple of fl32(pi), so exact.
__device__ __forceinline__ float pe_coef(int k) { return __builtin_ldexpf(3.14159274101257324f, k); }

// base_renderer.py:279: o + d*z as a rounded multiply, then a rounded add.
__device__ __forceinline__ float sample_coord(float o, float d, float z) {
  return __fadd_rn(o, __fmul_rn(d, z));
}

// sin and cos of an fp32 argument, for the bf16 path (whose encodings are
// rounded to bf16, 2^-9 relative): exact Cody-Waite reduction by 2*pi
// (6.28125 + 0.00193500518798828125 + 3.0199160e-07; q < 2^12 for |a| < 2^14.6,
// the products are exact), then the hardware v_sin/v_cos on revolutions in
// [-1/2, 1/2].  Error ~1e-6 absolute vs the correctly rounded value.
__device__ __forceinline__ void sincos_fast(float a, float* s, float* c) {
  const float q = __builtin_rintf(__fmul_rn(a, 0.15915493667125702f));
  float r = fmaf(-q, 6.28125f, a);
  r = fmaf(-q, 0.0019350051879882812f, r);
  r = fmaf(-q, 3.019916050561733e-07f, r);
  const float t = __fmul_rn(r, 0.15915493667125702f);
  *s = __builtin_amdgcn_sinf(t);
  *c = __builtin_amdgcn_cosf(t);
}

// sin and cos of an fp32 argument to within 1-2 ulp of torch's CPU sin/cos over the
// encodings' arguments (|a| = |fl(2^k pi) x| < 2^15: 1 ulp in tools/sincos_lab.py's
// emulation on 8.6k arguments; 2.0 ulp max, 76 % bit-exact on the GPU in
// test_gpu_restated.py, as ocml's sincosf measured before), for the fp32 and split
// paths.  Cody-Waite reduction by pi/2 in three fp32 parts with FMA -- the first
// step a - q*P1 is exact (a multiple of 2^-23 below 2 in magnitude) -- then
// minimax polynomials on [-pi/4, pi/4] (sin to r^9, cos to r^10; fitted in
// float64, rounded to fp32) and the quadrant's swap and signs.  About 20 VALU
// per pair against ocml's sincosf, which also evaluates its large-argument
// (Payne-Hanek) reduction for every lane.
__device__ __forceinline__ void sincos_acc(float a, float* s, float* c) {
  const float q = __builtin_rintf(__fmul_rn(a, 0x1.45f306p-1f));            // 2/pi
  float r = fmaf(-q, 0x1.921fb6p+0f, a);                                   // pi/2 = P1 + P2 + P3
  r = fmaf(-q, -0x1.777a5cp-25f, r);
  r = fmaf(-q, -0x1.ee59dap-50f, r);
  const float z = __fmul_rn(r, r);
  const float ps = fmaf(fmaf(fmaf(0x1.6c99b0p-19f, z, -0x1.a00e8cp-13f), z, 0x1.111108p-7f), z, -0x1.555556p-3f);
  const float sn = fmaf(__fmul_rn(r, z), ps, r);
  const float pc = fmaf(fmaf(fmaf(-0x1.23f15cp-22f, z, 0x1.a00ffap-16f), z, -0x1.6c16b6p-10f), z, 0x1.555556p-5f);
  const float cs = fmaf(__fmul_rn(z, z), pc, fmaf(-0.5f, z, 1.0f));
  const int qi = int(q);
  const float s0 = (qi & 1) ? cs : sn, c0 = (qi & 1) ? sn : cs;
  *s = (qi & 2) ? -s0 : s0;
  *c = ((qi + 1) & 2) ? -c0 : c0;
}

// sin/cos of fl(2^k*pi)*x: sincos_acc (the fp32 and split parity paths), the
// reduced-precision sincos_fast (the bf16 / fp8 paths), or ocml's sincosf (kOcml: the
// training kernels, whose gradient parity tests sit at the ReLU-flip floor measured
// with it; both are within an ulp or two of torch).
template <bool kFast, bool kOcml = false>
__device__ __forceinline__ void pe_sincos(float c, float x, float* s, float* co) {
  if (kFast) sincos_fast(__fmul_rn(c, x), s, co);
  else if (kOcml) sincosf(__fmul_rn(c, x), s, co);
  else sincos_acc(__fmul_rn(c, x), s, co);
}

// Position encoding slots of lane half h (nerf_layout.h pe_slot_feature):
// 15 sin/cos pairs + the raw coordinates it owns.
// Fast path: a lane half's frequencies are consecutive powers of two, so after
// one reduced sin/cos per coordinate the rest follow by angle doubling,
// sin 2t = 2 s c, cos 2t = 1 - 2 s^2.  The doubled argument 2^j * fl(2^k pi x)
// equals the reference's fl(2^(k+j) pi x) exactly (power-of-two scaling); the
// doubling adds ~1e-5 absolute error after four steps, far below bf16/e4m3
// rounding of the encodings.
template <int kFreqs>
__device__ __forceinline__ void sincos_doubling(float c0, float x, float* s, float* co) {
  sincos_fast(__fmul_rn(c0, x), &s[0], &co[0]);
#pragma unroll
  for (int k = 1; k < kFreqs; ++k) {
    s[k] = 2.0f * (s[k - 1] * co[k - 1]);
    co[k] = fmaf(-2.0f * s[k - 1], s[k - 1], 1.0f);
  }
}

// kNoPi: the original NeRF implementation's encoding sin(2^k x), cos(2^k x) (no pi; the
// teacher layout of SURVEY §8f row 1), accurate path only.
__device__ __forceinline__ float enc_coef(int k, bool no_pi) { return no_pi ? __builtin_ldexpf(1.0f, k) : pe_coef(k); }

template <bool kFast = false, bool kOcml = false, bool kNoPi = false>
__device__ __forceinline__ void pos_encode(float x0, float x1, float x2, int h, float (&pe)[32]) {
  static_assert(!(kFast && kNoPi), "the no-pi encoding has the accurate path only");
  const float xs[3] = {x0, x1, x2};
  if (kFast) {
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      float s[5], co[5];
      sincos_doubling<5>(pe_coef(5 * h), xs[m], s, co);
#pragma unroll
      for (int kk = 0; kk < 5; ++kk) {
        pe[6 * kk + m] = s[kk];
        pe[6 * kk + 3 + m] = co[kk];
      }
    }
  } else {
#pragma unroll
    for (int kk = 0; kk < 5; ++kk) {
      const float c = enc_coef(5 * h + kk, kNoPi);
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        float s, co;
        pe_sincos<false, kOcml>(c, xs[m], &s, &co);
        pe[6 * kk + m] = s;
        pe[6 * kk + 3 + m] = co;
      }
    }
  }
  pe[30] = h ? x2 : x0;
  pe[31] = h ? 0.0f : x1;
}

template <bool kFast = false, bool kOcml = false, bool kNoPi = false>
__device__ __forceinline__ void dir_encode(float d0, float d1, float d2, int h, float (&de)[16]) {
  static_assert(!(kFast && kNoPi), "the no-pi encoding has the accurate path only");
  const float ds[3] = {d0, d1, d2};
  if (kFast) {
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      float s[2], co[2];
      sincos_doubling<2>(pe_coef(2 * h), ds[m], s, co);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        de[6 * kk + m] = s[kk];
        de[6 * kk + 3 + m] = co[kk];
      }
    }
  } else {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const float c = enc_coef(2 * h + kk, kNoPi);
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        float s, co;
        pe_sincos<false, kOcml>(c, ds[m], &s, &co);
        de[6 * kk + m] = s;
        de[6 * kk + 3 + m] = co;
      }
    }
  }
  de[12] = h ? d2 : d0;
  de[13] = h ? 0.0f : d1;
  de[14] = 0.0f;
  de[15] = 0.0f;
}

// ReLU on the bit pattern: a negative float is a negative int32 and max(bits, 0)
// is +0 for it, x otherwise -- one v_max_i32 (a float max needs a NaN
// canonicalisation first: two instructions).  A NaN stays a NaN when its sign
// bit is clear, as torch.relu propagates it.
__device__ __forceinline__ float relu(float x) {
  return __builtin_bit_cast(float, __builtin_elementwise_max(__builtin_bit_cast(int, x), 0));
}

// torch.sigmoid: 1 / (1 + exp(-x))
__device__ __forceinline__ float sigmoid_ref(float x) { return __fdiv_rn(1.0f, __fadd_rn(1.0f, expf(-x))); }

// Density (nerf.py:114) and colour-1 + sigmoid (nerf.py:123-129) from the
// ReLU'd fp32 accumulators.  prm points at the params blob (LDS or global).
// Each lane sums its 128 (resp. 64) rows; the two lane halves of a column then
// add through a cross-half swap.
template <typename PTR>
__device__ __forceinline__ float density_head(const f32x16 (&x)[8], PTR prm, int h) {
  float part = 0.0f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    asm volatile("" ::: "memory");   // keep one tile of weights in flight, not all 128
    const f32x4* w4 = (const f32x4*)(prm + kSigW + (h * 8 + t) * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 w = w4[q];
#pragma unroll
      for (int i = 0; i < 4; ++i) part = fmaf(w[i], x[t][4 * q + i], part);
    }
  }
  const float tot = part + __shfl_xor(part, 32);
  return relu(tot + prm[kSigB]);
}

template <typename PTR>
__device__ __forceinline__ void color_head(const f32x16 (&hc)[8], PTR prm, int h, float (&rgb)[3]) {  // tiles 0..3
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float part = 0.0f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      asm volatile("" ::: "memory");
      const f32x4* w4 = (const f32x4*)(prm + kC1W + ((c * 2 + h) * 4 + t) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 w = w4[q];
#pragma unroll
        for (int i = 0; i < 4; ++i) part = fmaf(w[i], hc[t][4 * q + i], part);
      }
    }
    const float tot = part + __shfl_xor(part, 32);
    rgb[c] = sigmoid_ref(tot + prm[kC1B + c]);
  }
}

// Bias pre-load: accumulator register r of tile o for lane half h.
template <int NT, typename PTR>
__device__ __forceinline__ void load_bias(f32x16 (&acc)[8], PTR prm, int layer, int h) {
#pragma unroll
  for (int o = 0; o < NT; ++o) {
    const f32x4* b4 = (const f32x4*)(prm + kBiasOff + 256 * layer + (o * 2 + h) * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 b = b4[q];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[o][4 * q + i] = b[i];
    }
  }
}

template <int NT>
__device__ __forceinline__ void relu_tiles(f32x16 (&acc)[8]) {
#pragma unroll
  for (int o = 0; o < NT; ++o)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[o][r] = relu(acc[o][r]);
}

// Where a wave's 32 sample columns come from.
struct SampleSrc {
  const float* rays_o;     // [n_rays][3]        (mode 0)
  const float* rays_d;     // [n_rays][3]
  const float* z;          // z[ray*z_stride + s]
  int z_stride;
  int n_samples;
  const float* points;     // [P][3]             (mode 1: explicit points)
  const float* dirs;       // [P][3]
};

// Fetch the sample point and its view direction for sample p.
template <bool kExplicit>
__device__ __forceinline__ void fetch_sample(const SampleSrc& src, long p, float (&x)[3], float (&d)[3]) {
  if (kExplicit) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      x[c] = src.points[3 * p + c];
      d[c] = src.dirs[3 * p + c];
    }
  } else {
    const long ray = p / src.n_samples;
    const long s = p - ray * src.n_samples;
    const float zz = src.z[ray * src.z_stride + s];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      d[c] = src.rays_d[3 * ray + c];
      x[c] = sample_coord(src.rays_o[3 * ray + c], d[c], zz);
    }
  }
}

// ---- Compositing fused into the MLP epilogue (bf16 / fp8 render passes) ----
// The volume integral of execute_volume_rendering (pytorch_renderers.py:105-125)
// is associative over consecutive samples of a ray.  With S % 32 == 0 a wave's
// 32-sample column tile is one "segment" of one ray, so each wave composites
// its own segment in registers, and only a 32-B record per segment leaves the
// kernel (instead of 16 B per sample):
//   P      = prod_i (1 - alpha_i + 1e-10)            (double)
//   rgb, d = sum_i alpha_i * float(P_<i) * (c_i, z_i)  (fp32, P_<i the in-segment
//                                                        exclusive product)
// and composite_segments_kernel chains the records of a ray:
//   out = sum_k float(T_k) * part_k,  T_{k+1} = T_k * P_k  (double),
// which is the reference's sequential sum regrouped (differences at fp32
// rounding level; the fp32 parity path keeps the sequential kernel).
struct SegRecord {      // 32 B; written as two f32x4 by lanes 0 and 1 of the segment
  double P;
  float r, g, b, depth, acc, pad;
};
static_assert(sizeof(SegRecord) == 32, "segment record is two 16-B stores");

// Sample point, view direction and -- for fused compositing (seg) -- the
// integral's network-independent inputs of render-pass sample p:
// dist = (z_{s+1} - z_s, or 1e10 for the ray's last sample) * |d| and z_s, in the
// reference's operation order (pytorch_renderers.py:106-112).  idx32 (wave-
// uniform: the launch has fewer than 2^32 samples) divides in 32 bits.
__device__ __forceinline__ void fetch_render_sample(const SampleSrc& src, long p, bool idx32, bool seg,
                                                    float (&x)[3], float (&d)[3], float& dist, float& z) {
  const long ray = idx32 ? long(unsigned(p) / unsigned(src.n_samples)) : p / src.n_samples;
  const int s = int(p - ray * src.n_samples);
  const float* zr = src.z + ray * src.z_stride;
  z = zr[s];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    d[c] = src.rays_d[3 * ray + c];
    x[c] = sample_coord(src.rays_o[3 * ray + c], d[c], z);
  }
  if (seg) {
    const float norm = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(d[0], d[0]), __fmul_rn(d[1], d[1])), __fmul_rn(d[2], d[2])));
    const float delta = s + 1 < src.n_samples ? __fsub_rn(zr[s + 1], z) : 1e10f;
    dist = __fmul_rn(delta, norm);
  }
}

// DPP moves within 32-lane segments (gfx9 encodings): row_shr:n = 0x110+n,
// row_bcast:15 = 0x142 (rows 1 and 3 take lane 15 of the row below: row_mask
// 0xa), wave_shr:1 = 0x138.  Lanes without a source keep `identity`.
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ float dpp_f32(float v, float identity) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, identity),
                                                               __builtin_bit_cast(int, v), kCtrl, kRowMask, 0xf, false));
}
template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ double dpp_f64(double v, double identity) {
  typedef int i32x2_t __attribute__((ext_vector_type(2)));
  const i32x2_t vi = __builtin_bit_cast(i32x2_t, v), oi = __builtin_bit_cast(i32x2_t, identity);
  const i32x2_t r{__builtin_amdgcn_update_dpp(oi[0], vi[0], kCtrl, kRowMask, 0xf, false),
                  __builtin_amdgcn_update_dpp(oi[1], vi[1], kCtrl, kRowMask, 0xf, false)};
  return __builtin_bit_cast(double, r);
}
// inclusive scans over each 32-lane segment (Hillis-Steele within 16-lane rows,
// then row 1 (3) folds in lane 15 (47))
__device__ __forceinline__ double seg_scan_mul(double v) {
  v = __dmul_rn(dpp_f64<0x111>(v, 1.0), v);
  v = __dmul_rn(dpp_f64<0x112>(v, 1.0), v);
  v = __dmul_rn(dpp_f64<0x114>(v, 1.0), v);
  v = __dmul_rn(dpp_f64<0x118>(v, 1.0), v);
  return __dmul_rn(dpp_f64<0x142, 0xa>(v, 1.0), v);
}
__device__ __forceinline__ float seg_scan_add(float v) {
  v = __fadd_rn(dpp_f32<0x111>(v, 0.0f), v);
  v = __fadd_rn(dpp_f32<0x112>(v, 0.0f), v);
  v = __fadd_rn(dpp_f32<0x114>(v, 0.0f), v);
  v = __fadd_rn(dpp_f32<0x118>(v, 0.0f), v);
  return __fadd_rn(dpp_f32<0x142, 0xa>(v, 0.0f), v);
}
__device__ __forceinline__ float lane31(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 31));
}

// Composite the segment held by lanes 0..31 (sample j of the segment in lane j;
// lanes 32..63 scan their own copy, which no caller stores).  v = (sigma, r, g, b).
// Returns this lane's 16 B of the record (even lanes: P, r, g; odd: b, depth, acc, 0)
// and, in w_local, its sample's in-segment weight alpha * float(P_<j) (the
// hierarchical coarse pass turns it into the sample's weight with the product of
// the earlier segments' P: importance_wave_kernel).
__device__ __forceinline__ f32x4 seg_composite(f32x4 v, float dist, float z, int lane, float& w_local) {
  const float alpha = __fsub_rn(1.0f, expf(__fmul_rn(-relu(v[0]), dist)));
  const double P = seg_scan_mul(double(__fadd_rn(__fsub_rn(1.0f, alpha), 1e-10f)));
  const double Pex = dpp_f64<0x138>(P, 1.0);                   // exclusive: lane j takes lane j-1, lane 0 1.0
  const float w = __fmul_rn(alpha, float(Pex));
  w_local = w;
  const float r = lane31(seg_scan_add(__fmul_rn(w, v[1])));
  const float g = lane31(seg_scan_add(__fmul_rn(w, v[2])));
  const float b = lane31(seg_scan_add(__fmul_rn(w, v[3])));
  const float dep = lane31(seg_scan_add(__fmul_rn(w, z)));
  const float acc = lane31(seg_scan_add(w));
  const f32x2_t Pseg = __builtin_bit_cast(f32x2_t, P);
  const f32x4 lo{lane31(Pseg[0]), lane31(Pseg[1]), r, g};
  const f32x4 hi{b, dep, acc, 0.0f};
  return (lane & 1) ? hi : lo;
}

}  // namespace nerf
