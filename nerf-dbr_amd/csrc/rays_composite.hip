// Ray generation, alpha compositing and the inverse-CDF importance sampler.
// These are byte-light, per-ray kernels (<1% of frame time); what matters is
// that they follow the reference's arithmetic operation for operation.
#include "nerf_device.h"
#include "nerf_internal.h"

namespace nerf {
namespace {

struct Pose {
  float r[9];   // camera-to-world rotation, row-major
  float t[3];
};

// BaseUnifiedRenderer.generate_rays (base_renderer.py:223-258):
//   dir = ((i - W*0.5)/f, -(j - H*0.5)/f, -1)  with pixel corners i, j;
//   rays_d[k] = (dir0*R[k][0] + dir1*R[k][1]) + dir2*R[k][2]  (torch.sum order);
//   rays_o = t.  One thread per pixel of rows [row0, row1).
__global__ void rays_kernel(Pose pose, int width, float half_w, float half_h, float focal, int row0, long n,
                            float* __restrict__ rays_o, float* __restrict__ rays_d) {
  const long k = long(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int row = row0 + int(k / width);
  const int col = int(k % width);
  const float dx = __fdiv_rn(__fsub_rn(float(col), half_w), focal);
  const float dy = -__fdiv_rn(__fsub_rn(float(row), half_h), focal);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float p0 = __fmul_rn(dx, pose.r[3 * c + 0]);
    const float p1 = __fmul_rn(dy, pose.r[3 * c + 1]);
    const float p2 = -pose.r[3 * c + 2];
    rays_d[3 * k + c] = __fadd_rn(__fadd_rn(p0, p1), p2);
    rays_o[3 * k + c] = pose.t[c];
  }
}

// execute_volume_rendering (pytorch_renderers.py:105-125): one thread per ray.
// Transmittance is the exclusive product of (1 - alpha + 1e-10) accumulated the
// way torch's CPU cumprod does it: sequentially in double, each output rounded
// to fp32 (ATen cpu_cum_base_kernel uses acc_type<float> = double).
__global__ void composite_kernel(const float* __restrict__ sigma, int sigma_stride, const float* __restrict__ rgb,
                                 int rgb_stride, const float* __restrict__ z, int z_ray_stride,
                                 const float* __restrict__ rays_d, int n_rays, int n_samples,
                                 float* __restrict__ rgb_out, float* __restrict__ depth_out, OutStrides os,
                                 float* __restrict__ acc_out, float* __restrict__ weights_out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  if (n_samples == 1) {
    // The reference's quirk, kept for drop-in parity: with one sample,
    // `dists[..., :1]` of the empty difference tensor is empty, so every
    // per-sample array is empty and the image is all zeros
    // (pytorch_renderers.py:107-108; same in rendering.py:105-106).
    float* o = rgb_out + long(os.rgb) * r;
    o[0] = o[1] = o[2] = 0.0f;
    depth_out[long(os.depth) * r] = 0.0f;
    if (acc_out) acc_out[r] = 0.0f;
    return;
  }
  const float dx = rays_d[3L * r], dy = rays_d[3L * r + 1], dz = rays_d[3L * r + 2];
  const float norm = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
  const float* zr = z + long(r) * z_ray_stride;
  const long base = long(r) * n_samples;
  double T_acc = 1.0;
  float cr = 0.0f, cg = 0.0f, cb = 0.0f, dep = 0.0f, acc = 0.0f;
  float z_cur = zr[0];
  for (int s = 0; s < n_samples; ++s) {
    const float z_next = s + 1 < n_samples ? zr[s + 1] : 0.0f;
    const float dist = __fmul_rn(s + 1 < n_samples ? __fsub_rn(z_next, z_cur) : 1e10f, norm);
    const float sg = relu(sigma[(base + s) * sigma_stride]);
    const float alpha = __fsub_rn(1.0f, expf(__fmul_rn(-sg, dist)));
    const float w = __fmul_rn(alpha, float(T_acc));
    const float* c = rgb + (base + s) * rgb_stride;
    cr = __fadd_rn(cr, __fmul_rn(w, c[0]));
    cg = __fadd_rn(cg, __fmul_rn(w, c[1]));
    cb = __fadd_rn(cb, __fmul_rn(w, c[2]));
    dep = __fadd_rn(dep, __fmul_rn(w, z_cur));
    acc = __fadd_rn(acc, w);
    if (weights_out) weights_out[base + s] = w;
    T_acc = __dmul_rn(T_acc, double(__fadd_rn(__fsub_rn(1.0f, alpha), 1e-10f)));
    z_cur = z_next;
  }
  float* o = rgb_out + long(os.rgb) * r;
  o[0] = cr;
  o[1] = cg;
  o[2] = cb;
  depth_out[long(os.depth) * r] = dep;
  if (acc_out) acc_out[r] = acc;
}

// Fixed VolumeRenderer.importance_sample (rendering.py:54-100; the reference's
// gather at :89-90 crashes): pdf = (w+1e-5)/sum; the sum and the cdf are
// torch-CPU cumsums (sequential, double accumulator, fp32 outputs);
// u ascending per ray (inverse CDF is monotone, so the importance samples come
// out sorted and merge with the sorted coarse z in one pass).
constexpr int kMaxCoarse = 256;
__global__ void importance_kernel(const float* __restrict__ z_coarse, int z_ray_stride,
                                  const float* __restrict__ weights, const float* __restrict__ u,
                                  int u_ray_stride, int n_rays, int n_coarse, int n_importance,
                                  float* __restrict__ z_fine) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  const float* zr = z_coarse + long(r) * z_ray_stride;
  const float* wr = weights + long(r) * n_coarse;
  const float* ur = u + long(r) * u_ray_stride;
  float* out = z_fine + long(r) * (n_coarse + n_importance);
  float cdf[kMaxCoarse + 1];
  double sum = 0.0;
  for (int i = 0; i < n_coarse; ++i) sum = __dadd_rn(sum, double(__fadd_rn(wr[i], 1e-5f)));
  const float total = float(sum);
  cdf[0] = 0.0f;
  sum = 0.0;
  for (int i = 0; i < n_coarse; ++i) {
    sum = __dadd_rn(sum, double(__fdiv_rn(__fadd_rn(wr[i], 1e-5f), total)));
    cdf[i + 1] = float(sum);
  }
  int ic = 0;        // next coarse sample to emit
  int o = 0;
  int lo = 0;        // searchsorted hint: u ascending
  for (int k = 0; k < n_importance; ++k) {
    const float uk = ur[k];
    // torch.searchsorted(cdf, u, right=True): count of cdf entries <= u
    int idx = lo;
    while (idx <= n_coarse && cdf[idx] <= uk) ++idx;
    lo = idx;
    const int below = min(max(idx - 1, 0), n_coarse - 1);
    const int above = min(max(idx, 0), n_coarse - 1);
    const float cb = cdf[below], ca = cdf[above];
    float denom = __fsub_rn(ca, cb);
    if (denom < 1e-5f) denom = 1.0f;
    const float t = __fdiv_rn(__fsub_rn(uk, cb), denom);
    const float zb = zr[below];
    const float zs = __fadd_rn(zb, __fmul_rn(t, __fsub_rn(zr[above], zb)));
    while (ic < n_coarse && zr[ic] <= zs) out[o++] = zr[ic++];
    out[o++] = zs;
  }
  while (ic < n_coarse) out[o++] = zr[ic++];
}

// The same sampler, one wave per ray, bit-identical to importance_kernel:
//  * the normaliser and the cdf are the same sequential double sums -- every lane
//    runs the same ordered loop over the ray's weights (LDS broadcast reads) and
//    keeps the cdf entries of its own indices, so no per-thread array (scratch);
//  * searchsorted(cdf, u, right=True) is a binary search for the count of cdf
//    entries <= u, which equals the linear scan on a nondecreasing cdf;
//  * the merge writes every sample at its rank: importance sample k lands at
//    k + #{coarse z <= z_k}, coarse sample i at i + #{importance z < z_i} --
//    the sequential merge's order whenever both lists are nondecreasing (true for
//    sorted z and ascending u); otherwise lane 0 merges sequentially.
constexpr int kMaxImpWave = 1024;
constexpr int kSegSamples = 32;     // samples per segment record (nerf_device.h SegRecord)
constexpr int kImpWaves = 4;

__device__ __forceinline__ int count_le(const float* a, int n, float v) {   // #{i < n : a[i] <= v}
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int count_lt(const float* a, int n, float v) {   // #{i < n : a[i] < v}
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(64 * kImpWaves) void importance_wave_kernel(
    const float* __restrict__ z_coarse, int z_ray_stride, const float* __restrict__ weights,
    const float* __restrict__ u, int u_ray_stride, int n_rays, int n_coarse, int n_importance,
    float* __restrict__ z_fine, const SegRecord* __restrict__ seg) {
  __shared__ float s_a[kImpWaves][kMaxCoarse];
  __shared__ float s_cdf[kImpWaves][kMaxCoarse + 1];
  __shared__ float s_z[kImpWaves][kMaxCoarse];
  __shared__ float s_zs[kImpWaves][kMaxImpWave];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long r = long(blockIdx.x) * kImpWaves + wv;
  if (r >= n_rays) return;                                     // wave-uniform
  const float* zr = z_coarse + r * z_ray_stride;
  const float* wr = weights + r * n_coarse;
  const float* ur = u + r * u_ray_stride;
  float* out = z_fine + r * (n_coarse + n_importance);
  float* a = s_a[wv];
  float* cdf = s_cdf[wv];
  float* zc = s_z[wv];
  float* zs = s_zs[wv];
  for (int i = lane; i < n_coarse; i += 64) {
    float w = wr[i];
    if (seg != nullptr) {
      // fused coarse pass: w is the in-segment weight; the transmittance at the
      // segment's start is the product of the earlier records' P (double)
      const SegRecord* sr = seg + r * (n_coarse / kSegSamples);
      double T = 1.0;
      for (int k = 0; k < i / kSegSamples; ++k) T = __dmul_rn(T, sr[k].P);
      w = __fmul_rn(w, float(T));
    }
    a[i] = __fadd_rn(w, 1e-5f);
    zc[i] = zr[i];
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (lane == 0) cdf[0] = 0.0f;
  // Parallel form when it is provably exact.  A double sum of floats is exact in
  // any order when every partial sum fits in 53 bits: for the normaliser, when
  // e(max) + ceil(log2 n) - (e(min) - 24) <= 53 (e: frexp exponents, so the
  // smallest value's last bit is 2^(e(min)-24)); for the cdf (sums < 2), when the
  // smallest pdf has e >= -28.  Weights in [0, 1] (every composite output) give
  // spreads far inside both; otherwise every lane runs the sequential sums.
  const int per = (n_coarse + 63) >> 6;                       // elements per lane, contiguous
  const int i0 = min(lane * per, n_coarse), i1 = min(i0 + per, n_coarse);
  float amin = __builtin_inff(), amax = 0.0f;
  bool finite_pos = true;
  for (int i = i0; i < i1; ++i) {
    finite_pos = finite_pos && a[i] > 0.0f && a[i] < __builtin_inff();
    amin = fminf(amin, a[i]);
    amax = fmaxf(amax, a[i]);
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    amin = fminf(amin, __shfl_xor(amin, d));
    amax = fmaxf(amax, __shfl_xor(amax, d));
  }
  int log2n = 0;
  while ((1 << log2n) < n_coarse) ++log2n;
  bool exact = __all(finite_pos) &&
               __builtin_amdgcn_frexp_expf(amax) + log2n - (__builtin_amdgcn_frexp_expf(amin) - 24) <= 53;
  if (exact) {
    double loc = 0.0;
    for (int i = i0; i < i1; ++i) loc = __dadd_rn(loc, double(a[i]));
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) loc = __dadd_rn(loc, __shfl_xor(loc, d));
    const float total = float(loc);
    exact = __builtin_amdgcn_frexp_expf(__fdiv_rn(amin, total)) >= -28;   // wave-uniform (amin, total are)
    if (exact) {
      double part = 0.0;
      for (int i = i0; i < i1; ++i) part = __dadd_rn(part, double(__fdiv_rn(a[i], total)));
      double incl = part;                                     // inclusive scan over lanes
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const double o = __shfl_up(incl, d);
        if (lane >= d) incl = __dadd_rn(incl, o);
      }
      double run = __dsub_rn(incl, part);                     // exclusive: exact, so no rounding
      for (int i = i0; i < i1; ++i) {
        run = __dadd_rn(run, double(__fdiv_rn(a[i], total)));
        cdf[i + 1] = float(run);
      }
    }
  }
  if (!exact) {
    double sum = 0.0;
    for (int i = 0; i < n_coarse; ++i) sum = __dadd_rn(sum, double(a[i]));
    const float total = float(sum);
    sum = 0.0;
    for (int i = 0; i < n_coarse; ++i) {
      sum = __dadd_rn(sum, double(__fdiv_rn(a[i], total)));
      if ((i & 63) == lane) cdf[i + 1] = float(sum);
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  bool mono = true;
  for (int k = lane; k < n_importance; k += 64) {
    const float uk = ur[k];
    const int idx = count_le(cdf, n_coarse + 1, uk);
    const int below = min(max(idx - 1, 0), n_coarse - 1);
    const int above = min(max(idx, 0), n_coarse - 1);
    const float cb = cdf[below], ca = cdf[above];
    float denom = __fsub_rn(ca, cb);
    if (denom < 1e-5f) denom = 1.0f;
    const float t = __fdiv_rn(__fsub_rn(uk, cb), denom);
    const float zb = zc[below];
    zs[k] = __fadd_rn(zb, __fmul_rn(t, __fsub_rn(zc[above], zb)));
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  for (int k = lane + 1; k < n_importance; k += 64) mono = mono && !(zs[k] < zs[k - 1]);
  for (int i = lane + 1; i < n_coarse; i += 64) mono = mono && !(zc[i] < zc[i - 1]);
  if (__all(mono)) {
    for (int k = lane; k < n_importance; k += 64) out[k + count_le(zc, n_coarse, zs[k])] = zs[k];
    for (int i = lane; i < n_coarse; i += 64) out[i + count_lt(zs, n_importance, zc[i])] = zc[i];
  } else if (lane == 0) {
    int ic = 0, o = 0;
    for (int k = 0; k < n_importance; ++k) {
      while (ic < n_coarse && zc[ic] <= zs[k]) out[o++] = zc[ic++];
      out[o++] = zs[k];
    }
    while (ic < n_coarse) out[o++] = zc[ic++];
  }
}

// Compositing of the render path's packed MLP output (sigma, r, g, b) per
// sample: the arithmetic of composite_kernel, with 16-B loads issued eight
// samples at a time (whole cache lines per request).
__global__ void composite_packed_kernel(const f32x4* __restrict__ mlp, const float* __restrict__ z, int z_ray_stride,
                                        const float* __restrict__ rays_d, int n_rays, int n_samples,
                                        float* __restrict__ rgb_out, float* __restrict__ depth_out, OutStrides os,
                                        float* __restrict__ acc_out, float* __restrict__ weights_out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  const float dx = rays_d[3L * r], dy = rays_d[3L * r + 1], dz = rays_d[3L * r + 2];
  const float norm = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
  const float* zr = z + long(r) * z_ray_stride;
  const long base = long(r) * n_samples;
  double T_acc = 1.0;
  float cr = 0.0f, cg = 0.0f, cb = 0.0f, dep = 0.0f, acc = 0.0f;
  for (int s0 = 0; s0 < n_samples; s0 += 8) {
    f32x4 v[8];
    float zz[9];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = s0 + j < n_samples ? mlp[base + s0 + j] : f32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 9; ++j) zz[j] = s0 + j < n_samples ? zr[s0 + j] : 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int s = s0 + j;
      if (s >= n_samples) break;
      const float dist = __fmul_rn(s + 1 < n_samples ? __fsub_rn(zz[j + 1], zz[j]) : 1e10f, norm);
      const float alpha = __fsub_rn(1.0f, expf(__fmul_rn(-relu(v[j][0]), dist)));
      const float w = __fmul_rn(alpha, float(T_acc));
      cr = __fadd_rn(cr, __fmul_rn(w, v[j][1]));
      cg = __fadd_rn(cg, __fmul_rn(w, v[j][2]));
      cb = __fadd_rn(cb, __fmul_rn(w, v[j][3]));
      dep = __fadd_rn(dep, __fmul_rn(w, zz[j]));
      acc = __fadd_rn(acc, w);
      if (weights_out) weights_out[base + s] = w;
      T_acc = __dmul_rn(T_acc, double(__fadd_rn(__fsub_rn(1.0f, alpha), 1e-10f)));
    }
  }
  float* o = rgb_out + long(os.rgb) * r;
  o[0] = cr;
  o[1] = cg;
  o[2] = cb;
  depth_out[long(os.depth) * r] = dep;
  if (acc_out) acc_out[r] = acc;
}

// Second half of the compositing fused into the bf16 / fp8 MLP epilogue
// (nerf_device.h SegRecord): chain a ray's segment records in order,
//   rgb += float(T) * rgb_k, depth += float(T) * depth_k, T *= P_k (double),
// the regrouped form of composite_kernel's sequential sums.  One thread per ray.
__global__ void composite_segments_kernel(const SegRecord* __restrict__ seg, int n_rays, int n_segments,
                                          float* __restrict__ rgb_out, float* __restrict__ depth_out, OutStrides os) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  const SegRecord* sr = seg + long(r) * n_segments;
  double T = 1.0;
  float cr = 0.0f, cg = 0.0f, cb = 0.0f, dep = 0.0f;
  for (int k = 0; k < n_segments; ++k) {
    const SegRecord rec = sr[k];
    const float t = float(T);
    cr = __fadd_rn(cr, __fmul_rn(t, rec.r));
    cg = __fadd_rn(cg, __fmul_rn(t, rec.g));
    cb = __fadd_rn(cb, __fmul_rn(t, rec.b));
    dep = __fadd_rn(dep, __fmul_rn(t, rec.depth));
    T = __dmul_rn(T, rec.P);
  }
  float* o = rgb_out + long(os.rgb) * r;
  o[0] = cr;
  o[1] = cg;
  o[2] = cb;
  depth_out[long(os.depth) * r] = dep;
}

// Sample depths and points, one thread per (ray, sample).
// Uniform (BaseUnifiedRenderer.sample_points_on_rays, base_renderer.py:260-281):
//   z = table[s] (near*(1-t)+far*t, built on the host bit-exactly).
// Stratified (VolumeRenderer.sample_points_on_rays perturb=True, rendering.py:42-47,
// with torch.rand_like injected as t_rand [n_rays][S]):
//   mids_j = 0.5*(z[j+1]+z[j]); lower = [z0, mids]; upper = [mids, z_{S-1}];
//   z' = lower + (upper-lower)*t_rand.
// Points (rendering.py:50 / base_renderer.py:279): o + d*z, multiply then add.
__global__ void sample_kernel(const float* __restrict__ z_tab, const float* __restrict__ t_rand, int n_samples,
                              long n, const float* __restrict__ rays_o, const float* __restrict__ rays_d,
                              float* __restrict__ z_out, float* __restrict__ points_out) {
  const long i = long(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = int(i % n_samples);
  const long r = i / n_samples;
  float z = z_tab[s];
  if (t_rand) {
    const float lower = s == 0 ? z_tab[0] : __fmul_rn(0.5f, __fadd_rn(z_tab[s], z_tab[s - 1]));
    const float upper = s == n_samples - 1 ? z_tab[s] : __fmul_rn(0.5f, __fadd_rn(z_tab[s + 1], z_tab[s]));
    z = __fadd_rn(lower, __fmul_rn(__fsub_rn(upper, lower), t_rand[i]));
  }
  z_out[i] = z;
  if (points_out) {
#pragma unroll
    for (int c = 0; c < 3; ++c) points_out[3 * i + c] = __fadd_rn(rays_o[3 * r + c], __fmul_rn(rays_d[3 * r + c], z));
  }
}

// PositionalEncoding.encode (nerf.py:31-45) through the MLP kernels' own device
// code (nerf_device.h pos_encode / dir_encode): one thread per (sample, lane
// half h), each half writing the features its slots own (pe_slot_feature /
// dpe_slot_feature), so the result is exactly what the kernels feed the MFMAs
// before rounding to bf16 / e4m3.
template <bool kFast, bool kPos>
__global__ void encode_kernel(const float* __restrict__ x, long n, float* __restrict__ out) {
  const long i = long(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= 2 * n) return;
  const long p = i >> 1;
  const int h = int(i & 1);
  const float x0 = x[3 * p], x1 = x[3 * p + 1], x2 = x[3 * p + 2];
  if (kPos) {
    float pe[32];
    pos_encode<kFast>(x0, x1, x2, h, pe);
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int f = pe_slot_feature(h, q);
      if (f >= 0) out[p * kPosDim + f] = pe[q];
    }
  } else {
    float de[16];
    dir_encode<kFast>(x0, x1, x2, h, de);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int f = dpe_slot_feature(h, q);
      if (f >= 0) out[p * kDirDim + f] = de[q];
    }
  }
}

}  // namespace

hipError_t launch_sample(const float* z_tab, const float* t_rand, int n_rays, int n_samples, const float* rays_o,
                         const float* rays_d, float* z_out, float* points_out, hipStream_t stream) {
  const long n = long(n_rays) * n_samples;
  if (n <= 0) return hipSuccess;
  const int threads = 256;
  const dim3 grid{unsigned((n + threads - 1) / threads), 1, 1}, block{threads, 1, 1};
  hipLaunchKernelGGL(sample_kernel, grid, block, 0, stream, z_tab, t_rand, n_samples, n, rays_o, rays_d, z_out,
                     points_out);
  return hipGetLastError();
}

hipError_t launch_encode(const float* x, long n, int n_freqs, bool fast, float* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int threads = 256;
  const dim3 grid{unsigned((2 * n + threads - 1) / threads), 1, 1}, block{threads, 1, 1};
  if (n_freqs == kPosL) {
    if (fast) hipLaunchKernelGGL((encode_kernel<true, true>), grid, block, 0, stream, x, n, out);
    else hipLaunchKernelGGL((encode_kernel<false, true>), grid, block, 0, stream, x, n, out);
  } else if (n_freqs == kDirL) {
    if (fast) hipLaunchKernelGGL((encode_kernel<true, false>), grid, block, 0, stream, x, n, out);
    else hipLaunchKernelGGL((encode_kernel<false, false>), grid, block, 0, stream, x, n, out);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_generate_rays(const float* c2w, int width, int height, int row0, int row1, float focal,
                                float* rays_o, float* rays_d, hipStream_t stream) {
  Pose pose;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) pose.r[3 * i + j] = c2w[4 * i + j];
    pose.t[i] = c2w[4 * i + 3];
  }
  const long n = long(row1 - row0) * width;
  if (n <= 0) return hipSuccess;
  const int threads = 256;
  const dim3 grid{unsigned((n + threads - 1) / threads), 1, 1}, block{threads, 1, 1};
  // `width * 0.5` / `height * 0.5` are exact in fp32 for any image size we accept
  hipLaunchKernelGGL(rays_kernel, grid, block, 0, stream, pose, width, float(width) * 0.5f, float(height) * 0.5f,
                     focal, row0, n, rays_o, rays_d);
  return hipGetLastError();
}

hipError_t launch_composite(const float* sigma, int sigma_stride, const float* rgb, int rgb_stride, const float* z,
                            int z_ray_stride, const float* rays_d, int n_rays, int n_samples, float* rgb_out,
                            float* depth_out, float* acc_out, float* weights_out, hipStream_t stream, OutStrides os) {
  if (n_rays <= 0) return hipSuccess;
  const int threads = 128;
  const dim3 grid{unsigned((n_rays + threads - 1) / threads), 1, 1}, block{threads, 1, 1};
  if (sigma_stride == 4 && rgb_stride == 4 && rgb == sigma + 1 && n_samples > 1 &&
      (reinterpret_cast<uintptr_t>(sigma) & 15) == 0) {
    hipLaunchKernelGGL(composite_packed_kernel, grid, block, 0, stream, (const f32x4*)sigma, z, z_ray_stride, rays_d,
                       n_rays, n_samples, rgb_out, depth_out, os, acc_out, weights_out);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(composite_kernel, grid, block, 0, stream, sigma, sigma_stride, rgb, rgb_stride, z, z_ray_stride,
                     rays_d, n_rays, n_samples, rgb_out, depth_out, os, acc_out, weights_out);
  return hipGetLastError();
}

hipError_t launch_composite_segments(const float* seg, int n_rays, int n_segments, float* rgb_out, float* depth_out,
                                     hipStream_t stream, OutStrides os) {
  if (n_rays <= 0) return hipSuccess;
  const int threads = 256;
  const dim3 grid{unsigned((n_rays + threads - 1) / threads), 1, 1}, block{threads, 1, 1};
  hipLaunchKernelGGL(composite_segments_kernel, grid, block, 0, stream, (const SegRecord*)seg, n_rays, n_segments,
                     rgb_out, depth_out, os);
  return hipGetLastError();
}

hipError_t launch_importance(const float* z_coarse, int z_ray_stride, const float* weights, const float* u,
                             int u_ray_stride, int n_rays, int n_coarse, int n_importance, float* z_fine,
                             hipStream_t stream, const float* seg) {
  if (n_rays <= 0) return hipSuccess;
  if (n_coarse > kMaxCoarse) return hipErrorInvalidValue;
  if (n_importance <= kMaxImpWave) {
    const dim3 grid{unsigned((n_rays + kImpWaves - 1) / kImpWaves), 1, 1}, block{64 * kImpWaves, 1, 1};
    hipLaunchKernelGGL(importance_wave_kernel, grid, block, 0, stream, z_coarse, z_ray_stride, weights, u,
                       u_ray_stride, n_rays, n_coarse, n_importance, z_fine, (const SegRecord*)seg);
    return hipGetLastError();
  }
  const int threads = 64;
  const dim3 grid{unsigned((n_rays + threads - 1) / threads), 1, 1}, block{threads, 1, 1};
  hipLaunchKernelGGL(importance_kernel, grid, block, 0, stream, z_coarse, z_ray_stride, weights, u, u_ray_stride,
                     n_rays, n_coarse, n_importance, z_fine);
  return hipGetLastError();
}

}  // namespace nerf
