// Shape probe: does the chip hold a higher clock on v_mfma_f32_16x16x32_bf16
// than on v_mfma_f32_32x32x16_bf16 for the NeRF MLP's loop shape?
// Both kernels: 512-thread workgroups (8 waves, 2 per SIMD), one per CU, each
// wave owns 32 sample columns x 256 output rows in fp32 accumulators (128 VGPRs)
// and 256 k of bf16 B fragments (64 VGPRs); A fragments (weights) are re-read
// from a 32 KiB LDS slab, 1 KiB per wave-instruction; after each "layer" the
// accumulators are converted (cvt_pk_bf16 + pk_max_i16) into the next B.
// Random data.  Reports TFLOP/s and the in-kernel clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../nerf-dbr_amd/csrc/nerf_asm.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned cvt_relu_pair(float lo, float hi) {
  const bf16x2 p = __builtin_convertvector(f32x2{lo, hi}, bf16x2);
  const i16x2 m = __builtin_elementwise_max(__builtin_bit_cast(i16x2, p), i16x2(0));
  return __builtin_bit_cast(unsigned, m);
}

constexpr int kLayers = 8;

__global__ __launch_bounds__(512, 1) void k32(const u32x4* __restrict__ src, float* out, unsigned long long* clk, int reps) {
  __shared__ u32x4 lds[2048];   // 32 KiB
  for (int i = threadIdx.x; i < 2048; i += 512) lds[i] = src[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const unsigned lbase = nerf::lds_addr(&lds[0]) + lane * 16;
  u32x4 b[16];
  for (int u = 0; u < 16; ++u) b[u] = src[(u * 64 + lane + blockIdx.x) & 2047];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  f32x16 acc[8];
  for (int rep = 0; rep < reps; ++rep) {
    for (int l = 0; l < kLayers; ++l) {
#pragma unroll
      for (int o = 0; o < 8; ++o) acc[o] = f32x16{};
      bf16x8 ra[3][2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        ra[n][0] = nerf::ds_read_b128<bf16x8>(lbase, ((((n * 2) & 31) * 64) ^ 0) * 16);
        ra[n][1] = nerf::ds_read_b128<bf16x8>(lbase, ((((n * 2 + 1) & 31) * 64) ^ 0) * 16);
      }
#pragma unroll
      for (int n = 0; n < 64; ++n) {
        const int q = n >> 4, u = n & 15;
        if (n + 2 < 64) {
          const int m = n + 2, off = (m * 2) & 31, qq = m >> 4;
          ra[m % 3][0] = nerf::ds_read_b128<bf16x8>(lbase, (off * 64 + qq) * 16);
          ra[m % 3][1] = nerf::ds_read_b128<bf16x8>(lbase, ((off + 1) * 64 + qq) * 16);
        }
        nerf::wait_lgkm(n + 2 < 64 ? 4 : 2 * (63 - n));
        const bf16x8 bb = __builtin_bit_cast(bf16x8, b[u]);
        acc[2 * q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[n % 3][0], bb, acc[2 * q], 0, 0, 0);
        acc[2 * q + 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[n % 3][1], bb, acc[2 * q + 1], 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const f32x16& t = acc[u >> 1];
        const int s = (u & 1) * 8;
        b[u] = u32x4{cvt_relu_pair(t[s] * 0.0625f, t[s + 1] * 0.0625f), cvt_relu_pair(t[s + 2] * 0.0625f, t[s + 3] * 0.0625f),
                     cvt_relu_pair(t[s + 4] * 0.0625f, t[s + 5] * 0.0625f), cvt_relu_pair(t[s + 6] * 0.0625f, t[s + 7] * 0.0625f)};
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int u = 0; u < 16; ++u) s += __builtin_bit_cast(float, b[u][0]) + __builtin_bit_cast(float, b[u][3]);
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

__global__ __launch_bounds__(512, 1) void k16(const u32x4* __restrict__ src, float* out, unsigned long long* clk, int reps) {
  __shared__ u32x4 lds[2048];
  for (int i = threadIdx.x; i < 2048; i += 512) lds[i] = src[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const unsigned lbase = nerf::lds_addr(&lds[0]) + lane * 16;
  u32x4 b[2][8];
  for (int c = 0; c < 2; ++c)
    for (int u = 0; u < 8; ++u) b[c][u] = src[((c * 8 + u) * 64 + lane + blockIdx.x) & 2047];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  f32x4 acc[2][16];
  for (int rep = 0; rep < reps; ++rep) {
    for (int l = 0; l < kLayers; ++l) {
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int o = 0; o < 16; ++o) acc[c][o] = f32x4{};
      bf16x8 ra[3][2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        ra[n][0] = nerf::ds_read_b128<bf16x8>(lbase, (((n * 2) & 31) * 64) * 16);
        ra[n][1] = nerf::ds_read_b128<bf16x8>(lbase, (((n * 2 + 1) & 31) * 64) * 16);
      }
#pragma unroll
      for (int n = 0; n < 64; ++n) {
        const int g = n >> 3, u = n & 7;
        if (n + 2 < 64) {
          const int m = n + 2, off = (m * 2) & 31, gg = m >> 3;
          ra[m % 3][0] = nerf::ds_read_b128<bf16x8>(lbase, (off * 64 + gg) * 16);
          ra[m % 3][1] = nerf::ds_read_b128<bf16x8>(lbase, ((off + 1) * 64 + gg) * 16);
        }
        nerf::wait_lgkm(n + 2 < 64 ? 4 : 2 * (63 - n));
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const bf16x8 bb = __builtin_bit_cast(bf16x8, b[c][u]);
          acc[c][2 * g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra[n % 3][0], bb, acc[c][2 * g], 0, 0, 0);
          acc[c][2 * g + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra[n % 3][1], bb, acc[c][2 * g + 1], 0, 0, 0);
        }
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const f32x4& t0_ = acc[c][2 * u];
          const f32x4& t1_ = acc[c][2 * u + 1];
          b[c][u] = u32x4{cvt_relu_pair(t0_[0] * 0.0625f, t0_[1] * 0.0625f), cvt_relu_pair(t0_[2] * 0.0625f, t0_[3] * 0.0625f),
                          cvt_relu_pair(t1_[0] * 0.0625f, t1_[1] * 0.0625f), cvt_relu_pair(t1_[2] * 0.0625f, t1_[3] * 0.0625f)};
        }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int c = 0; c < 2; ++c)
    for (int u = 0; u < 8; ++u) s += __builtin_bit_cast(float, b[c][u][0]) + __builtin_bit_cast(float, b[c][u][3]);
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

// One wave per SIMD, two 32-sample columns per wave (accumulators in AGPRs):
// every A fragment read from LDS feeds two MFMAs, so LDS read bytes per FLOP halve.
__global__ __launch_bounds__(256, 1) void k32c2(const u32x4* __restrict__ src, float* out, unsigned long long* clk, int reps) {
  __shared__ u32x4 lds[2048];   // 32 KiB
  for (int i = threadIdx.x; i < 2048; i += 256) lds[i] = src[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const unsigned lbase = nerf::lds_addr(&lds[0]) + lane * 16;
  u32x4 b[2][16];
  for (int c = 0; c < 2; ++c)
    for (int u = 0; u < 16; ++u) b[c][u] = src[((c * 16 + u) * 64 + lane + blockIdx.x) & 2047];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  f32x16 acc[2][8];
  for (int rep = 0; rep < reps; ++rep) {
    for (int l = 0; l < kLayers; ++l) {
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int o = 0; o < 8; ++o) acc[c][o] = f32x16{};
      bf16x8 ra[3][2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        ra[n][0] = nerf::ds_read_b128<bf16x8>(lbase, (((n * 2) & 31) * 64) * 16);
        ra[n][1] = nerf::ds_read_b128<bf16x8>(lbase, (((n * 2 + 1) & 31) * 64) * 16);
      }
#pragma unroll
      for (int n = 0; n < 64; ++n) {
        const int q = n >> 4, u = n & 15;
        if (n + 2 < 64) {
          const int m = n + 2, off = (m * 2) & 31, qq = m >> 4;
          ra[m % 3][0] = nerf::ds_read_b128<bf16x8>(lbase, (off * 64 + qq) * 16);
          ra[m % 3][1] = nerf::ds_read_b128<bf16x8>(lbase, ((off + 1) * 64 + qq) * 16);
        }
        nerf::wait_lgkm(n + 2 < 64 ? 4 : 2 * (63 - n));
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const bf16x8 bb = __builtin_bit_cast(bf16x8, b[c][u]);
          acc[c][2 * q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[n % 3][0], bb, acc[c][2 * q], 0, 0, 0);
          acc[c][2 * q + 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[n % 3][1], bb, acc[c][2 * q + 1], 0, 0, 0);
        }
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const f32x16& t = acc[c][u >> 1];
          const int s = (u & 1) * 8;
          b[c][u] = u32x4{cvt_relu_pair(t[s] * 0.0625f, t[s + 1] * 0.0625f), cvt_relu_pair(t[s + 2] * 0.0625f, t[s + 3] * 0.0625f),
                          cvt_relu_pair(t[s + 4] * 0.0625f, t[s + 5] * 0.0625f), cvt_relu_pair(t[s + 6] * 0.0625f, t[s + 7] * 0.0625f)};
        }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int c = 0; c < 2; ++c)
    for (int u = 0; u < 16; ++u) s += __builtin_bit_cast(float, b[c][u][0]) + __builtin_bit_cast(float, b[c][u][3]);
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<unsigned> h(2048 * 4);
  srand(1);
  for (auto& v : h) {   // random bf16 pairs in about [-1, 1]
    auto rb = []() -> unsigned { float f = (rand() / (float)RAND_MAX) * 2.f - 1.f; unsigned u = __builtin_bit_cast(unsigned, f); return (u + 0x8000u) >> 16; };
    v = rb() | (rb() << 16);
  }
  u32x4* src; float* out; unsigned long long* clk;
  CK(hipMalloc(&src, h.size() * 4));
  CK(hipMalloc(&out, cus * 512 * 4));
  CK(hipMalloc(&clk, cus * 16));
  CK(hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const int reps = 40;
  const double flop = double(cus) * 8 /*waves*/ * reps * kLayers * 2.0 * 256 * 256 * 32;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<unsigned long long> hc(cus * 2);
  for (int round = 0; round < 6; ++round)
    for (int v = 0; v < 3; ++v) {
      for (int w = 0; w < 3; ++w) {   // back-to-back launches, then time the last
        if (v == 0) hipLaunchKernelGGL(k32, dim3(cus), dim3(512), 0, 0, src, out, clk, reps);
        else if (v == 1) hipLaunchKernelGGL(k16, dim3(cus), dim3(512), 0, 0, src, out, clk, reps);
        else hipLaunchKernelGGL(k32c2, dim3(cus), dim3(256), 0, 0, src, out, clk, reps);
      }
      CK(hipEventRecord(e0));
      for (int w = 0; w < 5; ++w) {
        if (v == 0) hipLaunchKernelGGL(k32, dim3(cus), dim3(512), 0, 0, src, out, clk, reps);
        else if (v == 1) hipLaunchKernelGGL(k16, dim3(cus), dim3(512), 0, 0, src, out, clk, reps);
        else hipLaunchKernelGGL(k32c2, dim3(cus), dim3(256), 0, 0, src, out, clk, reps);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipMemcpy(hc.data(), clk, cus * 16, hipMemcpyDeviceToHost));
      double ghz = 0;
      for (int i = 0; i < cus; ++i) ghz += double(hc[2 * i]) / double(hc[2 * i + 1]) * 0.1;
      printf("round %d %s: %.3f ms/launch  %.1f TFLOP/s  clock %.3f GHz\n", round, v == 2 ? "32x32x16, 4 waves x 2 cols" : v ? "16x16x32" : "32x32x16", ms / 5,
             flop / (ms / 5 * 1e-3) / 1e12, ghz / cus);
    }
  return 0;
}
