// Shape probe for the split-fp16 (f16x3) MLP loop: can two waves per SIMD on the
// 16x16x32 f16 MFMA (16 samples per wave, ~200 registers) beat the shipped shape, one
// wave per SIMD on 32x32x16 (32 samples per wave, ~420 registers)?  Both kernels run the
// real loop's skeleton on random operands: a 128-sample workgroup tile, 8 "layers" of
// 256 x 256 per tile, each product as three MFMAs (hi.hi + hi.lo + lo.hi), 4-KiB units
// (two output tiles' hi and lo A fragments) read from a 4-slot LDS ring that an LDS-DMA
// stream restages one 16-KiB chunk per 4 units (one s_barrier per chunk, as mlp_x3.h),
// the activations split into f16 hi / lo fragments (v_max_i32 ReLU, v_cvt_pk_f16_f32,
// v_fma_mix) as each group of output tiles is final, spread over the next group's units.
// Reports ms per launch, the MFMA-rate TFLOP/s (three MFMAs per product counted; the
// algorithmic rate is a third of it) and the in-kernel clock (s_memtime / s_memrealtime),
// each variant after seconds of back-to-back launches.  Not part of the library.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../nerf-dbr_amd/csrc/nerf_asm.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kLayers = 8;
constexpr int kChunkB = 16384;
constexpr int kSlots = 4;                            // 128 chunks per tile: slot = chunk-in-tile % 4
constexpr int kUnitB = 4096;
constexpr int kUnitsPerChunk = kChunkB / kUnitB;     // 4
constexpr int kUnitsPerTile = kLayers * 64;          // 512
constexpr int kChunksPerTile = kUnitsPerTile / kUnitsPerChunk;   // 128
static_assert(kChunksPerTile % kSlots == 0, "constant ring offsets across tiles");
constexpr int kBlobChunks = 132;
// ReLU'd activations keep their size from layer to layer (w ~ U(-0.25, 0.25): a 256-term
// sum has rms 2.31 x rms(x), ReLU leaves 1/sqrt(2) of it), so the MFMA operands stay
// random normal fp16 values as in the real network; a smaller factor decays them to zero
// within a few layers, and zero operands raise the clock (cdna_hip_programming.md 5.4 rule 25)
constexpr float kActScale = 0.6124f;

__device__ __forceinline__ float relu_i(float x) {
  return __builtin_bit_cast(float, __builtin_elementwise_max(__builtin_bit_cast(int, x), 0));
}
__device__ __forceinline__ void split_pair(float a, float b, unsigned& hi, unsigned& lo) {
  hi = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, f16x2));
  unsigned l;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(l) : "v"(hi), "v"(a), "v"(b));
  lo = l;
}

template <int kWaves>
__device__ __forceinline__ void stage(const char* blob, long g, char* lds, int wave, int lane) {
  constexpr int kPieces = kChunkB / (kWaves * 1024);
  const char* src = blob + (g % kChunksPerTile) * kChunkB;   // g folds to a constant
  char* dst = lds + ((g % kChunksPerTile) % kSlots) * kChunkB + wave * 1024;
#pragma unroll
  for (int i = 0; i < kPieces; ++i)
    nerf::lds_dma_16_s(src + i * kWaves * 1024, unsigned(wave * 1024 + lane * 16),
                       nerf::lds_addr(dst + i * kWaves * 1024));
}

template <int kWaves>
__device__ __forceinline__ void seam(const char* blob, long g_next, char* lds, int wave, int lane) {
  nerf::wait_vmcnt(0);
  nerf::compiler_fence();
  __builtin_amdgcn_s_barrier();
  nerf::compiler_fence();
  stage<kWaves>(blob, g_next, lds, wave, lane);
}

// ---- shipped shape: 4 waves (1 per SIMD), 32 samples per wave, v_mfma_f32_32x32x16_f16 --
constexpr int kPfA = 3;
__global__ __launch_bounds__(256, 1) void x3_32(const char* __restrict__ blob, float* out, unsigned long long* clk,
                                                int tiles) {
  __shared__ __attribute__((aligned(16))) char lds[kSlots * kChunkB];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned rb = nerf::lds_addr(lds) + lane * 16;
  stage<4>(blob, 0, lds, wave, lane);
  u32x4 iH[16], iL[16], oH[16], oL[16];
  for (int u = 0; u < 16; ++u) {
    iH[u] = ((const u32x4*)blob)[(u * 64 + lane + blockIdx.x) & 4095];
    iL[u] = ((const u32x4*)blob)[(u * 64 + lane + 7 * blockIdx.x + 1024) & 4095] & 0x03FF03FFu;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int tile = 0; tile < tiles; ++tile) {
    nerf::wait_vmcnt(0);            // the tile's chunk 0 (staged by the last seam) lands
    __syncthreads();
    const char* bl0 = blob;
    asm volatile("" : "+s"(bl0));   // keep the 128 chunk addresses out of SGPRs across tiles
    stage<4>(bl0, 1, lds, wave, lane);
    f16x8 ra[kPfA + 1][4];
#pragma unroll
    for (int m = 0; m < kPfA; ++m)
#pragma unroll
      for (int f = 0; f < 4; ++f)
        ra[m][f] = nerf::ds_read_b128<f16x8>(rb, int(((m / 4) % kSlots) * kChunkB + (m % 4) * kUnitB + f * 1024));
#pragma unroll
    for (int l = 0; l < kLayers; l += 2) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        u32x4(&bh)[16] = half ? oH : iH;
        u32x4(&bl)[16] = half ? oL : iL;
        u32x4(&ch)[16] = half ? iH : oH;
        u32x4(&cl)[16] = half ? iL : oL;
        f32x16 acc[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int u = 0; u < 16; ++u) {
            const int n = q * 16 + u;                           // unit within the layer
            const int lu = (l + half) * 64 + n;                 // unit within the tile
            if ((lu + kPfA) % 4 == 0 && lu + kPfA < kUnitsPerTile)
              seam<4>(bl0, (lu + kPfA) / 4 + 1, lds, wave, lane);
            if (u == 0) acc[2 * q] = acc[2 * q + 1] = f32x16{};
            const int m = lu + kPfA;
            if (m < kUnitsPerTile) {
#pragma unroll
              for (int f = 0; f < 4; ++f)
                ra[m % (kPfA + 1)][f] = nerf::ds_read_b128<f16x8>(
                    rb, int(((m / 4) % kSlots) * kChunkB + (m % 4) * kUnitB + f * 1024));
            }
            nerf::wait_lgkm(0);
            const f16x8 h = __builtin_bit_cast(f16x8, bh[u]), lo = __builtin_bit_cast(f16x8, bl[u]);
#pragma unroll
            for (int o = 0; o < 2; ++o) {
              f32x16 a = acc[2 * q + o];
              a = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[lu % (kPfA + 1)][o], h, a, 0, 0, 0);
              a = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[lu % (kPfA + 1)][o], lo, a, 0, 0, 0);
              acc[2 * q + o] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[lu % (kPfA + 1)][2 + o], h, a, 0, 0, 0);
            }
            // convert the previous quarter's two tiles, one dword pair per unit
            if (q >= 1) {
              const int t = 2 * (q - 1) + (u >> 3), pr = u & 7;
              unsigned hh, ll;
              split_pair(relu_i(acc[t][2 * pr] * kActScale), relu_i(acc[t][2 * pr + 1] * kActScale), hh, ll);
              ch[2 * t + (pr >> 2)][pr & 3] = hh;
              cl[2 * t + (pr >> 2)][pr & 3] = ll;
            }
          }
        }
#pragma unroll
        for (int t = 6; t < 8; ++t)
#pragma unroll
          for (int pr = 0; pr < 8; ++pr) {
            unsigned hh, ll;
            split_pair(relu_i(acc[t][2 * pr] * kActScale), relu_i(acc[t][2 * pr + 1] * kActScale), hh, ll);
            ch[2 * t + (pr >> 2)][pr & 3] = hh;
            cl[2 * t + (pr >> 2)][pr & 3] = ll;
          }
      }
    }
  }
  nerf::wait_vmcnt(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int u = 0; u < 16; ++u) s += __builtin_bit_cast(float, iH[u][0]) + __builtin_bit_cast(float, iL[u][3]);
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

// ---- candidate: 8 waves (2 per SIMD), 16 samples per wave, v_mfma_f32_16x16x32_f16 --
// A unit = one 32-wide k-step of an "eighth" (two 16-row output tiles): A_hi t0, t1,
// A_lo t0, t1 (1 KiB each).  A layer = 8 eighths x 8 k-steps = 64 units, as the shipped one.
template <int kPf>
__global__ __launch_bounds__(512, 1) void x3_16(const char* __restrict__ blob, float* out, unsigned long long* clk,
                                                int tiles) {
  __shared__ __attribute__((aligned(16))) char lds[kSlots * kChunkB];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned rb = nerf::lds_addr(lds) + lane * 16;
  stage<8>(blob, 0, lds, wave, lane);
  u32x4 iH[8], iL[8], oH[8], oL[8];
  for (int u = 0; u < 8; ++u) {
    iH[u] = ((const u32x4*)blob)[(u * 64 + lane + blockIdx.x) & 4095];
    iL[u] = ((const u32x4*)blob)[(u * 64 + lane + 7 * blockIdx.x + 1024) & 4095] & 0x03FF03FFu;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int tile = 0; tile < tiles; ++tile) {
    nerf::wait_vmcnt(0);
    __syncthreads();
    const char* bl0 = blob;
    asm volatile("" : "+s"(bl0));
    stage<8>(bl0, 1, lds, wave, lane);
    f16x8 ra[kPf + 1][4];
#pragma unroll
    for (int m = 0; m < kPf; ++m)
#pragma unroll
      for (int f = 0; f < 4; ++f)
        ra[m][f] = nerf::ds_read_b128<f16x8>(rb, int(((m / 4) % kSlots) * kChunkB + (m % 4) * kUnitB + f * 1024));
#pragma unroll
    for (int l = 0; l < kLayers; l += 2) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        u32x4(&bh)[8] = half ? oH : iH;
        u32x4(&bl)[8] = half ? oL : iL;
        u32x4(&ch)[8] = half ? iH : oH;
        u32x4(&cl)[8] = half ? iL : oL;
        f32x4 acc[16];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int n = e * 8 + u;
            const int lu = (l + half) * 64 + n;
            if ((lu + kPf) % 4 == 0 && lu + kPf < kUnitsPerTile)
              seam<8>(bl0, (lu + kPf) / 4 + 1, lds, wave, lane);
            if (u == 0) acc[2 * e] = acc[2 * e + 1] = f32x4{};
            const int m = lu + kPf;
            if (m < kUnitsPerTile) {
#pragma unroll
              for (int f = 0; f < 4; ++f)
                ra[m % (kPf + 1)][f] = nerf::ds_read_b128<f16x8>(
                    rb, int(((m / 4) % kSlots) * kChunkB + (m % 4) * kUnitB + f * 1024));
            }
            nerf::wait_lgkm(0);
            const f16x8 h = __builtin_bit_cast(f16x8, bh[u]), lo = __builtin_bit_cast(f16x8, bl[u]);
#pragma unroll
            for (int o = 0; o < 2; ++o) {
              f32x4 a = acc[2 * e + o];
              a = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[lu % (kPf + 1)][o], h, a, 0, 0, 0);
              a = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[lu % (kPf + 1)][o], lo, a, 0, 0, 0);
              acc[2 * e + o] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[lu % (kPf + 1)][2 + o], h, a, 0, 0, 0);
            }
            // the previous eighth's two tiles (8 values per lane) -> next k-step e-1, over 4 units
            if (e >= 1 && u < 4) {
              const int t = 2 * (e - 1) + (u >> 1), p = (u & 1) * 2;
              unsigned h0, l0;
              split_pair(relu_i(acc[t][p] * kActScale), relu_i(acc[t][p + 1] * kActScale), h0, l0);
              ch[e - 1][(u >> 1) * 2 + (p >> 1)] = h0;
              cl[e - 1][(u >> 1) * 2 + (p >> 1)] = l0;
            }
          }
        }
#pragma unroll
        for (int t = 14; t < 16; ++t)
#pragma unroll
          for (int p = 0; p < 4; p += 2) {
            unsigned hh, ll;
            split_pair(relu_i(acc[t][p] * kActScale), relu_i(acc[t][p + 1] * kActScale), hh, ll);
            ch[7][(t - 14) * 2 + (p >> 1)] = hh;
            cl[7][(t - 14) * 2 + (p >> 1)] = ll;
          }
      }
    }
  }
  nerf::wait_vmcnt(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int u = 0; u < 8; ++u) s += __builtin_bit_cast(float, iH[u][0]) + __builtin_bit_cast(float, iL[u][3]);
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

int main(int argc, char** argv) {
  const int tiles = argc > 1 ? atoi(argv[1]) : 24;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t blob_bytes = size_t(kBlobChunks) * kChunkB;
  std::vector<unsigned short> h(blob_bytes / 2);
  srand(1);
  for (auto& v : h) {   // random fp16 in about [-0.25, 0.25], like trained weights
    const float f = ((rand() / (float)RAND_MAX) * 2.f - 1.f) * 0.25f;
    const _Float16 x = (_Float16)f;
    v = __builtin_bit_cast(unsigned short, x);
  }
  char* blob;
  float* out;
  unsigned long long* clk;
  CK(hipMalloc(&blob, blob_bytes));
  CK(hipMalloc(&out, size_t(cus) * 512 * 4));
  CK(hipMalloc(&clk, size_t(cus) * 16));
  CK(hipMemcpy(blob, h.data(), blob_bytes, hipMemcpyHostToDevice));
  // MFMA FLOP: three MFMAs per product of a 256 x 256 layer on 128 samples, per tile and CU
  const double flop = double(cus) * tiles * kLayers * 3.0 * 2.0 * 256 * 256 * 128;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<unsigned long long> hc(size_t(cus) * 2);
  const char* names[3] = {"32x32x16 f16, 4 waves (1/SIMD), 32 samples/wave, prefetch 3",
                          "16x16x32 f16, 8 waves (2/SIMD), 16 samples/wave, prefetch 1",
                          "16x16x32 f16, 8 waves (2/SIMD), 16 samples/wave, prefetch 2"};
  auto launch = [&](int v) {
    if (v == 0) hipLaunchKernelGGL(x3_32, dim3(cus), dim3(256), 0, 0, blob, out, clk, tiles);
    else if (v == 1) hipLaunchKernelGGL(x3_16<1>, dim3(cus), dim3(512), 0, 0, blob, out, clk, tiles);
    else hipLaunchKernelGGL(x3_16<2>, dim3(cus), dim3(512), 0, 0, blob, out, clk, tiles);
  };
  // Power-limited regime (MI355X_MICROARCH.md 'DVFS give-back' item 6): each variant runs
  // back to back for warm_s seconds before its timed second, so the clock it reports is
  // the one the chip holds under that load, not the boost a short burst sees.
  const double warm_s = argc > 2 ? atof(argv[2]) : 3.0;
  for (int round = 0; round < 2; ++round)
    for (int v = 0; v < 2; ++v) {   // (prefetch 2 uses scratch for its fragment ring in this build)
      CK(hipEventRecord(e0));
      launch(v);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float one = 0;
      CK(hipEventElapsedTime(&one, e0, e1));
      const int n_warm = int(warm_s * 1e3 / one) + 1, n_time = int(1e3 / one) + 1;
      for (int w = 0; w < n_warm; ++w) launch(v);
      CK(hipEventRecord(e0));
      for (int w = 0; w < n_time; ++w) launch(v);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipGetLastError());
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipMemcpy(hc.data(), clk, size_t(cus) * 16, hipMemcpyDeviceToHost));
      double ghz = 0;
      for (int i = 0; i < cus; ++i) ghz += double(hc[2 * i]) / double(hc[2 * i + 1]) * 0.1;
      const double tf = flop / (ms / n_time * 1e-3) / 1e12;
      printf("round %d %-62s %.3f ms/launch  %.1f TFLOP/s MFMA-rate (%.3f of 2.5 PF, %.3f of 833 algorithmic)  clock %.3f GHz  (%d warm + %d timed)\n",
             round, names[v], ms / n_time, tf, tf / 2500.0, tf / 3.0 / 833.3, ghz / cus, n_warm, n_time);
      fflush(stdout);
    }
  return 0;
}
