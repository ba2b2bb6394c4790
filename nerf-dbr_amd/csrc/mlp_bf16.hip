// bf16 NeRF MLP on gfx950 (v_mfma_f32_32x32x16_bf16, fp32 accumulate): the
// throughput path.
//
// Replaces NeRFModel.forward (src/models/nerf.py:92-131) fused with
// sample_points_on_rays (src/benchmark/base_renderer.py:260-281) and the
// positional encoding (nerf.py:24-45).  Activations and weights are rounded to
// bf16 (RNE) at MFMA inputs; accumulation, bias, ReLU, the density/colour heads
// and everything outside the MLP stay fp32.
//
// Geometry: 256-thread workgroups (4 waves, one per SIMD) of 256 samples; a
// wave owns two 32-sample column tiles, so every A (weight) fragment it reads
// feeds two MFMAs.  A lane keeps one layer's 2x8 accumulator tiles (256 fp32)
// and the previous layer as packed bf16 B fragments (128 VGPRs): activations
// never leave registers (nerf_layout.h).  The position encoding waits in LDS
// for layers 0 and 4.
//
// Weight stream: the packed 1.04 MB blob is cut into 16 KiB chunks (2 k-steps
// of a 256-wide layer).  A 4-slot LDS ring is filled by global_load_lds_dwordx4
// (lane-linear 1 KiB pieces) three chunks ahead; one raw s_barrier per chunk
// publishes the chunk two ahead (counted vmcnt, never 0 in the loop), and the
// first k-step's fragments of the next chunk are read before that barrier, so
// ds_read latency never stalls the MFMA pipe at a chunk seam.  Per chunk a SIMD
// runs 32 MFMAs (1024 cycles) against 16 KiB of L2->LDS traffic per CU.
#include "nerf_device.h"
#include "nerf_internal.h"

namespace nerf {
namespace {

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kCols = 2;                                   // column tiles per wave
constexpr int kSamplesPerBlock = kWaves * kCols * kSamplesPerWave;   // 256
constexpr int kTotalChunks = bf16_blob_chunks();
constexpr int kSlots = 4, kAhead = 3;                      // ring slots, load lookahead (chunks)
constexpr int kGldsPerStage = kChunkBytes / (kThreads * 16);   // 4 per wave
constexpr int kLdsParamOff = kSlots * kChunkBytes;
constexpr int kLdsPeOff = kLdsParamOff + ((kParamFloats * 4 + 1023) / 1024) * 1024;
constexpr int kLdsDeOff = kLdsPeOff + kWaves * kCols * 4 * 1024;
constexpr int kLdsBytes = kLdsDeOff + kWaves * kCols * 2 * 1024;
static_assert(kLdsParamOff % 16 == 0 && kLdsPeOff % 16 == 0, "LDS carve must stay 16-B aligned");
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
static_assert(kGldsPerStage * kThreads * 16 == kChunkBytes, "stage geometry");

template <int L>
constexpr int bf16_chunk0() {
  int c = 0;
  for (int l = 0; l < L; ++l) c += bf16_layer_chunks(l);
  return c;
}

typedef __attribute__((address_space(3))) void lds_void;

// Chunk g -> ring slot g % kSlots.  Each wave moves 4 KiB as four lane-linear
// 1 KiB LDS-DMA pieces (destination = wave-uniform base + lane*16).
__device__ __forceinline__ void stage_chunk(const char* __restrict__ blob, int g, char* lds, int wave_u, int lane) {
  const char* src = blob + size_t(g) * kChunkBytes + wave_u * 1024 + lane * 16;
  char* dst = lds + (g % kSlots) * kChunkBytes + wave_u * 1024;
#pragma unroll
  for (int i = 0; i < kGldsPerStage; ++i)
    __builtin_amdgcn_global_load_lds((const void*)(src + i * kThreads * 16), (lds_void*)(dst + i * kThreads * 16),
                                     16, 0, 0);
}

__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ bf16x8 pack8(const float* v) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
  return r;
}

// ReLU'd accumulators -> next layer's B fragments (register 8s..8s+7 of tile t
// is k-step 2t+s; nerf_layout.h hid_bf16_feature).
__device__ __forceinline__ void to_fragments(const f32x16 (&acc)[kCols][8], bf16x8 (&bh)[kCols][16]) {
#pragma unroll
  for (int c = 0; c < kCols; ++c)
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = relu(acc[c][t][8 * s + j]);
        bh[c][2 * t + s] = pack8(v);
      }
}

// The k-step fragments of one chunk-slot: NT tiles x 1 KiB, this lane's 16 B each.
// (nt is a constant after unrolling)
__device__ __forceinline__ void read_frags(bf16x8 (&a)[8], const char* slot_lane, int uu, int nt) {
#pragma unroll
  for (int o = 0; o < 8; ++o)
    if (o < nt) a[o] = *(const bf16x8*)(slot_lane + (uu * nt + o) * 1024);
}

struct Ctx {
  const char* blob;
  char* lds;
  int wave_u, lane, h;
};

// End of chunk g: publish chunk g+2, prefetch the first k-step of chunk g+1.
__device__ __forceinline__ void chunk_seam(const Ctx& cx, int g, bf16x8 (&a)[8], int nt_next) {
  // stage(g+2) must have landed; stage(g+3) (issued at the start of g) may fly.
  if (g + kAhead < kTotalChunks) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kGldsPerStage) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");      // this wave's reads of slot g are done
  if (g + 1 < kTotalChunks) read_frags(a, cx.lds + ((g + 1) % kSlots) * kChunkBytes + cx.lane * 16, 0, nt_next);
  compiler_fence();
  __builtin_amdgcn_s_barrier();
  compiler_fence();
}

// Extra (non-hidden) inputs live in LDS: 4 position-encoding k-steps per
// column tile at kLdsPeOff, 2 direction-encoding k-steps at kLdsDeOff.
template <int L, int NT, int NT_NEXT>
__device__ __forceinline__ void layer_bf16(f32x16 (&acc)[kCols][8], const bf16x8 (&bh)[kCols][16],
                                           bf16x8 (&a)[8], const Ctx& cx) {
  constexpr LayerShape sh = layer_shape(L);
  constexpr int KH = sh.hidden / 16;
  constexpr int KU = ksteps_bf16(L);
  constexpr int UPC = kChunkBytes / (NT * 1024);     // k-steps per chunk
  constexpr int NCH = bf16_layer_chunks(L);
  constexpr int G0 = bf16_chunk0<L>();
  const float* prm = (const float*)(cx.lds + kLdsParamOff);
#pragma unroll
  for (int c = 0; c < kCols; ++c) load_bias<NT>(acc[c], prm, L, cx.h);
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int g = G0 + ch;
    if (g + kAhead < kTotalChunks) stage_chunk(cx.blob, g + kAhead, cx.lds, cx.wave_u, cx.lane);
    const char* slot_lane = cx.lds + (g % kSlots) * kChunkBytes + cx.lane * 16;
#pragma unroll
    for (int uu = 0; uu < UPC; ++uu) {
      const int u = ch * UPC + uu;
      if (u < KU) {
        bf16x8 an[8];
        if (uu + 1 < UPC && u + 1 < KU) read_frags(an, slot_lane, uu + 1, NT);
        bf16x8 b[kCols];
#pragma unroll
        for (int c = 0; c < kCols; ++c) {
          if (u < KH) {
            b[c] = bh[c][u < KH ? u : 0];
          } else if (sh.extra == kPos) {
            b[c] = *(const bf16x8*)(cx.lds + kLdsPeOff + ((cx.wave_u * kCols + c) * 4 + (u - KH)) * 1024 +
                                    cx.lane * 16);
          } else {
            b[c] = *(const bf16x8*)(cx.lds + kLdsDeOff + ((cx.wave_u * kCols + c) * 2 + (u - KH)) * 1024 +
                                    cx.lane * 16);
          }
        }
#pragma unroll
        for (int o = 0; o < NT; ++o)
#pragma unroll
          for (int c = 0; c < kCols; ++c)
            acc[c][o] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[o], b[c], acc[c][o], 0, 0, 0);
        if (uu + 1 < UPC && u + 1 < KU) {
#pragma unroll
          for (int o = 0; o < NT; ++o) a[o] = an[o];
        }
      }
    }
    chunk_seam(cx, g, a, ch + 1 < NCH ? NT : NT_NEXT);
  }
}

template <bool kExplicit>
__global__ __launch_bounds__(kThreads, 1) void mlp_bf16_kernel(const char* __restrict__ blob,
                                                               const float* __restrict__ prm_g, SampleSrc src,
                                                               long n_points, f32x4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  const int lane = threadIdx.x & 63;
  const int wave_u = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5;
  const Ctx cx{blob, lds, wave_u, lane, h};
  const long p0 = (long(blockIdx.x) * kWaves + wave_u) * (kCols * kSamplesPerWave) + (lane & 31);

  // Kick off the weight stream, then do the per-sample prologue under it.
#pragma unroll
  for (int g = 0; g < kAhead; ++g) stage_chunk(blob, g, lds, wave_u, lane);
  for (int i = threadIdx.x; i < kParamFloats / 4; i += kThreads)
    ((f32x4*)(lds + kLdsParamOff))[i] = ((const f32x4*)prm_g)[i];

#pragma unroll 1
  for (int c = 0; c < kCols; ++c) {
    const long p = p0 + c * kSamplesPerWave;
    float x[3], d[3], pef[32], def[16];
    fetch_sample<kExplicit>(src, p < n_points ? p : n_points - 1, x, d);
    pos_encode(x[0], x[1], x[2], h, pef);
    dir_encode(d[0], d[1], d[2], h, def);
    char* pe_dst = lds + kLdsPeOff + (wave_u * kCols + c) * 4096 + lane * 16;
    char* de_dst = lds + kLdsDeOff + (wave_u * kCols + c) * 2048 + lane * 16;
#pragma unroll
    for (int u = 0; u < 4; ++u) *(bf16x8*)(pe_dst + u * 1024) = pack8(pef + 8 * u);
    *(bf16x8*)(de_dst) = pack8(def);
    *(bf16x8*)(de_dst + 1024) = pack8(def + 8);
  }
  // chunks 0 and 1 published; first fragments of chunk 0 in registers
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kGldsPerStage) : "memory");
  __syncthreads();
  bf16x8 a[8];
  read_frags(a, lds + lane * 16, 0, 8);

  f32x16 acc[kCols][8];
  bf16x8 bh[kCols][16];
  layer_bf16<L0, 8, 8>(acc, bh, a, cx);
  to_fragments(acc, bh);
  layer_bf16<L1, 8, 8>(acc, bh, a, cx);
  to_fragments(acc, bh);
  layer_bf16<L2, 8, 8>(acc, bh, a, cx);
  to_fragments(acc, bh);
  layer_bf16<L3, 8, 8>(acc, bh, a, cx);
  to_fragments(acc, bh);
  layer_bf16<L4, 8, 8>(acc, bh, a, cx);   // skip: [x, pe] (nerf.py:109-110)
  to_fragments(acc, bh);
  layer_bf16<L5, 8, 8>(acc, bh, a, cx);
  to_fragments(acc, bh);
  layer_bf16<L6, 8, 8>(acc, bh, a, cx);
  to_fragments(acc, bh);
  layer_bf16<L7, 8, 4>(acc, bh, a, cx);
  const float* prm = (const float*)(lds + kLdsParamOff);
  float sigma[kCols];
#pragma unroll
  for (int c = 0; c < kCols; ++c) {
    relu_tiles<8>(acc[c]);
    sigma[c] = density_head(acc[c], prm, h);
  }
  to_fragments(acc, bh);
  layer_bf16<C0, 4, 4>(acc, bh, a, cx);   // [x, PE4(d)] (nerf.py:117-121)
#pragma unroll
  for (int c = 0; c < kCols; ++c) {
    relu_tiles<4>(acc[c]);
    float rgb[3];
    color_head(acc[c], prm, h, rgb);
    const long p = p0 + c * kSamplesPerWave;
    if (p < n_points && h == 0) out[p] = f32x4{sigma[c], rgb[0], rgb[1], rgb[2]};
  }
}

}  // namespace

hipError_t launch_mlp_bf16(const void* blob, const float* params, const SampleSrc& src, long n_points, float* out,
                           bool explicit_points, hipStream_t stream) {
  if (n_points <= 0) return hipSuccess;
  const long blocks = (n_points + kSamplesPerBlock - 1) / kSamplesPerBlock;
  if (blocks > 0x7FFFFFFFL) return hipErrorInvalidValue;
  const dim3 grid{unsigned(blocks), 1, 1}, block{kThreads, 1, 1};
  if (explicit_points)
    hipLaunchKernelGGL(mlp_bf16_kernel<true>, grid, block, 0, stream, (const char*)blob, params, src, n_points,
                       (f32x4*)out);
  else
    hipLaunchKernelGGL(mlp_bf16_kernel<false>, grid, block, 0, stream, (const char*)blob, params, src, n_points,
                       (f32x4*)out);
  return hipGetLastError();
}

}  // namespace nerf
