// NeRFTrainer.train_step on gfx950, fp32 throughout.
//
// Replaces src/training/trainer.py:83-138 (train_step) with _get_rays (:271-292),
// _render_rays (:294-316), _query_network (:318-351), VolumeRenderer's stratified
// sampling and volume_render (src/utils/rendering.py:17-52, 102-143), autograd,
// clip_grad_norm_, optim.Adam and ExponentialLR.
//
// Structure of one step (both nets, one stream, no host synchronisation):
//   rays of the selected pixels -> per net: samples + encodings (rows for the weight
//   gradients) -> the whole forward in ONE register-stationary launch (mlp_f32.hip's
//   shape: activations stay in registers from layer to layer; each layer's rows and ReLU
//   bits are written for the backward) -> volume render forward + MSE + its backward per
//   ray -> head backward -> the whole backward-data chain in ONE launch of the same shape
//   run backwards (dZ of every layer written) -> weight gradients as split-K GEMM partials
//   over the samples -> one reduction into the flat gradients -> grad norm, clip, Adam,
//   and the relayout of the updated weights into the two kernels' fragment blobs.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "nerf_asm.h"
#include "nerf_device.h"
#include "nerf_internal.h"
#include "train_x3_layout.h"

namespace nerf {
namespace {

#define HIP_TRY(expr)                                                                                 \
  do {                                                                                                \
    hipError_t e_ = (expr);                                                                           \
    if (e_ != hipSuccess) return set_error(NERF_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                           __FILE__, __LINE__);                                      \
  } while (0)

// ---------------------------------------------------------------- layouts --
// Flat parameters of one NeRFModel in state-dict order (src/models/nerf.py:72-90):
// layers.0..7 (weight [256][in], bias [256]), density_head ([1][256], [1]),
// color_layers.0 ([128][283], [128]), color_layers.1 ([3][128], [3]).
constexpr int kTrunkIn[8] = {63, 256, 256, 256, 319, 256, 256, 256};
constexpr int kH = 256, kC0 = 128, kDirDim = 27;

struct TensorDesc {
  long off;
  int rows, cols;
};

constexpr TensorDesc tensor_desc(int i) {
  long off = 0;
  for (int j = 0; j <= i; ++j) {
    int rows = 0, cols = 1;
    if (j < 16) {
      rows = kH;
      cols = (j % 2 == 0) ? kTrunkIn[j / 2] : 1;
    } else if (j == 16) {
      rows = 1, cols = kH;
    } else if (j == 17) {
      rows = 1;
    } else if (j == 18) {
      rows = kC0, cols = kH + kDirDim;
    } else if (j == 19) {
      rows = kC0;
    } else if (j == 20) {
      rows = 3, cols = kC0;
    } else {
      rows = 3;
    }
    if (j == i) return TensorDesc{off, rows, cols};
    off += long(rows) * cols;
  }
  return TensorDesc{0, 0, 0};
}
constexpr long kNetFloats = tensor_desc(21).off + 3;   // 530,052
static_assert(kNetFloats == 530052, "NeRFModel parameter count");
constexpr long w_off(int l) { return tensor_desc(2 * l).off; }
constexpr long b_off(int l) { return tensor_desc(2 * l + 1).off; }
constexpr long kFDensW = tensor_desc(16).off, kFDensB = tensor_desc(17).off;
constexpr long kFC0W = tensor_desc(18).off, kFC0B = tensor_desc(19).off;
constexpr long kFC1W = tensor_desc(20).off, kFC1B = tensor_desc(21).off;

constexpr int round_up(int x, int m) { return (x + m - 1) / m * m; }

// Operand copies of one net's weights, rewritten after every update (relayout_kernel):
//   F32   the f32 MFMA blob of mlp_f32.hip (nerf_layout.h: per layer [u/4][tile][lane][4]),
//         read by the fused forward kernel
//   PRM   the params blob (biases in accumulator order, density and colour-1 rows)
constexpr int kHeadLd = 132, kHeadK = kH + kDirDim;   // head rows [P][132]; colour-0 inputs 283
constexpr long kF32Blob = 0;
constexpr long kPrmBlob = kF32Blob + round_up(f32_blob_floats(), 64);
//   BWD   the transposed weights for the fused backward-data chain (train_bwd_kernel), in
//         the forward blob's fragment order: per backward layer b (0 the head, then layers
//         7..1) [u/4][tile][lane][4], A[row = input feature][k-step u, half h] =
//         W[output feature hid_f32_feature(u, h)][input]; the head's k runs over the 128
//         colour-0 rows, then one k-step for the density row (half 0), zero-padded to 68
constexpr int kBwdLayers = 8;
constexpr int kHeadBwdKsteps = 68;
constexpr int bwd_ksteps(int b) { return b == 0 ? kHeadBwdKsteps : kH / 2; }
constexpr int bwd_layer_floats(int b) { return bwd_ksteps(b) * 8 * 64; }
constexpr long bwd_layer_offset(int b) {
  long o = 0;
  for (int i = 0; i < b; ++i) o += bwd_layer_floats(i);
  return o;
}
constexpr int bwd_trunk_layer(int b) { return 8 - b; }   // b = 1..7 -> layers 7..1
constexpr long kBwdBlob = kPrmBlob + round_up(kParamFloats, 64);
constexpr long kGemmFloats = kBwdBlob + round_up(int(bwd_layer_offset(kBwdLayers)), 64);

// Per-sample activation workspace (floats per sample; each array [P][ld])
constexpr int kPeLd = 64, kDpeLd = 28;

// weight-gradient k tiles: 16 sample rows (one LDS-DMA buffer of 26-37 KiB, four in flight)
#ifndef NERF_WG_BK
#define NERF_WG_BK 16
#endif
constexpr int BK = NERF_WG_BK;
#ifndef NERF_WG_BUFS
#define NERF_WG_BUFS 4
#endif
constexpr int kWBufs = BK == 16 ? NERF_WG_BUFS : 2;   // LDS-DMA buffers in flight (LDS budget)
#ifndef NERF_WGRAD_X3
#define NERF_WGRAD_X3 1
#endif
constexpr bool kWgradX3 = NERF_WGRAD_X3;   // split-bf16 weight gradients (wgrad_tile_x3); 0: fp32 MFMA
// precision NERF_BF16X3 also runs the backward-data chain on the split-bf16 MFMA
// (train_bwd_x3.hip); 0: the fp32 chain (train_bwd_kernel) under both precisions
#ifndef NERF_TRAIN_BWD_X3
#define NERF_TRAIN_BWD_X3 1
#endif

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// ------------------------------------------------------- weight gradients --
// Partial weight gradients dW[m][n] = sum_k dZ[k][m] X[k][n] over one split of the samples
// (k), on the split-bf16 MFMA (wgrad_tile_x3; NERF_WGRAD_X3=0: v_mfma_f32_32x32x2_f32,
// wgrad_tile).  One workgroup tile covers the whole [M][N] gradient
// (256 x 256 over 8 waves of 64 x 128 for the 256-wide layers; wgrad_shape), so both
// operands are read once.  k tiles of BK sample rows move HBM -> LDS by LDS-DMA
// (global_load_lds_dwordx4: 1 KiB per wave instruction, no registers, no VALU), kWBufs
// buffers deep and issued kWBufs - 1 tiles ahead: each wave waits for its own pieces with a
// counted vmcnt, and one barrier per k tile publishes the tile and frees the buffer of the
// tile before.  The first column tile's waves also sum dZ over k for their rows (the bias
// gradient).
struct Src2 {                // columns [0, w1) from p1, [w1, ...) from p2 (w1 % 4 == 0)
  const float* p1 = nullptr;
  const float* p2 = nullptr;
  int ld1 = 0, ld2 = 0, w1 = 0x7fffffff;
};

struct GemmArgs {
  int M = 0, N = 0, K = 0;
  Src2 a, b;                        // A: dZ rows (a.p1, [K][a.ld1]); B: X rows, two sources
  float* c = nullptr;               // [split][M][ldc]
  int ldc = 0;
  float* bias_part = nullptr;       // [split][M] sums of A over the split's k
  int k_split = 0;                  // k range per blockIdx.z (multiple of BK)
  long c_split = 0;                 // floats per split partial
};

__device__ __forceinline__ f32x4 ld4(const float* p) { return *(const f32x4*)p; }

// Geometry of a k tile and of the workgroup tile.  LDS image of a k tile, each part
// row-contiguous as in HBM: A [BK][BMT] (dZ rows), B1 [BK][W1] (the first source's
// columns), B2 [BK][W2] (the second source's, e.g. layer 4's position encodings).  Every
// wave issues the same number of DMA instructions per k tile (the list wraps around:
// a repeated instruction writes the same bytes again), so one vmcnt count fits all.
template <int BMT, int W1, int W2, int WAVES>
struct WGeo {
  static constexpr int kThreads = 64 * WAVES;
  static constexpr int kWM = BMT / 64, kWN = WAVES / kWM;
  // 32-column MFMA tiles of a wave (column group wn): kTN1 of B1 (columns 32 (kTN1 wn + j)),
  // then B2's tiles b = wn, wn + kWN, ... (columns W1 + 32 b), so every tile lies in one
  // part and its LDS rows have a constant stride
  static constexpr int kTN1 = W1 / 32 / kWN, kTN2All = (W2 + 31) / 32;
  static constexpr int kTN2 = (kTN2All + kWN - 1) / kWN;
  static constexpr int kTN = kTN1 + kTN2;
  static constexpr int kR16A = BMT / 4, kR16B1 = W1 / 4, kR16B2 = W2 / 4;   // 16-B pieces per row
  static constexpr int kInsA = BK * kR16A / 64, kInsB1 = BK * kR16B1 / 64, kInsB2 = (BK * kR16B2 + 63) / 64;
  static constexpr int kIns = kInsA + kInsB1 + kInsB2;
  static constexpr int kInsPerWave = (kIns + WAVES - 1) / WAVES;
  static constexpr int kOffB1 = BK * BMT * 4, kOffB2 = kOffB1 + BK * W1 * 4;
  static constexpr int kBufBytes = round_up(kOffB2 + BK * W2 * 4 + 128, 1024);   // B2's last tile reads past W2
  static constexpr int kBufs = kWBufs;
  static_assert(kBufs >= 2 && kBufs <= 4, "pipeline depth");
  static_assert(kWM * kWN == WAVES && kTN1 * 32 * kWN == W1, "tile geometry");
  static_assert(BK * kR16A % 64 == 0 && BK * kR16B1 % 64 == 0, "whole DMA instructions");
  static_assert(kBufs * kBufBytes <= 160 * 1024, "LDS budget");
};

// The DMA instructions of this wave for the k tile at k0 into the buffer at LDS byte
// address buf.  Rows past K re-read row K-1 (in bounds; A's are zeroed before use).
template <int R16>
__device__ __forceinline__ unsigned piece_off(int q, int lim, int ld) {   // R16 constant: no division
  return unsigned(min(q / R16, lim) * ld * 4 + (q % R16) * 16);
}
template <class G>
__device__ __forceinline__ void issue_ktile(const GemmArgs& g, int k0, int K, unsigned buf, int wave, int lane) {
  const int lim = K - 1 - k0;
#pragma unroll
  for (int s = 0; s < G::kInsPerWave; ++s) {
    const int ins = (s * (G::kThreads / 64) + wave) % G::kIns;   // wave-uniform
    if (ins < G::kInsA) {
      const int q = 64 * ins + lane;
      lds_dma_16_s(g.a.p1 + long(k0) * g.a.ld1, piece_off<G::kR16A>(q, lim, g.a.ld1), buf + unsigned(ins * 1024));
    } else if (ins < G::kInsA + G::kInsB1) {
      const int ii = ins - G::kInsA, q = 64 * ii + lane;
      lds_dma_16_s(g.b.p1 + long(k0) * g.b.ld1, piece_off<G::kR16B1>(q, lim, g.b.ld1),
                   buf + unsigned(G::kOffB1 + ii * 1024));
    } else if (G::kInsB2 > 0) {
      const int ii = ins - G::kInsA - G::kInsB1, q = 64 * ii + lane;
      if (q < BK * G::kR16B2)   // B2's last instruction may be partial
        lds_dma_16_s(g.b.p2 + long(k0) * g.b.ld2, piece_off<(G::kR16B2 > 0 ? G::kR16B2 : 1)>(q, lim, g.b.ld2),
                     buf + unsigned(G::kOffB2 + ii * 1024));
    }
  }
}

// Output column of the wave's column tile j (>= W1 + W2 when the wave has no such tile).
template <class G, int W1>
__device__ __forceinline__ int wtile_col(int wn, int j) {
  return j < G::kTN1 ? 32 * (G::kTN1 * wn + j) : W1 + 32 * (wn + G::kWN * (j - G::kTN1));
}

// One k tile from LDS into the wave's 64 x (32 TN) accumulator block; waves of the first
// column group also add their row's BK dZ values to the bias sum.
template <class G, int BMT, int W1, int W2>
__device__ __forceinline__ void wgrad_tile(const float* __restrict__ buf, f32x16 (&acc)[2][G::kTN], float& bsum,
                                           int wm, int wn, int h, int l32, int t) {
  const float* as = buf + wm * 64 + l32;
  const float* b1 = buf + G::kOffB1 / 4 + 32 * G::kTN1 * wn + l32;
  const float* b2 = buf + G::kOffB2 / 4 + 32 * wn + l32;
#pragma unroll
  for (int kk = 0; kk < BK / 2; ++kk) {
    const int k = 2 * kk + h;
    const float a0 = as[k * BMT], a1 = as[k * BMT + 32];
    float b[G::kTN];
#pragma unroll
    for (int j = 0; j < G::kTN; ++j)
      b[j] = j < G::kTN1 ? b1[k * W1 + 32 * j] : b2[k * W2 + 32 * G::kWN * (j - G::kTN1)];
#pragma unroll
    for (int j = 0; j < G::kTN; ++j) {
      if (j >= G::kTN1 && wtile_col<G, W1>(wn, j) >= W1 + W2) continue;   // wave-uniform: no such tile
      acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b[j], acc[0][j], 0, 0, 0);
      acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b[j], acc[1][j], 0, 0, 0);
    }
  }
  if (t < BMT) {
#pragma unroll
    for (int kr = 0; kr < BK; ++kr) bsum = __fadd_rn(bsum, buf[kr * BMT + t]);
  }
}

// The same k tile on the bf16 MFMA (v_mfma_f32_32x32x16_bf16, one MFMA per 16 sample rows):
// each fp32 operand v is split into v_hi = bf16(v) and v_lo = bf16(v - v_hi) as it is read
// from LDS, and each product is A_hi.B_hi + A_hi.B_lo + A_lo.B_hi (mlp_bf16x3.hip's scheme;
// the dropped A_lo.B_lo is ~2^-16 relative), accumulated in fp32.  Per product the error is
// ~2^-17 relative; over a gradient's k ~ 1e5 samples it stays below the fp32 summation-order
// differences already present (those grow as sqrt(k), this does not).  Lane l holds rows
// k = 8 (l / 32) + q, q < 8, of its A row / B column, so BK = 16 is one MFMA k step.
typedef __bf16 wg_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void wg_split8(const float (&v)[8], u32x4_t& hi, u32x4_t& lo) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const float a = v[2 * d], b = v[2 * d + 1];
    const unsigned h2 = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{a, b}, wg_bf16x2));
    const float ha = __builtin_bit_cast(float, h2 << 16), hb = __builtin_bit_cast(float, h2 & 0xFFFF0000u);
    hi[d] = h2;
    lo[d] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{__fsub_rn(a, ha), __fsub_rn(b, hb)}, wg_bf16x2));
  }
}
template <class G, int BMT, int W1, int W2>
__device__ __forceinline__ void wgrad_tile_x3(const float* __restrict__ buf, f32x16 (&acc)[2][G::kTN], float& bsum,
                                              int wm, int wn, int h, int l32, int t) {
  static_assert(BK == 16, "one bf16 MFMA k step per k tile");
  const float* as = buf + 8 * h * BMT + wm * 64 + l32;
  const float* b1 = buf + G::kOffB1 / 4 + 8 * h * W1 + 32 * G::kTN1 * wn + l32;
  const float* b2 = buf + G::kOffB2 / 4 + 8 * h * W2 + 32 * wn + l32;
  u32x4_t ahi[2], alo[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = as[q * BMT + 32 * i];
    wg_split8(v, ahi[i], alo[i]);
  }
#pragma unroll
  for (int j = 0; j < G::kTN; ++j) {
    if (j >= G::kTN1 && wtile_col<G, W1>(wn, j) >= W1 + W2) continue;   // wave-uniform: no such tile
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = j < G::kTN1 ? b1[q * W1 + 32 * j] : b2[q * W2 + 32 * G::kWN * (j - G::kTN1)];
    u32x4_t bhi, blo;
    wg_split8(v, bhi, blo);
    const bf16x8 bh = __builtin_bit_cast(bf16x8, bhi), bl = __builtin_bit_cast(bf16x8, blo);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16x8 ah = __builtin_bit_cast(bf16x8, ahi[i]), al = __builtin_bit_cast(bf16x8, alo[i]);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[i][j], 0, 0, 0);
    }
  }
  if (t < BMT) {
#pragma unroll
    for (int kr = 0; kr < BK; ++kr) bsum = __fadd_rn(bsum, buf[kr * BMT + t]);
  }
}

// One split (k range) of one job: the workgroup's whole M x N partial.
// An opaque SGPR copy: the job's arguments come from a dynamically indexed kernel-argument
// table, and without this the compiler re-loads them per use inside the k loop (each
// reload's lgkmcnt(0) also waits for every LDS read in flight).
template <typename T>
__device__ __forceinline__ T pin_sgpr(T v) {
  asm volatile("" : "+s"(v));
  return v;
}

template <int BMT, int W1, int W2, int WAVES>
__device__ __forceinline__ void wgrad_split(GemmArgs g, int split, float* lds) {
  using G = WGeo<BMT, W1, W2, WAVES>;
  g.a.p1 = pin_sgpr(g.a.p1), g.b.p1 = pin_sgpr(g.b.p1), g.b.p2 = pin_sgpr(g.b.p2);
  g.a.ld1 = pin_sgpr(g.a.ld1), g.b.ld1 = pin_sgpr(g.b.ld1), g.b.ld2 = pin_sgpr(g.b.ld2);
  g.K = pin_sgpr(g.K), g.k_split = pin_sgpr(g.k_split);
  const int t = threadIdx.x;
  const int lane = t & 63, h = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w % G::kWM, wn = w / G::kWM;
  const int kbeg = split * g.k_split;
  const int kend = min(g.K, kbeg + g.k_split);
  const int nt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const unsigned lds0 = lds_addr(lds);
  f32x16 acc[2][G::kTN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < G::kTN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  float bsum = 0.0f;
  // tiles 0 .. kBufs-2 in flight; iteration it: own pieces of tile it landed (younger
  // tiles' may still be in flight), barrier (tile it published, buffer of tile it-1 free),
  // tile it+kBufs-1 into that buffer, then tile it from LDS
  if (nt > 0) issue_ktile<G>(g, kbeg, kend, lds0, w, lane);
#pragma unroll
  for (int p = 1; p < G::kBufs - 1; ++p)
    if (p < nt) issue_ktile<G>(g, kbeg + p * BK, kend, lds0 + unsigned(p * G::kBufBytes), w, lane);
  int buf = 0;
  for (int it = 0; it < nt; ++it) {
    if (G::kBufs == 4 && it + 2 < nt) wait_vmcnt(2 * G::kInsPerWave);   // younger tiles may stay in flight
    else if (G::kBufs >= 3 && it + 1 < nt) wait_vmcnt(G::kInsPerWave);
    else wait_vmcnt(0);
    compiler_fence();
    __builtin_amdgcn_s_barrier();
    compiler_fence();
    if (it + G::kBufs - 1 < nt) {
      const int nb = buf >= 1 ? buf - 1 : G::kBufs - 1;      // (it + kBufs - 1) % kBufs
      issue_ktile<G>(g, kbeg + (it + G::kBufs - 1) * BK, kend, lds0 + unsigned(nb * G::kBufBytes), w, lane);
    }
    float* cur = lds + buf * (G::kBufBytes / 4);
    const int valid = kend - (kbeg + it * BK);
    if (valid < BK) {                 // the split's partial last k tile: A rows past K as zeros
      for (int i = t; i < BK * BMT; i += G::kThreads)
        if (i / BMT >= valid) cur[i] = 0.0f;
      __syncthreads();
    }
    if constexpr (kWgradX3) wgrad_tile_x3<G, BMT, W1, W2>(cur, acc, bsum, wm, wn, h, l32, t);
    else wgrad_tile<G, BMT, W1, W2>(cur, acc, bsum, wm, wn, h, l32, t);
    buf = buf + 1 == G::kBufs ? 0 : buf + 1;
  }
  float* c = g.c + long(split) * g.c_split;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < G::kTN; ++j) {
      const int n = wtile_col<G, W1>(wn, j) + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = wm * 64 + i * 32 + acc_row(r, h);
        if (n < g.N && m < g.M) c[long(m) * g.ldc + n] = acc[i][j][r];
      }
    }
  if (t < BMT && t < g.M) g.bias_part[long(split) * g.M + t] = bsum;
}

// All weight-gradient jobs of a net in one launch (they only need the forward's rows and
// the backward-data chain's dZ): job j owns workgroups [first[j], first[j+1]), one split
// each, with splits in proportion to the job's MFMA work, so every CU gets about the same
// work, the chip fills once, and the partials (one M x N block per workgroup) stay few.
enum WShape { kW256x256 = 0, kW256x319, kW256x63, kW128x283, kNumWShapes };
constexpr int kMaxWJobs = 9;
struct WGroup {
  GemmArgs g[kMaxWJobs];
  int shape[kMaxWJobs];
  int first[kMaxWJobs + 1];
  int n;
};
constexpr int kWgradLdsBytes = std::max(
    std::max(WGeo<256, 256, 0, 8>::kBufs * WGeo<256, 256, 0, 8>::kBufBytes,
             WGeo<256, 256, 64, 8>::kBufs * WGeo<256, 256, 64, 8>::kBufBytes),
    std::max(WGeo<256, 64, 0, 8>::kBufs * WGeo<256, 64, 0, 8>::kBufBytes,
             WGeo<128, 256, 28, 8>::kBufs * WGeo<128, 256, 28, 8>::kBufBytes));

__global__ __launch_bounds__(512) void wgrad_group_kernel(WGroup grp) {
  __shared__ __attribute__((aligned(1024))) float lds[kWgradLdsBytes / 4];
  int j = 0;
  while (j + 1 < grp.n && int(blockIdx.x) >= grp.first[j + 1]) ++j;
  const int split = int(blockIdx.x) - grp.first[j];
  switch (grp.shape[j]) {
    case kW256x256: wgrad_split<256, 256, 0, 8>(grp.g[j], split, lds); break;
    case kW256x319: wgrad_split<256, 256, 64, 8>(grp.g[j], split, lds); break;
    case kW256x63: wgrad_split<256, 64, 0, 8>(grp.g[j], split, lds); break;
    default: wgrad_split<128, 256, 28, 8>(grp.g[j], split, lds); break;
  }
}

// ---------------------------------------------------------- element-wise --
struct Pose {
  float r[9];   // camera-to-world rotation, row-major
  float t[3];
};

// _get_rays (trainer.py:271-292) for the selected pixels (:106-114), and their targets.
__global__ void train_rays_kernel(Pose pose, int width, int n_pix, float half_w, float half_h, float focal,
                                  const int* __restrict__ select, int n_rays, const float* __restrict__ image,
                                  float* __restrict__ rays_o, float* __restrict__ rays_d, float* __restrict__ target,
                                  int* __restrict__ bad) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rays) return;
  int idx = select[r];
  if (idx < 0 || idx >= n_pix) {
    *bad = 1;
    idx = 0;
  }
  const int row = idx / width, col = idx - (idx / width) * width;
  const float dx = __fdiv_rn(__fsub_rn(float(col), half_w), focal);
  const float dy = -__fdiv_rn(__fsub_rn(float(row), half_h), focal);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float p0 = __fmul_rn(dx, pose.r[3 * c + 0]);
    const float p1 = __fmul_rn(dy, pose.r[3 * c + 1]);
    const float p2 = -pose.r[3 * c + 2];
    rays_d[3 * r + c] = __fadd_rn(__fadd_rn(p0, p1), p2);
    rays_o[3 * r + c] = pose.t[c];
    target[3 * r + c] = image[3L * idx + c];
  }
}

// Sample points o + d*z and their encodings (nerf.py:24-45): pe [P][64] =
// [x, sin/cos(2^k pi x) k < 10, 0], dpe [P][28] = [d, sin/cos(2^k pi d) k < 4, 0].
__global__ __launch_bounds__(256) void train_encode_kernel(const float* __restrict__ rays_o, const float* __restrict__ rays_d,
                                    const float* __restrict__ z, int z_stride, int n_samples, long n_points,
                                    float* __restrict__ pe, float* __restrict__ dpe) {
  const long p = long(blockIdx.x) * blockDim.x + threadIdx.x;
  if (p >= n_points) return;
  const long ray = p / n_samples;
  const int s = int(p - ray * n_samples);
  const float zz = z[ray * z_stride + s];
  float x[3], d[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    d[c] = rays_d[3 * ray + c];
    x[c] = sample_coord(rays_o[3 * ray + c], d[c], zz);
  }
  float v[kPeLd];
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = x[c];
#pragma unroll
  for (int k = 0; k < 10; ++k)
#pragma unroll
    for (int c = 0; c < 3; ++c) pe_sincos<false, true>(pe_coef(k), x[c], &v[3 + 6 * k + c], &v[6 + 6 * k + c]);
  v[63] = 0.0f;
  f32x4* po = (f32x4*)(pe + p * kPeLd);
#pragma unroll
  for (int q = 0; q < kPeLd / 4; ++q) po[q] = f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
  float u[kDpeLd];
#pragma unroll
  for (int c = 0; c < 3; ++c) u[c] = d[c];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < 3; ++c) pe_sincos<false, true>(pe_coef(k), d[c], &u[3 + 6 * k + c], &u[6 + 6 * k + c]);
  u[27] = 0.0f;
  f32x4* du = (f32x4*)(dpe + p * kDpeLd);
#pragma unroll
  for (int q = 0; q < kDpeLd / 4; ++q) du[q] = f32x4{u[4 * q], u[4 * q + 1], u[4 * q + 2], u[4 * q + 3]};
}

// volume_render (rendering.py:102-143) forward, the MSE term of this ray, and the
// backward of both (autograd's graph for these ops, restated):
//   g_c          = 2 (rgb_map_c - target_c) / (3 n_rays)          (mse_loss backward)
//   g_w_i        = sum_c g_c c_ic,  g_c_ic = w_i g_c                 (sum(w[...,None]*rgb))
//   g_alpha_i    = g_w_i T_i - g_q_i,  g_T_i = g_w_i alpha_i         (w = alpha * T)
//   g_q_j        = (sum_{i>=j} g_t_i t_i) / q_j,  g_t_i = g_T_{i+1}  (cumprod backward, the
//                  reversed cumsum accumulated in double as torch's CPU cumsum)
//   g_sigma_i    = g_alpha_i e_i dist_i [sigma_i > 0]                (alpha = 1 - exp(-relu(s) d))
// then the sigmoid and density-ReLU backward: dpre[p] = (d r, d g, d b, d sigma) pre-activation.
// One wave per ray: lane l holds the contiguous chunk of samples [l c, (l + 1) c), c =
// ceil(S / 64).  The transmittance product and the backward's reversed cumsum are scans in
// double over the lanes -- the same products and sums as the sequential restatement,
// associated differently (~1e-16 relative, far below the floats they are rounded to);
// rgb_map is summed in sample order, lane after lane.  tbuf holds t_s = float(prod_{i <= s} q_i) for the
// backward (written and read by the same lane).
constexpr int kMaxChunk = 16;   // samples per lane at most (1024 per ray)
__global__ __launch_bounds__(256) void render_train_kernel(const f32x4* __restrict__ rgbs,
                                                           const float* __restrict__ z, int z_stride,
                                                           const float* __restrict__ rays_d,
                                                           const float* __restrict__ target, int n_rays,
                                                           int n_samples, float gnorm, float* __restrict__ tbuf,
                                                           f32x4* __restrict__ dpre, float* __restrict__ loss_ray) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n_rays) return;                                   // wave-uniform
  const float dx = rays_d[3L * r], dy = rays_d[3L * r + 1], dz = rays_d[3L * r + 2];
  const float norm = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz)));
  const float* zr = z + long(r) * z_stride;
  const long base = long(r) * n_samples;
  const int c = (n_samples + 63) / 64;                       // <= kMaxChunk (n_samples <= 1024)
  const int s0 = min(lane * c, n_samples), s1 = min(s0 + c, n_samples);
  auto dist_of = [&](int s) { return __fmul_rn(s + 1 < n_samples ? __fsub_rn(zr[s + 1], zr[s]) : 1e10f, norm); };
  // forward: this lane's product of q, then the exclusive product over the lanes before it
  double lp = 1.0;
  for (int s = s0; s < s1; ++s) {
    const float e = expf(__fmul_rn(-relu(rgbs[base + s][3]), dist_of(s)));
    lp = __dmul_rn(lp, double(__fadd_rn(__fsub_rn(1.0f, __fsub_rn(1.0f, e)), 1e-10f)));
  }
  double incl = lp;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double o = __shfl_up(incl, d);
    if (lane >= d) incl = __dmul_rn(o, incl);
  }
  double excl = __shfl_up(incl, 1);
  if (lane == 0) excl = 1.0;
  double tacc = excl;
  float wc[kMaxChunk][3];     // this lane's w_s c_s, in sample order
#pragma unroll
  for (int j = 0; j < kMaxChunk; ++j) {
    const int s = s0 + j;
    if (s < s1) {
      const f32x4 v = rgbs[base + s];
      const float alpha = __fsub_rn(1.0f, expf(__fmul_rn(-relu(v[3]), dist_of(s))));
      const float w = __fmul_rn(alpha, float(tacc));
#pragma unroll
      for (int k = 0; k < 3; ++k) wc[j][k] = __fmul_rn(w, v[k]);
      tacc = __dmul_rn(tacc, double(__fadd_rn(__fsub_rn(1.0f, alpha), 1e-10f)));
      tbuf[base + s] = float(tacc);
    }
  }
  // rgb_map = sum_s w_s c_s in sample order (torch's order for this reduction): the running
  // sum passes from lane to lane, each adding its chunk term by term
  float rm[3] = {0.0f, 0.0f, 0.0f};
  const int used = (n_samples + c - 1) / c;                  // lanes holding samples
  for (int l = 0; l < used; ++l) {
    if (lane == l)
#pragma unroll
      for (int j = 0; j < kMaxChunk; ++j)
        if (s0 + j < s1)
#pragma unroll
          for (int k = 0; k < 3; ++k) rm[k] = __fadd_rn(rm[k], wc[j][k]);
#pragma unroll
    for (int k = 0; k < 3; ++k)
      rm[k] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, rm[k]), l));
  }
  float g[3], loss = 0.0f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float diff = __fsub_rn(rm[k], target[3L * r + k]);
    loss = __fadd_rn(loss, __fmul_rn(diff, diff));
    g[k] = __fmul_rn(gnorm, diff);
  }
  if (lane == 0) loss_ray[r] = loss;
  // backward.  g_t_s = g_T_{s+1} = g_w_{s+1} alpha_{s+1} (0 for the last sample): a chunk's
  // last sample takes it from the next lane's first
  auto gw_of = [&](const f32x4& v) {
    return __fadd_rn(__fadd_rn(__fmul_rn(g[0], v[0]), __fmul_rn(g[1], v[1])), __fmul_rn(g[2], v[2]));
  };
  float first = 0.0f;
  if (s0 < s1) {
    const f32x4 v = rgbs[base + s0];
    first = __fmul_rn(gw_of(v), __fsub_rn(1.0f, expf(__fmul_rn(-relu(v[3]), dist_of(s0)))));
  }
  float next = __shfl_down(first, 1);
  if (lane == 63) next = 0.0f;
  // this lane's sum of t_s g_t_s, then the sum over the lanes after it (the reversed cumsum)
  double ls = 0.0;
  float nx = next;
  for (int s = s1 - 1; s >= s0; --s) {
    const f32x4 v = rgbs[base + s];
    ls = __dadd_rn(ls, double(__fmul_rn(tbuf[base + s], nx)));
    nx = __fmul_rn(gw_of(v), __fsub_rn(1.0f, expf(__fmul_rn(-relu(v[3]), dist_of(s)))));
  }
  double sinc = ls;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double o = __shfl_down(sinc, d);
    if (lane + d < 64) sinc = __dadd_rn(sinc, o);
  }
  double suffix = __shfl_down(sinc, 1);
  if (lane == 63) suffix = 0.0;
  float g_t = next;
  for (int s = s1 - 1; s >= s0; --s) {
    const float dist = dist_of(s);
    const f32x4 v = rgbs[base + s];
    const float sg = relu(v[3]);
    const float e = expf(__fmul_rn(-sg, dist));
    const float alpha = __fsub_rn(1.0f, e);
    const float T = s > s0 ? tbuf[base + s - 1] : float(excl);
    const float t_s = tbuf[base + s];
    const float q = __fadd_rn(__fsub_rn(1.0f, alpha), 1e-10f);
    const float w = __fmul_rn(alpha, T);
    const float gw = gw_of(v);
    suffix = __dadd_rn(suffix, double(__fmul_rn(t_s, g_t)));
    const float g_q = __fdiv_rn(float(suffix), q);
    const float g_alpha = __fsub_rn(__fmul_rn(gw, T), g_q);
    const float g_sig = sg > 0.0f ? __fmul_rn(__fmul_rn(g_alpha, e), dist) : 0.0f;
    g_t = __fmul_rn(gw, alpha);    // g_T_s = g_t_{s-1}
    f32x4 d;
#pragma unroll
    for (int k = 0; k < 3; ++k) d[k] = __fmul_rn(__fmul_rn(__fmul_rn(w, g[k]), __fsub_rn(1.0f, v[k])), v[k]);
    d[3] = g_sig;
    dpre[base + s] = d;
  }
}

// Backward of colour-1 and the colour-0 / density ReLUs: dhc [P][132] = the head
// GEMM's pre-activation gradient (columns 0..127 colour-0, 128 density, then zeros).
__global__ void head_bwd_kernel(const float* __restrict__ hc, const f32x4* __restrict__ dpre,
                                const float* __restrict__ prm, long n_points, float* __restrict__ dhc) {
  const long e = long(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= n_points * (kHeadLd / 4)) return;
  const long p = e / (kHeadLd / 4);
  const int n = int(e - p * (kHeadLd / 4)) * 4;
  const f32x4 d = dpre[p];
  f32x4 o = {0.0f, 0.0f, 0.0f, 0.0f};
  if (n < kC0) {
    const f32x4 hv = ld4(hc + p * kHeadLd + n);
    const float* w1 = prm + kFC1W;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = __fadd_rn(__fadd_rn(__fmul_rn(d[0], w1[n + j]), __fmul_rn(d[1], w1[kC0 + n + j])),
                                 __fmul_rn(d[2], w1[2 * kC0 + n + j]));
      o[j] = hv[j] > 0.0f ? gj : 0.0f;
    }
  } else {
    o[0] = d[3];
  }
  *(f32x4*)(dhc + p * kHeadLd + n) = o;
}

// ------------------------------------------------------- fused forward --
// The forward of one net in one launch, in mlp_f32.hip's register-stationary shape
// (4 waves x 32 samples, one wave per SIMD, H^T = W . X^T with the accumulator of a
// layer as the next layer's B operand, A fragments read as float4 from the f32 blob
// in L2), plus what the backward needs: every trunk layer's post-ReLU rows [P][256]
// and its ReLU bits [P][8] words, the colour-0 output and the density [P][132],
// and (r, g, b, sigma) per sample.  Same numerics as the parity render path.
template <int L>
constexpr int f32_layer_offset_t() {
  int off = 0;
  for (int l = 0; l < L; ++l) off += f32_layer_floats(l);
  return off;
}

// prev holds the previous layer's pre-activation accumulators: tile t is ReLU'd at the start
// of k-step group 4t, the first group that reads it, together with its ReLU bit word (the
// backward's mask), so that work runs between this layer's MFMAs instead of as a serial
// block at the layer boundary.  prev_row (optional): where the ReLU'd activations go as a
// row of this lane's sample, one 16-B piece per group after that group's weight loads (no
// weight load waits behind more than one store: vmcnt counts loads and stores in issue
// order); prev_bits (optional): the previous layer's 8 bit words for this sample, stored by
// lane half 0 once all eight are known.  Weight fragments run one k-step group ahead: pf
// holds this layer's group 0 on entry (loaded during the previous layer's last group) and
// the next layer's (LN; -1: none) on exit, so a group's loads have a whole group of MFMAs
// (2,048 cycles) to arrive.
template <int L, int NT, int NEXT, int LN, int NTN>
__device__ __forceinline__ void fwd_layer(f32x16 (&acc)[8], f32x16 (&prev)[8], const float (&ext)[NEXT],
                                          const f32x4* __restrict__ blob, const float* __restrict__ prm, int lane,
                                          int h, f32x4 (&pf)[8], float* __restrict__ prev_row = nullptr,
                                          unsigned* __restrict__ prev_bits = nullptr) {
  constexpr LayerShape sh = layer_shape(L);
  constexpr int KH = sh.hidden / 2;
  constexpr int KU = ksteps_f32(L);
  constexpr int G = KU / 4;
  static_assert(KU == KH + (sh.extra == kNone ? 0 : NEXT), "layer/ext mismatch");
  static_assert(KH == 0 || KH == 128, "hidden inputs: none or 256 features (8 tiles)");
  load_bias<NT>(acc, prm, L, h);
  const f32x4* a_base = blob + f32_layer_offset_t<L>() / 4 + lane;
  f32x4 a[2][NT];
  unsigned wbits[8];
#pragma unroll
  for (int o = 0; o < NT; ++o) a[0][o] = pf[o];
#pragma unroll
  for (int ug = 0; ug < G; ++ug) {
    if (ug + 1 < G) {
#pragma unroll
      for (int o = 0; o < NT; ++o) a[(ug + 1) & 1][o] = a_base[((ug + 1) * NT + o) * 64];
    } else if (LN >= 0) {
      const f32x4* n_base = blob + f32_layer_offset_t<(LN >= 0 ? LN : 0)>() / 4 + lane;
#pragma unroll
      for (int o = 0; o < NTN; ++o) pf[o] = n_base[o * 64];
    }
    if (KH > 0 && ug % 4 == 0 && ug < KH / 4) {   // tile t of prev: ReLU, then its bit word
      const int t = ug / 4;
      unsigned m = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        prev[t][r] = relu(prev[t][r]);
        m |= (prev[t][r] > 0.0f ? 1u : 0u) << acc_row(r, h);
      }
      const auto sw = __builtin_amdgcn_permlane32_swap(m, m, false, false);
      wbits[t] = unsigned(sw[0]) | unsigned(sw[1]);
    }
    // row piece pc = 4t + j of prev goes out one group late (after group pc + 1's loads), so
    // that it is younger than the loads the next group waits for: vmcnt retires loads and
    // stores in issue order, and a store issued before a group's loads made that group wait
    // for the store's completion too.  A layer without encoding groups stores its last piece
    // (and the bit words) after its last group's loads.
    if (KH > 0 && prev_row != nullptr) {
      auto store_piece = [&](int pc) {
        const int t = pc >> 2, j = pc & 3;
        *(f32x4*)(prev_row + 32 * t + 8 * j + 4 * h) =
            f32x4{prev[t][4 * j], prev[t][4 * j + 1], prev[t][4 * j + 2], prev[t][4 * j + 3]};
        if (pc == KH / 4 - 1 && prev_bits != nullptr && h == 0) {
          ((u32x4_t*)prev_bits)[0] = u32x4_t{wbits[0], wbits[1], wbits[2], wbits[3]};
          ((u32x4_t*)prev_bits)[1] = u32x4_t{wbits[4], wbits[5], wbits[6], wbits[7]};
        }
      };
      if (ug >= 1 && ug - 1 < KH / 4) store_piece(ug - 1);
      if (ug == G - 1 && G == KH / 4) store_piece(ug);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = 4 * ug + i;
      const float b = u < KH ? prev[u >> 4][u & 15] : ext[u - KH];
#pragma unroll
      for (int o = 0; o < NT; ++o) acc[o] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ug & 1][o][i], b, acc[o], 0, 0, 0);
    }
  }
}

// Rows of this lane's sample: register 4j..4j+3 of tile t are features 32t + 8j + 4h + 0..3.
template <int NT>
__device__ __forceinline__ void store_rows(const f32x16 (&a)[8], float* __restrict__ row, int h) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *(f32x4*)(row + 32 * t + 8 * j + 4 * h) = f32x4{a[t][4 * j], a[t][4 * j + 1], a[t][4 * j + 2], a[t][4 * j + 3]};
}

struct FwdOut {
  float* h[8];
  unsigned* mb[8];
  float* hc;
  f32x4* rgbs;
};

__global__ __launch_bounds__(256, 1) void train_fwd_kernel(const f32x4* __restrict__ blob,
                                                           const float* __restrict__ prm, SampleSrc src, long n_points,
                                                           FwdOut o) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int h = lane >> 5;
  const long p = (long(blockIdx.x) * 4 + wave) * kSamplesPerWave + (lane & 31);
  const bool valid = p < n_points;
  const long pc = valid ? p : n_points - 1;
  f32x4 pf[8];                      // layer 0's first weight fragments, in flight during the encoding
#pragma unroll
  for (int o = 0; o < 8; ++o) pf[o] = blob[lane + o * 64];
  float x[3], d[3];
  fetch_sample<false>(src, pc, x, d);
  float pe[32], de[16];
  pos_encode<false, true>(x[0], x[1], x[2], h, pe);
  dir_encode<false, true>(d[0], d[1], d[2], h, de);
  f32x16 a[8], b[8];
  // each layer's ReLU, bit words and rows happen while the next layer runs (fwd_layer)
  float* const nul = nullptr;
  unsigned* const nulb = nullptr;
#define ROW(l) (valid ? o.h[l] + p * kH : nul)
#define BITS(l) (valid ? o.mb[l] + p * (kH / 32) : nulb)
  fwd_layer<L0, 8, 32, L1, 8>(a, b, pe, blob, prm, lane, h, pf);
  fwd_layer<L1, 8, 32, L2, 8>(b, a, pe, blob, prm, lane, h, pf, ROW(0), BITS(0));
  fwd_layer<L2, 8, 32, L3, 8>(a, b, pe, blob, prm, lane, h, pf, ROW(1), BITS(1));
  fwd_layer<L3, 8, 32, L4, 8>(b, a, pe, blob, prm, lane, h, pf, ROW(2), BITS(2));
  fwd_layer<L4, 8, 32, L5, 8>(a, b, pe, blob, prm, lane, h, pf, ROW(3), BITS(3));   // skip: [x, pe] (nerf.py:109-110)
  fwd_layer<L5, 8, 32, L6, 8>(b, a, pe, blob, prm, lane, h, pf, ROW(4), BITS(4));
  fwd_layer<L6, 8, 32, L7, 8>(a, b, pe, blob, prm, lane, h, pf, ROW(5), BITS(5));
  fwd_layer<L7, 8, 32, C0, 4>(b, a, pe, blob, prm, lane, h, pf, ROW(6), BITS(6));
  fwd_layer<C0, 4, 16, -1, 0>(a, b, de, blob, prm, lane, h, pf, ROW(7), BITS(7));   // [x, PE4(d)] (nerf.py:117-121)
  const float sigma = density_head(b, prm, h);    // b: layer 7's outputs, ReLU'd inside C0's pass
#undef ROW
#undef BITS
  relu_tiles<4>(a);
  if (valid) store_rows<4>(a, o.hc + p * kHeadLd, h);
  float rgb[3];
  color_head(a, prm, h, rgb);
  if (valid && h == 0) {
    o.hc[p * kHeadLd + kC0] = sigma;
    o.rgbs[p] = f32x4{rgb[0], rgb[1], rgb[2], sigma};
  }
}

// ------------------------------------------------ fused backward-data chain --
// dZ_{l-1} = (W_l^T dZ_l) * bit(H_{l-1}) for the head and layers 7..1 in one launch, the
// forward's register-stationary shape run backwards: dX^T[in, sample] = W^T[in, out] .
// dZ^T[out, sample], so a layer's masked accumulator is the next one's B operand.  Starts
// from the head's pre-activation gradient rows [P][132] (colour-0, density); writes dZ_l
// rows [P][256] for l = 7..0 (the weight gradients' A operand), each stored piecewise
// during the following layer as in the forward.
// Weight fragments one k-step group ahead as in fwd_layer: pf holds this layer's group 0
// on entry and the next backward layer's (its blob at next_blob; nullptr: none) on exit.
template <int KU>
__device__ __forceinline__ void bwd_layer(f32x16 (&acc)[8], const f32x16 (&prev)[8], float dens,
                                          const f32x4* __restrict__ blob, const f32x4* __restrict__ next_blob,
                                          int lane, int h, f32x4 (&pf)[8], float* __restrict__ prev_row) {
  constexpr int KH = KU == kHeadBwdKsteps ? kC0 / 2 : KU;   // k-steps fed by prev; the head's next is the density
  constexpr int G = KU / 4;
#pragma unroll
  for (int o = 0; o < 8; ++o)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[o][r] = 0.0f;
  const f32x4* a_base = blob + lane;
  f32x4 a[2][8];
#pragma unroll
  for (int o = 0; o < 8; ++o) a[0][o] = pf[o];
#pragma unroll
  for (int ug = 0; ug < G; ++ug) {
    if (ug + 1 < G) {
#pragma unroll
      for (int o = 0; o < 8; ++o) a[(ug + 1) & 1][o] = a_base[((ug + 1) * 8 + o) * 64];
    } else if (next_blob != nullptr) {
#pragma unroll
      for (int o = 0; o < 8; ++o) pf[o] = next_blob[lane + o * 64];
    }
    if (prev_row != nullptr) {     // 256-wide dZ rows: 32 pieces of 16 B, one group late (fwd_layer)
      auto store_piece = [&](int pc) {
        const int t = pc >> 2, j = pc & 3;
        *(f32x4*)(prev_row + 32 * t + 8 * j + 4 * h) =
            f32x4{prev[t][4 * j], prev[t][4 * j + 1], prev[t][4 * j + 2], prev[t][4 * j + 3]};
      };
      if (ug >= 1 && ug - 1 < 32) store_piece(ug - 1);
      if (ug == G - 1 && G == 32) store_piece(ug);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = 4 * ug + i;
      const float b = u < KH ? prev[u >> 4][u & 15] : (u == KH && h == 0 ? dens : 0.0f);
#pragma unroll
      for (int o = 0; o < 8; ++o) acc[o] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ug & 1][o][i], b, acc[o], 0, 0, 0);
    }
  }
}

__device__ __forceinline__ void apply_bits(f32x16 (&acc)[8], const u32x4_t (&w)[2], int h) {
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const unsigned word = w[t >> 2][t & 3];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = (word >> acc_row(r, h)) & 1u ? acc[t][r] : 0.0f;
  }
}

struct BwdIo {
  const float* dhc;          // [P][132]
  const unsigned* mb[8];     // ReLU bits of H_0..H_7, [P][8]
  float* dz[8];              // out: dZ_0..dZ_7 rows [P][256]
};

__global__ __launch_bounds__(256, 1) void train_bwd_kernel(const f32x4* __restrict__ blob, long n_points, BwdIo io) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int h = lane >> 5;
  const long p = (long(blockIdx.x) * 4 + wave) * kSamplesPerWave + (lane & 31);
  const bool valid = p < n_points;
  const long pc = valid ? p : n_points - 1;
  f32x4 pf[8];                      // the head's first weight fragments, in flight during the row loads
#pragma unroll
  for (int o = 0; o < 8; ++o) pf[o] = blob[bwd_layer_offset(0) / 4 + lane + o * 64];
  f32x16 a[8], b[8];
  // the head's gradient rows as a 4-tile "accumulator" (feature 32t + acc_row(r, h))
  const float* row = io.dhc + pc * kHeadLd;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 v = ld4(row + 32 * t + 8 * j + 4 * h);
#pragma unroll
      for (int q = 0; q < 4; ++q) b[t][4 * j + q] = v[q];
    }
  const float dens = row[kC0];
  u32x4_t w[2];
  auto load_bits = [&](int l) {
    const u32x4_t* src = (const u32x4_t*)(io.mb[l] + pc * (kH / 32));
    w[0] = src[0];
    w[1] = src[1];
  };
  float* const nul = nullptr;
#define DZ(l) (valid ? io.dz[l] + p * kH : nul)
  load_bits(7);
#define BLOB(b) (blob + bwd_layer_offset(b) / 4)
  bwd_layer<kHeadBwdKsteps>(a, b, dens, BLOB(0), BLOB(1), lane, h, pf, nul);
  apply_bits(a, w, h);                                              // dZ_7
  load_bits(6);
  bwd_layer<128>(b, a, 0.0f, BLOB(1), BLOB(2), lane, h, pf, DZ(7));
  apply_bits(b, w, h);                                              // dZ_6
  load_bits(5);
  bwd_layer<128>(a, b, 0.0f, BLOB(2), BLOB(3), lane, h, pf, DZ(6));
  apply_bits(a, w, h);                                              // dZ_5
  load_bits(4);
  bwd_layer<128>(b, a, 0.0f, BLOB(3), BLOB(4), lane, h, pf, DZ(5));
  apply_bits(b, w, h);                                              // dZ_4
  load_bits(3);
  bwd_layer<128>(a, b, 0.0f, BLOB(4), BLOB(5), lane, h, pf, DZ(4));   // layer 4's hidden inputs
  apply_bits(a, w, h);                                              // dZ_3
  load_bits(2);
  bwd_layer<128>(b, a, 0.0f, BLOB(5), BLOB(6), lane, h, pf, DZ(3));
  apply_bits(b, w, h);                                              // dZ_2
  load_bits(1);
  bwd_layer<128>(a, b, 0.0f, BLOB(6), BLOB(7), lane, h, pf, DZ(2));
  apply_bits(a, w, h);                                              // dZ_1
  load_bits(0);
  bwd_layer<128>(b, a, 0.0f, BLOB(7), nullptr, lane, h, pf, DZ(1));
  apply_bits(b, w, h);                                              // dZ_0
#undef BLOB
  if (valid) store_rows<8>(b, io.dz[0] + p * kH, h);
#undef DZ
}

// --------------------------------------------------- gradient reduction --
// Sums the split-K partials of one weight-gradient GEMM in split order and
// scatters them into the flat gradients: rows [0, r1) to (w0 + m*ld0, n < nw0;
// bias b0 + m), rows [r1, M) to (w1 + (m-r1)*ld1, n < nw1; bias b1 + m - r1).
struct RedJob {
  const float* part;
  const float* bpart;
  int splits, M, N;
  int r1;
  long w0, b0;
  int ld0, nw0;
  long w1, b1;
  int ld1, nw1;
};
constexpr int kMaxJobs = 11;
struct RedJobs {
  RedJob j[kMaxJobs];
};

__global__ void reduce_grads_kernel(RedJobs jobs, float* __restrict__ grads) {
  const RedJob& jb = jobs.j[blockIdx.y];
  const long e = long(blockIdx.x) * blockDim.x + threadIdx.x;
  const long mn = long(jb.M) * jb.N;
  const float* src;
  long stride, dst;
  if (e < mn) {
    const int m = int(e / jb.N), n = int(e - long(m) * jb.N);
    const bool g0 = m < jb.r1;
    if (n >= (g0 ? jb.nw0 : jb.nw1)) return;
    src = jb.part + e;
    stride = mn;
    dst = g0 ? jb.w0 + long(m) * jb.ld0 + n : jb.w1 + long(m - jb.r1) * jb.ld1 + n;
  } else if (e < mn + jb.M) {
    const int m = int(e - mn);
    src = jb.bpart + m;
    stride = jb.M;
    dst = m < jb.r1 ? jb.b0 + m : jb.b1 + (m - jb.r1);
  } else {
    return;
  }
  // four interleaved partial sums (split k into sum k % 4), then combined: a fixed
  // order, so the result is deterministic, with four loads in flight per thread
  float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  int k = 0;
  for (; k + 4 <= jb.splits; k += 4)
#pragma unroll
    for (int q = 0; q < 4; ++q) s4[q] = __fadd_rn(s4[q], src[(k + q) * stride]);
  for (; k < jb.splits; ++k) s4[k & 3] = __fadd_rn(s4[k & 3], src[k * stride]);
  grads[dst] = __fadd_rn(__fadd_rn(s4[0], s4[1]), __fadd_rn(s4[2], s4[3]));
}

// The same reduction for jobs with many splits (the skinny layers': one per 256 samples):
// one workgroup per element, thread t sums splits t, t + 256, ..., then a fixed-order tree
// over the 256 threads (deterministic).
__global__ __launch_bounds__(256) void reduce_wide_kernel(RedJobs jobs, int first, float* __restrict__ grads) {
  const RedJob& jb = jobs.j[first + blockIdx.y];
  const long e = blockIdx.x;
  const long mn = long(jb.M) * jb.N;
  if (e >= mn + jb.M) return;                            // uniform per workgroup
  const float* src;
  long stride, dst;
  if (e < mn) {
    const int m = int(e / jb.N), n = int(e - long(m) * jb.N);
    src = jb.part + e, stride = mn;
    dst = jb.w0 + long(m) * jb.ld0 + n;
  } else {
    const int m = int(e - mn);
    src = jb.bpart + m, stride = jb.M;
    dst = jb.b0 + m;
  }
  __shared__ float red[256];
  float acc = 0.0f;
  for (int k = threadIdx.x; k < jb.splits; k += 256) acc = __fadd_rn(acc, src[k * stride]);
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (int(threadIdx.x) < w) red[threadIdx.x] = __fadd_rn(red[threadIdx.x], red[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) grads[dst] = red[0];
}

// Weight gradients of the skinny layers in one launch: colour-1 (3 rows over the 128
// colour-0 outputs, A = the r, g, b of dpre) and density (1 row over layer 7's 256 outputs,
// A = dpre's sigma); partial[split][m][n] = sum over the split's samples of A[p][m] * B[p][n]
// and the bias partials sum_p A[p][m].  Per sample phase (every 4th sample of the split) one
// wave takes the colour columns (two per lane, float2 loads) and one the density columns
// (four per lane, float4 loads), so no wave diverges; the four phase sums are then added in
// a fixed order.  HBM-bound: dpre, the colour-0 rows and layer 7's rows are read once.
__global__ __launch_bounds__(512) void skinny_wgrad_kernel(const f32x4* __restrict__ dpre,
                                                           const float* __restrict__ hc, int ldh,
                                                           const float* __restrict__ h7, long P, int chunk,
                                                           float* __restrict__ pc, float* __restrict__ pcb,
                                                           float* __restrict__ pd, float* __restrict__ pdb) {
  __shared__ float red[4][4][256];   // [phase][colour row 0-2 | density 3][column]
  __shared__ float bred[4][4];
  const int split = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ph = wv >> 1;
  const bool colour = (wv & 1) == 0;                       // wave-uniform
  const long p0 = long(split) * chunk;
  const long p1 = p0 + chunk < P ? p0 + chunk : P;
  float acc[3][4] = {}, bs[4] = {};
#pragma unroll 4
  for (long p = p0 + ph; p < p1; p += 4) {
    const f32x4 a = dpre[p];
    if (colour) {
      const f32x2_t b = *(const f32x2_t*)(hc + p * ldh + 2 * lane);
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        acc[m][0] = fmaf(a[m], b[0], acc[m][0]);
        acc[m][1] = fmaf(a[m], b[1], acc[m][1]);
        bs[m] = __fadd_rn(bs[m], a[m]);
      }
    } else {
      const f32x4 b = ld4(h7 + p * kH + 4 * lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[0][j] = fmaf(a[3], b[j], acc[0][j]);
      bs[3] = __fadd_rn(bs[3], a[3]);
    }
  }
  if (colour) {
#pragma unroll
    for (int m = 0; m < 3; ++m) *(f32x2_t*)&red[ph][m][2 * lane] = f32x2_t{acc[m][0], acc[m][1]};
    if (lane == 0)
#pragma unroll
      for (int m = 0; m < 3; ++m) bred[ph][m] = bs[m];
  } else {
    *(f32x4*)&red[ph][3][4 * lane] = f32x4{acc[0][0], acc[0][1], acc[0][2], acc[0][3]};
    if (lane == 0) bred[ph][3] = bs[3];
  }
  __syncthreads();
  const int t = threadIdx.x;
  auto sum4 = [&](int m, int n) {
    return __fadd_rn(__fadd_rn(red[0][m][n], red[1][m][n]), __fadd_rn(red[2][m][n], red[3][m][n]));
  };
  if (t < 3 * kC0) pc[long(split) * 3 * kC0 + t] = sum4(t / kC0, t % kC0);
  else if (t < 3 * kC0 + 3) pcb[long(split) * 3 + (t - 3 * kC0)] =
      __fadd_rn(__fadd_rn(bred[0][t - 3 * kC0], bred[1][t - 3 * kC0]), __fadd_rn(bred[2][t - 3 * kC0], bred[3][t - 3 * kC0]));
  if (t < kH) pd[long(split) * kH + t] = sum4(3, t);
  if (t == kH) pdb[split] = __fadd_rn(__fadd_rn(bred[0][3], bred[1][3]), __fadd_rn(bred[2][3], bred[3][3]));
}

// Sum of squares of all gradients (double), per block.
__global__ void sumsq_kernel(const float* __restrict__ g, long n, double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  for (long i = long(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x) {
    const double v = g[i];
    s += v * v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (int(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// Loss (trainer.py:117-119: mean over [n_rays][3] per net, summed) and the clip
// coefficient of clip_grad_norm_: min(max_norm / (total_norm + 1e-6), 1).
// out: [0] loss, [1] coarse MSE, [2] fine MSE; coef: the factor Adam applies.
__global__ void finalize_kernel(const float* __restrict__ loss_ray, int n_rays, int n_total,
                                const double* __restrict__ sq_part, int n_part, float max_norm, float* __restrict__ out,
                                float* __restrict__ coef) {
  __shared__ double red[3][256];
  double a = 0.0, b = 0.0, q = 0.0;
  for (int i = threadIdx.x; i < n_rays; i += blockDim.x) {
    a += loss_ray[i];
    b += loss_ray[n_rays + i];
  }
  if (sq_part)
    for (int i = threadIdx.x; i < n_part; i += blockDim.x) q += sq_part[i];
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  red[2][threadIdx.x] = q;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (int(threadIdx.x) < o)
      for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float denom = float(3.0 * n_total);
    const float mc = __fdiv_rn(float(red[0][0]), denom), mf = __fdiv_rn(float(red[1][0]), denom);
    if (out) {
      out[0] = __fadd_rn(mc, mf);
      out[1] = mc;
      out[2] = mf;
    }
    if (coef) {
      float c = 1.0f;
      if (sq_part && max_norm > 0.0f) {
        const float total = float(sqrt(red[2][0]));
        c = fminf(__fdiv_rn(max_norm, __fadd_rn(total, 1e-6f)), 1.0f);
      }
      *coef = c;
    }
  }
}

// torch.optim.Adam, single-tensor form (torch/optim/adam.py), after clip_grad_norm_'s
// in-place scaling: g *= coef; g += wd * p; m = lerp(m, g, 1 - b1); v = v*b2 + (1-b2)*g*g;
// p += (-step_size * m) / (sqrt(v) / bc2_sqrt + eps).
struct AdamArgs {
  float one_minus_b1, b2, one_minus_b2, wd, neg_step_size, bc2_sqrt, eps;
};
__global__ void adam_kernel(float* __restrict__ p, float* __restrict__ grad, float* __restrict__ m,
                            float* __restrict__ v, long n, const float* __restrict__ coef, AdamArgs a) {
  const long i = long(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float g = __fmul_rn(grad[i], *coef);
  grad[i] = g;                       // the reference's param.grad after the step: the clipped gradient
  const float pv = p[i];
  if (a.wd != 0.0f) g = fmaf(pv, a.wd, g);
  const float mv = fmaf(a.one_minus_b1, __fsub_rn(g, m[i]), m[i]);
  const float vv = __fadd_rn(__fmul_rn(v[i], a.b2), __fmul_rn(__fmul_rn(a.one_minus_b2, g), g));
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(vv), a.bc2_sqrt), a.eps);
  p[i] = __fadd_rn(pv, __fdiv_rn(__fmul_rn(a.neg_step_size, mv), denom));
  m[i] = mv;
  v[i] = vv;
}

// Flat parameters -> the GEMM operand copies (layout above), both nets.
__global__ void relayout_kernel(const float* __restrict__ params, float* __restrict__ gemmw) {
  const long e = long(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= kGemmFloats) return;
  const float* prm = params + blockIdx.y * kNetFloats;
  float* out = gemmw + blockIdx.y * kGemmFloats;
  float v = 0.0f;
  if (e < kF32Blob + f32_blob_floats()) {
    // pack.cpp's f32 blob, element by element: layer l, k-step group ug, tile o, lane, i
    long o = e - kF32Blob;
    int l = 0;
    while (l < kNumMfmaLayers - 1 && o >= f32_layer_floats(l)) o -= f32_layer_floats(l++);
    const int nt = out_tiles(l);
    const int i = int(o & 3), lane = int((o >> 2) & 63), tile = int((o >> 8) % nt), ug = int((o >> 8) / nt);
    const int row = 32 * tile + (lane & 31), col = f32_k_col(l, 4 * ug + i, lane >> 5);
    if (col >= 0) v = l == C0 ? prm[kFC0W + long(row) * kHeadK + col] : prm[w_off(l) + long(row) * kTrunkIn[l] + col];
  } else if (e >= kPrmBlob && e < kPrmBlob + kParamFloats) {
    const int q = int(e - kPrmBlob);
    if (q < kSigW) {                       // bias[l][tile][h][r]
      const int l = q / 256, rem = q % 256, tile = rem / 32, hh = (rem / 16) & 1, r = rem & 15;
      const int row = 32 * tile + acc_row(r, hh);
      if (tile < out_tiles(l)) v = l == C0 ? prm[kFC0B + row] : prm[b_off(l) + row];
    } else if (q < kSigB) {                // density weight [h][t][r]
      const int rem = q - kSigW, hh = rem / 128, t = (rem / 16) & 7, r = rem & 15;
      v = prm[kFDensW + 32 * t + acc_row(r, hh)];
    } else if (q == kSigB) {
      v = prm[kFDensB];
    } else if (q >= kC1W && q < kC1B) {    // colour-1 weight [c][h][t][r]
      const int rem = q - kC1W, c = rem / 128, hh = (rem / 64) & 1, t = (rem / 16) & 3, r = rem & 15;
      v = prm[kFC1W + c * kC0 + 32 * t + acc_row(r, hh)];
    } else if (q >= kC1B && q < kC1B + 3) {
      v = prm[kFC1B + (q - kC1B)];
    }
  } else if (e >= kBwdBlob && e < kBwdBlob + bwd_layer_offset(kBwdLayers)) {
    long o = e - kBwdBlob;
    int b = 0;
    while (b < kBwdLayers - 1 && o >= bwd_layer_floats(b)) o -= bwd_layer_floats(b++);
    const int i4 = int(o & 3), lane = int((o >> 2) & 63), tile = int((o >> 8) & 7), ug = int(o >> 11);
    const int u = 4 * ug + i4, hh = lane >> 5, in = 32 * tile + (lane & 31);
    if (b == 0) {
      if (u < kC0 / 2) v = prm[kFC0W + long(hid_f32_feature(u, hh)) * kHeadK + in];
      else if (u == kC0 / 2 && hh == 0) v = prm[kFDensW + in];
    } else {
      const int l = bwd_trunk_layer(b);
      v = prm[w_off(l) + long(hid_f32_feature(u, hh)) * kTrunkIn[l] + in];
    }
  }
  out[e] = v;
}

inline unsigned blocks_for(long n, int per) { return unsigned((n + per - 1) / per); }

}  // namespace
}  // namespace nerf

using namespace nerf;

// ----------------------------------------------------------------- host --
namespace nerf {
namespace {
// Flat parameters -> the split-bf16 blob of the forward (launch_mlp_bf16x3_train), both nets:
// pack.cpp's nerf_pack_weights_bf16x3 element by element (stream element i of bf16 unit
// n = i / 1024: layer l, quarter q, k-step u, tile-in-quarter o2, lane, j; then the heads'
// units of two k-steps), W_hi = bf16(W) into unit 2n and W_lo = bf16(W - W_hi) into 2n + 1.
constexpr int kX3UnitElems = kUnitBytes / 2;
constexpr long kX3Elems = long(kHeadUnitBase + kHeadUnits) * kX3UnitElems;
constexpr long kX3NetElems = kBf16x3BlobBytes / 2;
__global__ void pack_x3_kernel(const float* __restrict__ params, unsigned short* __restrict__ blob) {
  const long i = long(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= kX3Elems) return;
  const float* prm = params + blockIdx.y * kNetFloats;
  unsigned short* out = blob + blockIdx.y * kX3NetElems;
  const int n = int(i / kX3UnitElems), off = int(i % kX3UnitElems);
  const int lane = (off / 8) % 64, j = off % 8, half = off / 512;
  float v = 0.0f;
  if (n < kHeadUnitBase) {
    int l = 0;
    while (l + 1 < kNumMfmaLayers && bf16_unit_base(l + 1) <= n) ++l;
    const int ku = ksteps_bf16(l), r = n - bf16_unit_base(l), q = r / ku, u = r % ku;
    const int col = bf16_k_col(l, u, lane >> 5, j), row = 32 * (2 * q + half) + (lane & 31);
    const int spec = l == C0 ? 9 : l;
    const TensorDesc d = tensor_desc(2 * spec);
    if (col >= 0) v = prm[d.off + long(row) * d.cols + col];
  } else {
    const int u = 2 * (n - kHeadUnitBase) + half, row = lane & 31;
    int dens = 0;
    const int f = head_k_row_col(u, row, lane >> 5, j, &dens);
    if (f >= 0) v = dens ? prm[kFDensW + f] : prm[kFC1W + long(row) * kC0 + f];
  }
  const __bf16 hi = __bf16(v);                         // round to nearest even
  const float hf = float(hi);
  const __bf16 lo = __bf16(__fsub_rn(v, hf));          // exact in fp32
  out[long(2 * n) * kX3UnitElems + off] = __builtin_bit_cast(unsigned short, hi);
  out[long(2 * n + 1) * kX3UnitElems + off] = __builtin_bit_cast(unsigned short, lo);
}

// Flat parameters -> the split-bf16 weight stream of the backward-data chain
// (train_bwd_x3.hip, train_x3_layout.h), both nets: unit n = (backward layer b, quarter q,
// k-step u), element (tile-in-quarter o2, lane, j) = W[hid_bf16_feature(u, lane / 32, j)]
// [32 (2q + o2) + lane % 32] of the colour-0 layer (b = 0, its 256 hidden columns) or trunk
// layer 8 - b; its bf16 hi half into the unit's first 2 KiB, lo = bf16(w - hi) into the second.
constexpr long kBwdX3Elems = long(kBwdX3Units) * kX3UnitElems;        // elements of the hi (or lo) halves
constexpr long kBwdX3NetElems = kBwdX3BlobBytes / 2;
__global__ void pack_bwd_x3_kernel(const float* __restrict__ params, unsigned short* __restrict__ blob) {
  const long i = long(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= kBwdX3Elems) return;
  const float* prm = params + blockIdx.y * kNetFloats;
  unsigned short* out = blob + blockIdx.y * kBwdX3NetElems;
  const int n = int(i / kX3UnitElems), off = int(i % kX3UnitElems);
  const int lane = (off / 8) % 64, j = off % 8, o2 = off / 512;
  int b = 0;
  while (b + 1 < kBwdX3Layers && bwd_x3_unit_base(b + 1) <= n) ++b;
  const int ku = bwd_x3_ksteps(b), r = n - bwd_x3_unit_base(b), q = r / ku, u = r % ku;
  const int row = 32 * (2 * q + o2) + (lane & 31), f = hid_bf16_feature(u, lane >> 5, j);
  const int l = bwd_x3_trunk_layer(b);
  const float v = b == 0 ? prm[kFC0W + long(f) * kHeadK + row] : prm[w_off(l) + long(f) * kTrunkIn[l] + row];
  const __bf16 hi = __bf16(v);
  const __bf16 lo = __bf16(__fsub_rn(v, float(hi)));
  out[long(2 * n) * kX3UnitElems + off] = __builtin_bit_cast(unsigned short, hi);
  out[long(2 * n + 1) * kX3UnitElems + off] = __builtin_bit_cast(unsigned short, lo);
}
}  // namespace
}  // namespace nerf

struct nerf_trainer {
  int device = 0;
  nerf_train_config cfg{};
  double lr = 0.0;
  long steps = 0;
  float* params = nullptr;   // [2][kNetFloats]
  float* grads = nullptr;    // the gradient store in use: own_grads or a caller's buffer
  float* own_grads = nullptr;
  float* m = nullptr;
  float* v = nullptr;
  float* gemmw = nullptr;    // [2][kGemmFloats]
  unsigned short* x3 = nullptr;   // [2][kX3NetElems]: split-bf16 blob of the forward
  unsigned short* bx3 = nullptr;  // [2][kBwdX3NetElems]: split-bf16 blob of the backward-data chain
  bool fwd_x3 = false;            // forward and backward-data on the split-bf16 MFMA (nerf_trainer_set_precision)
  float* ztab = nullptr;     // coarse table [n_coarse], fine table [n_fine]
  float* scal = nullptr;     // [0] clip coefficient, then double sum-of-squares partials
  int* bad = nullptr;        // device flag: a select index out of range
  float* ws = nullptr;       // per-step workspace
  size_t ws_cap = 0;
  float* part = nullptr;     // weight-gradient partials (one net at a time)
  size_t part_cap = 0;
  bool profiling = false;
  bool have_times = false;
  hipEvent_t ev[14] = {};
  double gemm_flops = 0.0;
  // stream ordering: the workspace and state are reused by every call, so a call on a
  // stream other than the last one's waits for the last call's work (done)
  hipEvent_t done = nullptr;
  hipStream_t last_stream = nullptr;
  bool pending = false;
  // the coarse net's pass runs on a second stream beside the fine net's (they share only
  // the rays): fork after the rays and samples, join before the loss and the update
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};

namespace {

// The kernels' operand copies of both nets' weights (after every change of the parameters).
hipError_t pack_operands(nerf_trainer* tr, hipStream_t s) {
  hipLaunchKernelGGL(relayout_kernel, dim3(blocks_for(kGemmFloats, 256), 2), dim3(256), 0, s, (const float*)tr->params,
                     tr->gemmw);
  if (tr->fwd_x3) {
    hipLaunchKernelGGL(pack_x3_kernel, dim3(blocks_for(kX3Elems, 256), 2), dim3(256), 0, s, (const float*)tr->params,
                       tr->x3);
    hipLaunchKernelGGL(pack_bwd_x3_kernel, dim3(blocks_for(kBwdX3Elems, 256), 2), dim3(256), 0, s,
                       (const float*)tr->params, tr->bx3);
  }
  return hipGetLastError();
}

constexpr int kSqBlocks = 256;

struct DeviceGuardT {
  int prev = -1;
  explicit DeviceGuardT(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
    else prev = -1;
  }
  ~DeviceGuardT() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int grow_buf(float*& p, size_t& cap, size_t need, const char* what) {
  if (need <= cap) return NERF_OK;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  const size_t n = need + need / 8;
  hipError_t e = hipMalloc((void**)&p, n * sizeof(float));
  if (e != hipSuccess) return set_error(NERF_E_HIP, "hipMalloc %s (%zu bytes): %s", what, n * sizeof(float), hipGetErrorString(e));
  cap = n;
  return NERF_OK;
}

inline size_t al64(size_t x) { return (x + 63) / 64 * 64; }

// Per-net activation arrays inside the workspace.
struct Acts {
  float *pe, *dpe, *h[8], *hc, *rgbs, *dpre, *tb, *dhc, *dz[8];
  unsigned* mb[8];   // ReLU bits of h[l]: [P][8] words
};

size_t acts_floats(long P) {
  const size_t p = size_t(P);
  return al64(p * kPeLd) + al64(p * kDpeLd) + 8 * al64(p * kH) + al64(p * kHeadLd) + 2 * al64(p * 4) + al64(p) +
         al64(p * kHeadLd) + 8 * al64(p * kH) + 8 * al64(p * (kH / 32));
}

size_t head_floats(int n_rays, int n_coarse) {
  return al64(size_t(n_rays) * 9) + al64(size_t(n_rays) * n_coarse) + al64(size_t(n_rays) * 2);
}

Acts carve_acts(float* base, long P) {
  const size_t p = size_t(P);
  Acts a;
  float* q = base;
  auto take = [&](size_t n) {
    float* r = q;
    q += al64(n);
    return r;
  };
  a.pe = take(p * kPeLd);
  a.dpe = take(p * kDpeLd);
  for (auto& hh : a.h) hh = take(p * kH);
  a.hc = take(p * kHeadLd);
  a.rgbs = take(p * 4);
  a.dpre = take(p * 4);
  a.tb = take(p);
  a.dhc = take(p * kHeadLd);
  for (auto& d : a.dz) d = take(p * kH);
  for (auto& b : a.mb) b = (unsigned*)take(p * (kH / 32));
  return a;
}

// The four weight-gradient shapes of a NeRFModel (M x N: B's sources)
//   256 x 256: the previous layer's rows; 256 x 319: [layer 3's rows, the position
//   encodings]; 256 x 63: the position encodings; 128 x 283: [layer 7's rows, the direction
//   encodings].  Each runs as one workgroup tile; the host checks the operands fit it.
int wgrad_shape(const GemmArgs& g) {
  const bool two = g.b.w1 < g.N;
  const int W1 = two ? g.b.w1 : round_up(g.N, 4), W2 = two ? round_up(g.N - g.b.w1, 4) : 0;
  auto aligned = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (g.a.ld1 % 4 || g.b.ld1 % 4 || (two && (g.b.ld2 % 4 || W2 > g.b.ld2)) || W1 > g.b.ld1 || g.M > g.a.ld1 ||
      !aligned(g.a.p1) || !aligned(g.b.p1) || (two && !aligned(g.b.p2)))
    return -1;
  if (g.M == 256 && W1 == 256 && W2 == 0) return kW256x256;
  if (g.M == 256 && W1 == 256 && W2 == 64) return kW256x319;
  if (g.M == 256 && W1 == 64 && W2 == 0) return kW256x63;
  if (g.M == 128 && W1 == 256 && W2 == 28) return kW128x283;
  return -1;
}

struct WJob {
  int M, N;
  int splits, k_split;
  size_t off, boff;   // partial and bias-partial offsets in the part buffer
};

WJob plan_wjob(int M, int N, long P, int want, size_t& cursor) {
  WJob j{M, N, 1, 0, 0, 0};
  const int ktiles = int(blocks_for(P, BK));
  const int splits = std::max(1, std::min(want, std::max(1, ktiles / 4)));
  j.k_split = int(blocks_for(ktiles, splits)) * BK;
  j.splits = int(blocks_for(P, j.k_split));
  j.off = cursor;
  cursor += al64(size_t(j.splits) * M * N);
  j.boff = cursor;
  cursor += al64(size_t(j.splits) * M);
  return j;
}

// Workgroups per weight-gradient job of a net, one per CU in all: in proportion to the
// job's time per sample relative to a 256 x 256 layer.  On the split-bf16 MFMA the jobs are
// close to HBM-bound, so the weights sit near their operand bytes per sample (256 x 319
// 1.125, 256 x 63 0.625, 128 x 283 0.80); the values were tuned on MI355X from there
// (tools/train_lab.py, whole-step wall time).  On the fp32 MFMA they were the MFMA times:
// 1.30, 0.34, 0.74.
void wgrad_splits(int (&want)[kMaxWJobs]) {
  double w[kMaxWJobs], total = 0.0;
#ifndef NERF_WG_COST
#define NERF_WG_COST 0.52, 1.16, 0.78
#endif
  const double c[3] = {NERF_WG_COST};
  for (int l = 0; l < 8; ++l) w[l] = l == 0 ? c[0] : l == 4 ? c[1] : 1.0;
  w[8] = c[2];
  for (double x : w) total += x;
  const int cus = current_device_cus();
  int sum = 0;
  double frac[kMaxWJobs];
  for (int i = 0; i < kMaxWJobs; ++i) {
    const double e = cus * w[i] / total;
    sum += (want[i] = std::max(1, int(e)));
    frac[i] = e - int(e);
  }
  while (sum < cus) {                     // leftover CUs to the largest remainders
    int b = 0;
    for (int i = 1; i < kMaxWJobs; ++i)
      if (frac[i] > frac[b]) b = i;
    ++want[b], ++sum, frac[b] = -1.0;
  }
}

double gemm_macs_per_sample() {
  double fwd = 0.0;
  for (int l = 0; l < 8; ++l) fwd += double(kTrunkIn[l]) * kH;
  fwd += double(kHeadK) * kC0 + kH;                       // colour-0 + density
  const double bwd_data = 7.0 * kH * kH + double(kC0 + 1) * kH;
  return 2.0 * fwd + bwd_data;                            // forward, weight grads, data grads
}

// The weight-gradient partials of one net's pass over P samples: the skinny layers' (one
// split per kSkinnyChunk samples) and the nine GEMM jobs'; floats = the buffer size.
constexpr int kSkinnyChunk = 256;   // samples per block of the skinny weight-gradient kernel
struct PartPlan {
  WJob jc1, jd, jl[8], jh;
  size_t floats;
};
PartPlan plan_parts(long P) {
  PartPlan pp;
  size_t cur = 0;
  const int sk_splits = int(blocks_for(P, kSkinnyChunk));
  pp.jc1 = WJob{3, kC0, sk_splits, kSkinnyChunk, 0, 0};
  pp.jd = WJob{1, kH, sk_splits, kSkinnyChunk, 0, 0};
  for (WJob* j : {&pp.jc1, &pp.jd}) {
    j->off = cur;
    cur += al64(size_t(j->splits) * j->M * j->N);
    j->boff = cur;
    cur += al64(size_t(j->splits) * j->M);
  }
  int want[kMaxWJobs];
  wgrad_splits(want);
  for (int l = 7; l >= 0; --l) pp.jl[l] = plan_wjob(kH, kTrunkIn[l], P, want[l], cur);
  pp.jh = plan_wjob(kC0, kHeadK, P, want[8], cur);
  pp.floats = cur;
  return pp;
}

// Forward + backward of one net on P = n_rays * S samples, in its own activation region
// (acts) and partials buffer (part, plan_parts(P).floats); gradients into grads (flat).
int net_pass(nerf_trainer* tr, int net, const float* rays_o, const float* rays_d, const float* target,
             const float* z, int z_stride, int n_rays, int n_total, int S, float* loss_ray, hipStream_t s, int ev0,
             float* acts, float* part) {
  const long P = long(n_rays) * S;
  Acts a = carve_acts(acts, P);
  const float* prm = tr->params + net * kNetFloats;
  const float* gw = tr->gemmw + net * kGemmFloats;
  float* grads = tr->grads + net * kNetFloats;
  auto mark = [&](int i) -> int {
    if (tr->profiling) HIP_TRY(hipEventRecord(tr->ev[ev0 + i], s));
    return NERF_OK;
  };
  int rc;
  hipLaunchKernelGGL(train_encode_kernel, dim3(blocks_for(P, 256)), dim3(256), 0, s, rays_o, rays_d, z, z_stride, S,
                     P, a.pe, a.dpe);
  HIP_TRY(hipGetLastError());
  if ((rc = mark(1)) != NERF_OK) return rc;

  // forward (nerf.py:104-121)
  {
    FwdOut fo;
    for (int l = 0; l < 8; ++l) fo.h[l] = a.h[l], fo.mb[l] = a.mb[l];
    fo.hc = a.hc;
    fo.rgbs = (f32x4*)a.rgbs;
    SampleSrc src{rays_o, rays_d, z, z_stride, S, nullptr, nullptr};
    if (tr->fwd_x3) {
      X3TrainOut xo;
      for (int l = 0; l < 8; ++l) xo.h[l] = a.h[l], xo.mb[l] = a.mb[l];
      xo.hc = a.hc;
      xo.rgbs = a.rgbs;
      HIP_TRY(launch_mlp_bf16x3_train(tr->x3 + net * kX3NetElems, gw + kPrmBlob, src, P, xo, s));
    } else {
      hipLaunchKernelGGL(train_fwd_kernel, dim3(blocks_for(P, 4 * kSamplesPerWave)), dim3(256), 0, s,
                         (const f32x4*)(gw + kF32Blob), gw + kPrmBlob, src, P, fo);
      HIP_TRY(hipGetLastError());
    }
  }
  if ((rc = mark(2)) != NERF_OK) return rc;
  // volume render + loss, their backward (rendering.py:102-143, trainer.py:117-126)
  const float gnorm = float(2.0 / (3.0 * n_total));   // mse_loss backward over the whole step's rays
  hipLaunchKernelGGL(render_train_kernel, dim3(blocks_for(n_rays, 4)), dim3(256), 0, s, (const f32x4*)a.rgbs, z,
                     z_stride, rays_d, target, n_rays, S, gnorm, a.tb, (f32x4*)a.dpre, loss_ray);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(head_bwd_kernel, dim3(blocks_for(P * (kHeadLd / 4), 256)), dim3(256), 0, s, a.hc,
                     (const f32x4*)a.dpre, prm, P, a.dhc);
  HIP_TRY(hipGetLastError());
  if ((rc = mark(3)) != NERF_OK) return rc;

  // backward GEMMs; weight gradients as split partials
  const PartPlan pp = plan_parts(P);
  const WJob &jc1 = pp.jc1, &jd = pp.jd, &jh = pp.jh;
  const WJob* jl = pp.jl;
  hipLaunchKernelGGL(skinny_wgrad_kernel, dim3(jc1.splits), dim3(512), 0, s, (const f32x4*)a.dpre,
                     (const float*)a.hc, kHeadLd, (const float*)a.h[7], P, kSkinnyChunk, part + jc1.off,
                     part + jc1.boff, part + jd.off, part + jd.boff);
  HIP_TRY(hipGetLastError());
  {
    // dZ_7 .. dZ_0 in one launch (the head's and layers 7..1's data gradients with the ReLU bits)
    if (tr->fwd_x3 && NERF_TRAIN_BWD_X3) {
      BwdX3Io io;
      io.dhc = a.dhc;
      io.wsig = gw + kPrmBlob + kSigW;
      for (int l = 0; l < 8; ++l) io.mb[l] = a.mb[l], io.dz[l] = a.dz[l];
      HIP_TRY(launch_train_bwd_x3(tr->bx3 + net * kBwdX3NetElems, P, io, s));
    } else {
      BwdIo io;
      io.dhc = a.dhc;
      for (int l = 0; l < 8; ++l) io.mb[l] = a.mb[l], io.dz[l] = a.dz[l];
      hipLaunchKernelGGL(train_bwd_kernel, dim3(blocks_for(P, 4 * kSamplesPerWave)), dim3(256), 0, s,
                         (const f32x4*)(gw + kBwdBlob), P, io);
      HIP_TRY(hipGetLastError());
    }
  }
  if ((rc = mark(4)) != NERF_OK) return rc;
  {
    // every weight-gradient GEMM of the net in one launch
    WGroup grp{};
    int nwg = 0;
    auto add = [&](const WJob& j, const float* A, int lda, Src2 B) -> bool {
      GemmArgs& g = grp.g[grp.n];
      g.M = j.M, g.N = j.N, g.K = int(P);
      g.a = Src2{A, nullptr, lda, 0, 0x7fffffff};
      g.b = B;
      g.c = part + j.off, g.ldc = j.N;
      g.bias_part = part + j.boff;
      g.k_split = j.k_split;
      g.c_split = long(j.M) * j.N;
      if ((grp.shape[grp.n] = wgrad_shape(g)) < 0) return false;
      grp.first[grp.n++] = nwg;
      nwg += j.splits;
      return true;
    };
    bool ok = add(jh, a.dhc, kHeadLd, Src2{a.h[7], a.dpe, kH, kDpeLd, kH});
    for (int l = 7; l >= 0; --l) {
      Src2 X;
      if (l == 0) X = Src2{a.pe, nullptr, kPeLd, 0, 0x7fffffff};
      else if (l == 4) X = Src2{a.h[3], a.pe, kH, kPeLd, kH};
      else X = Src2{a.h[l - 1], nullptr, kH, 0, 0x7fffffff};
      ok = ok && add(jl[l], a.dz[l], kH, X);
    }
    if (!ok) return set_error(NERF_E_INVALID, "weight-gradient operands do not fit a kernel shape");
    grp.first[grp.n] = nwg;
    hipLaunchKernelGGL(wgrad_group_kernel, dim3(nwg), dim3(512), 0, s, grp);
    HIP_TRY(hipGetLastError());
  }
  if ((rc = mark(5)) != NERF_OK) return rc;

  // partials -> flat gradients
  RedJobs jobs{};
  auto job = [&](int i, const WJob& j, int r1, long w0, long b0, int ld0, int nw0, long w1, long b1, int ld1,
                 int nw1) {
    jobs.j[i] = RedJob{part + j.off, part + j.boff, j.splits, j.M, j.N, r1, w0, b0, ld0, nw0, w1, b1, ld1, nw1};
  };
  long maxe = 0;
  for (int l = 0; l < 8; ++l) {
    job(l, jl[l], kH, w_off(l), b_off(l), kTrunkIn[l], kTrunkIn[l], 0, 0, 0, 0);
    maxe = std::max(maxe, long(jl[l].M) * jl[l].N + jl[l].M);
  }
  job(8, jh, kC0, kFC0W, kFC0B, kHeadK, kHeadK, 0, 0, 0, 0);
  job(9, jd, 1, kFDensW, kFDensB, kH, kH, 0, 0, 0, 0);
  job(10, jc1, 3, kFC1W, kFC1B, kC0, kC0, 0, 0, 0, 0);
  maxe = std::max(maxe, long(jh.M) * jh.N + jh.M);
  hipLaunchKernelGGL(reduce_grads_kernel, dim3(blocks_for(maxe, 256), 9), dim3(256), 0, s, jobs, grads);
  HIP_TRY(hipGetLastError());
  // the skinny layers' partials (one split per 256 samples): a workgroup per element
  hipLaunchKernelGGL(reduce_wide_kernel, dim3(std::max(long(jd.M) * jd.N + jd.M, long(jc1.M) * jc1.N + jc1.M), 2),
                     dim3(256), 0, s, jobs, 9, grads);
  HIP_TRY(hipGetLastError());
  tr->gemm_flops += 2.0 * gemm_macs_per_sample() * double(P);
  return NERF_OK;
}

int update_impl(nerf_trainer* tr, hipStream_t s) {
  double* sq = (double*)(tr->scal + 4);
  const long n = 2 * kNetFloats;
  const bool clip = tr->cfg.grad_clip > 0.0;
  if (clip) {
    hipLaunchKernelGGL(sumsq_kernel, dim3(kSqBlocks), dim3(256), 0, s, tr->grads, n, sq);
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, s, (const float*)nullptr, 0, 1,
                     clip ? (const double*)sq : (const double*)nullptr, kSqBlocks, float(tr->cfg.grad_clip),
                     (float*)nullptr, tr->scal);
  HIP_TRY(hipGetLastError());
  // torch.optim.Adam step scalars (adam.py, _single_tensor_adam): python floats
  const double step = double(tr->steps + 1);
  const double bc1 = 1.0 - std::pow(tr->cfg.beta1, step);
  const double bc2 = 1.0 - std::pow(tr->cfg.beta2, step);
  AdamArgs aa;
  aa.one_minus_b1 = float(1.0 - tr->cfg.beta1);
  aa.b2 = float(tr->cfg.beta2);
  aa.one_minus_b2 = float(1.0 - tr->cfg.beta2);
  aa.wd = float(tr->cfg.weight_decay);
  aa.neg_step_size = float(-(tr->lr / bc1));
  aa.bc2_sqrt = float(std::pow(bc2, 0.5));
  aa.eps = float(tr->cfg.eps);
  hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, tr->params, tr->grads, tr->m, tr->v, n,
                     (const float*)tr->scal, aa);
  HIP_TRY(hipGetLastError());
  HIP_TRY(pack_operands(tr, s));
  tr->steps += 1;
  tr->lr = tr->lr * tr->cfg.lr_gamma;   // ExponentialLR.step: lr * gamma
  return NERF_OK;
}

size_t param_offset(int i) { return size_t(tensor_desc(i).off); }
size_t param_count(int i) { return size_t(tensor_desc(i).rows) * size_t(tensor_desc(i).cols); }

}  // namespace

extern "C" {

int nerf_trainer_create(int device, const nerf_train_config* cfg, const float* const* coarse,
                        const float* const* fine, int n_params, nerf_trainer** out) {
  if (!out) return set_error(NERF_E_INVALID, "null out pointer");
  *out = nullptr;
  if (!cfg || !coarse || !fine) return set_error(NERF_E_INVALID, "nerf_trainer_create: null argument");
  if (n_params != NERF_N_PARAMS) return set_error(NERF_E_INVALID, "expected %d parameter tensors, got %d", NERF_N_PARAMS, n_params);
  if (cfg->n_coarse < 2 || cfg->n_coarse > 1024 || cfg->n_fine < 2 || cfg->n_fine > 1024)
    return set_error(NERF_E_INVALID, "nerf_trainer_create: sample counts %d / %d (2..1024)", cfg->n_coarse, cfg->n_fine);
  if (!(cfg->lr >= 0.0) || !(cfg->beta1 >= 0.0 && cfg->beta1 < 1.0) || !(cfg->beta2 >= 0.0 && cfg->beta2 < 1.0) ||
      !(cfg->eps >= 0.0) || !(cfg->weight_decay >= 0.0))
    return set_error(NERF_E_INVALID, "nerf_trainer_create: bad optimizer settings");
  for (int i = 0; i < NERF_N_PARAMS; ++i)
    if (!coarse[i] || !fine[i]) return set_error(NERF_E_INVALID, "nerf_trainer_create: null tensor %d", i);
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd)
    return set_error(NERF_E_NO_DEVICE, "no HIP device %d (count %d)", device, nd);
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_error(NERF_E_NO_DEVICE, "device %d is %s; this library is built for gfx950 (MI355X)", device,
                     prop.gcnArchName);
  DeviceGuardT dg(device);
  nerf_trainer* tr = new nerf_trainer();
  tr->device = device;
  tr->cfg = *cfg;
  tr->lr = cfg->lr;
  auto fail = [&](int rc) {
    nerf_trainer_destroy(tr);
    return rc;
  };
  const size_t bytes = sizeof(float) * 2 * kNetFloats;
  for (float** p : {&tr->params, &tr->own_grads, &tr->m, &tr->v})
    if (hipMalloc((void**)p, bytes) != hipSuccess) return fail(set_error(NERF_E_HIP, "hipMalloc trainer state"));
  tr->grads = tr->own_grads;
  if (hipMalloc((void**)&tr->gemmw, sizeof(float) * 2 * kGemmFloats) != hipSuccess ||
      hipMalloc((void**)&tr->x3, sizeof(unsigned short) * 2 * kX3NetElems) != hipSuccess ||
      hipMemset(tr->x3, 0, sizeof(unsigned short) * 2 * kX3NetElems) != hipSuccess ||
      hipMalloc((void**)&tr->bx3, sizeof(unsigned short) * 2 * kBwdX3NetElems) != hipSuccess ||
      hipMalloc((void**)&tr->ztab, sizeof(float) * 2048) != hipSuccess ||
      hipMalloc((void**)&tr->scal, sizeof(float) * (4 + 2 * kSqBlocks)) != hipSuccess ||
      hipMalloc((void**)&tr->bad, sizeof(int)) != hipSuccess)
    return fail(set_error(NERF_E_HIP, "hipMalloc trainer buffers"));
  std::vector<float> host(2 * kNetFloats);
  for (int net = 0; net < 2; ++net) {
    const float* const* src = net ? fine : coarse;
    for (int i = 0; i < NERF_N_PARAMS; ++i)
      std::memcpy(host.data() + net * kNetFloats + param_offset(i), src[i], sizeof(float) * param_count(i));
  }
  if (hipMemcpy(tr->params, host.data(), bytes, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(tr->grads, 0, bytes) != hipSuccess || hipMemset(tr->m, 0, bytes) != hipSuccess ||
      hipMemset(tr->v, 0, bytes) != hipSuccess || hipMemset(tr->bad, 0, sizeof(int)) != hipSuccess)
    return fail(set_error(NERF_E_HIP, "trainer upload failed"));
  // uniform depth tables z = near*(1-t) + far*t over torch.linspace(0, 1, n)
  // (rendering.py:37-38): t is computed here as torch's CPU linspace does for
  // these sizes (checked against torch by tests/test_host_layout.py)
  std::vector<float> zt(2048, 0.0f), tv;
  for (int net = 0; net < 2; ++net) {
    const int n = net ? cfg->n_fine : cfg->n_coarse;
    tv.assign(n, 0.0f);
    nerf_linspace01(n, tv.data());
    nerf_uniform_z(tv.data(), n, cfg->near_, cfg->far_, zt.data() + 1024 * net);
  }
  if (hipMemcpy(tr->ztab, zt.data(), sizeof(float) * 2048, hipMemcpyHostToDevice) != hipSuccess)
    return fail(set_error(NERF_E_HIP, "trainer z upload failed"));
  for (auto& e : tr->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(set_error(NERF_E_HIP, "hipEventCreate"));
  if (hipEventCreateWithFlags(&tr->done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&tr->fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&tr->join, hipEventDisableTiming) != hipSuccess ||
      hipStreamCreateWithFlags(&tr->side, hipStreamNonBlocking) != hipSuccess)
    return fail(set_error(NERF_E_HIP, "trainer events / stream"));
  if (pack_operands(tr, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return fail(set_error(NERF_E_HIP, "trainer relayout failed"));
  *out = tr;
  return NERF_OK;
}

void nerf_trainer_destroy(nerf_trainer* tr) {
  if (!tr) return;
  DeviceGuardT dg(tr->device);
  (void)hipDeviceSynchronize();
  for (float* p : {tr->params, tr->own_grads, tr->m, tr->v, tr->gemmw, tr->ztab, tr->scal, tr->ws, tr->part})
    if (p) (void)hipFree(p);
  if (tr->bad) (void)hipFree(tr->bad);
  if (tr->x3) (void)hipFree(tr->x3);
  if (tr->bx3) (void)hipFree(tr->bx3);
  for (auto& e : tr->ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : {tr->done, tr->fork, tr->join})
    if (e) (void)hipEventDestroy(e);
  if (tr->side) (void)hipStreamDestroy(tr->side);
  delete tr;
}

}  // extern "C"

namespace {

// A call on a different stream than the previous call's waits for that call's work.
int order_after_last(nerf_trainer* tr, hipStream_t s) {
  if (tr->pending && s != tr->last_stream) HIP_TRY(hipStreamWaitEvent(s, tr->done, 0));
  return NERF_OK;
}
int record_done(nerf_trainer* tr, hipStream_t s) {
  HIP_TRY(hipEventRecord(tr->done, s));
  tr->last_stream = s;
  tr->pending = true;
  return NERF_OK;
}

int train_impl(nerf_trainer* tr, const float* image, int height, int width, float focal, const float* c2w,
               const int32_t* select, int n_rays, int n_total, const float* t_rand, bool update, float* loss_out,
               void* stream) {
  if (!tr) return set_error(NERF_E_INVALID, "null trainer");
  if (n_total < n_rays) return set_error(NERF_E_INVALID, "nerf_train: n_rays_total %d < n_rays %d", n_total, n_rays);
  if (!image || !c2w || !select || !t_rand) return set_error(NERF_E_INVALID, "nerf_train_step: null argument");
  if (height <= 0 || width <= 0 || n_rays <= 0 || long(height) * width > 0x7fffffffL)
    return set_error(NERF_E_INVALID, "nerf_train_step: bad sizes %dx%d, %d rays", height, width, n_rays);
  if (!(focal > 0.0f)) return set_error(NERF_E_INVALID, "nerf_train_step: focal must be positive");
  const int Smax = std::max(tr->cfg.n_coarse, tr->cfg.n_fine);
  if (long(n_rays) * Smax > 0x7fffffffL / 2) return set_error(NERF_E_INVALID, "nerf_train_step: too many samples");
  DeviceGuardT dg(tr->device);
  hipStream_t s = (hipStream_t)stream;
  const long Pc = long(n_rays) * tr->cfg.n_coarse, Pf = long(n_rays) * tr->cfg.n_fine;
  // workspace: rays_o, rays_d, targets [n_rays][3] each | coarse z [n_rays][n_coarse] |
  // per-ray squared errors [2][n_rays] | the coarse net's activations | the fine net's;
  // partials: the coarse net's | the fine net's (both nets' passes may run at once)
  const size_t head = head_floats(n_rays, tr->cfg.n_coarse);
  const size_t acts_c = acts_floats(Pc), parts_c = plan_parts(Pc).floats;
  int rc;
  if ((rc = order_after_last(tr, s)) != NERF_OK) return rc;
  if ((rc = grow_buf(tr->ws, tr->ws_cap, head + acts_c + acts_floats(Pf) + 64, "training workspace")) != NERF_OK ||
      (rc = grow_buf(tr->part, tr->part_cap, parts_c + plan_parts(Pf).floats, "gradient partials")) != NERF_OK)
    return rc;
  float* rays_o = tr->ws;
  float* rays_d = rays_o + 3 * size_t(n_rays);
  float* target = rays_d + 3 * size_t(n_rays);
  float* zc = tr->ws + al64(size_t(n_rays) * 9);
  float* loss_ray = zc + al64(size_t(n_rays) * tr->cfg.n_coarse);
  tr->have_times = false;
  tr->gemm_flops = 0.0;
  auto mark = [&](int i) -> int {
    if (tr->profiling) HIP_TRY(hipEventRecord(tr->ev[i], s));
    return NERF_OK;
  };
  if ((rc = mark(0)) != NERF_OK) return rc;
  Pose pose;
  for (int c = 0; c < 3; ++c) {
    for (int j = 0; j < 3; ++j) pose.r[3 * c + j] = c2w[4 * c + j];
    pose.t[c] = c2w[4 * c + 3];
  }
  hipLaunchKernelGGL(train_rays_kernel, dim3(blocks_for(n_rays, 256)), dim3(256), 0, s, pose, width, height * width,
                     float(width * 0.5), float(height * 0.5), focal, (const int*)select, n_rays, image, rays_o, rays_d,
                     target, tr->bad);
  HIP_TRY(hipGetLastError());
  // coarse samples stratified with the injected draw (rendering.py:42-47)
  HIP_TRY(launch_sample(tr->ztab, t_rand, n_rays, tr->cfg.n_coarse, nullptr, nullptr, zc, nullptr, s));
  // the two nets' passes: concurrently (coarse on the side stream), or one after the other
  // on the caller's stream when profiling (the stage events time one pass at a time)
  const bool concurrent = !tr->profiling;
  hipStream_t sc = s;
  if (concurrent) {
    HIP_TRY(hipEventRecord(tr->fork, s));
    HIP_TRY(hipStreamWaitEvent(tr->side, tr->fork, 0));
    sc = tr->side;
  }
  if ((rc = net_pass(tr, 0, rays_o, rays_d, target, zc, tr->cfg.n_coarse, n_rays, n_total, tr->cfg.n_coarse, loss_ray,
                     sc, 0, tr->ws + head, tr->part)) != NERF_OK)
    return rc;
  if (concurrent) HIP_TRY(hipEventRecord(tr->join, sc));
  if ((rc = mark(6)) != NERF_OK) return rc;
  if ((rc = net_pass(tr, 1, rays_o, rays_d, target, tr->ztab + 1024, 0, n_rays, n_total, tr->cfg.n_fine,
                     loss_ray + n_rays, s, 6, tr->ws + head + acts_c, tr->part + parts_c)) != NERF_OK)
    return rc;
  if (concurrent) HIP_TRY(hipStreamWaitEvent(s, tr->join, 0));
  if ((rc = mark(12)) != NERF_OK) return rc;
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, s, (const float*)loss_ray, n_rays, n_total,
                     (const double*)nullptr, 0, 0.0f, loss_out, (float*)nullptr);
  HIP_TRY(hipGetLastError());
  if (update && (rc = update_impl(tr, s)) != NERF_OK) return rc;
  if ((rc = mark(13)) != NERF_OK) return rc;
  tr->have_times = tr->profiling;
  return record_done(tr, s);
}

}  // namespace

extern "C" {

int nerf_train_step(nerf_trainer* tr, const float* image, int height, int width, float focal, const float* c2w,
                    const int32_t* select, int n_rays, const float* t_rand, int flags, float* loss_out, void* stream) {
  return train_impl(tr, image, height, width, focal, c2w, select, n_rays, n_rays, t_rand,
                    !(flags & NERF_TRAIN_NO_UPDATE), loss_out, stream);
}

int nerf_train_backward(nerf_trainer* tr, const float* image, int height, int width, float focal, const float* c2w,
                        const int32_t* select, int n_rays, int n_rays_total, const float* t_rand, float* loss_out,
                        void* stream) {
  return train_impl(tr, image, height, width, focal, c2w, select, n_rays, n_rays_total, t_rand, false, loss_out,
                    stream);
}

int nerf_trainer_set_grad_buffer(nerf_trainer* tr, float* grads_dev) {
  if (!tr) return set_error(NERF_E_INVALID, "null trainer");
  float* next = grads_dev ? grads_dev : tr->own_grads;
  if (next == tr->grads) return NERF_OK;
  DeviceGuardT dg(tr->device);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(next, tr->grads, sizeof(float) * 2 * kNetFloats, hipMemcpyDeviceToDevice));
  tr->grads = next;
  return NERF_OK;
}

int nerf_trainer_update(nerf_trainer* tr, void* stream) {
  if (!tr) return set_error(NERF_E_INVALID, "null trainer");
  DeviceGuardT dg(tr->device);
  const hipStream_t s = (hipStream_t)stream;
  int rc;
  if ((rc = order_after_last(tr, s)) != NERF_OK || (rc = update_impl(tr, s)) != NERF_OK) return rc;
  return record_done(tr, s);
}

int nerf_trainer_read(nerf_trainer* tr, int what, int net, float* const* host_out, int n_params) {
  if (!tr || !host_out) return set_error(NERF_E_INVALID, "nerf_trainer_read: null argument");
  if (net != NERF_NET_COARSE && net != NERF_NET_FINE) return set_error(NERF_E_INVALID, "bad net %d", net);
  if (n_params != NERF_N_PARAMS) return set_error(NERF_E_INVALID, "expected %d tensors", NERF_N_PARAMS);
  const float* src = what == NERF_TR_PARAMS ? tr->params : what == NERF_TR_GRADS ? tr->grads
                   : what == NERF_TR_EXP_AVG ? tr->m : what == NERF_TR_EXP_AVG_SQ ? tr->v : nullptr;
  if (!src) return set_error(NERF_E_INVALID, "nerf_trainer_read: bad state %d", what);
  DeviceGuardT dg(tr->device);
  HIP_TRY(hipDeviceSynchronize());
  int bad = 0;
  HIP_TRY(hipMemcpy(&bad, tr->bad, sizeof(int), hipMemcpyDeviceToHost));
  if (bad) return set_error(NERF_E_INVALID, "a train_step's select held an index outside the image");
  std::vector<float> host(kNetFloats);
  HIP_TRY(hipMemcpy(host.data(), src + net * kNetFloats, sizeof(float) * kNetFloats, hipMemcpyDeviceToHost));
  for (int i = 0; i < NERF_N_PARAMS; ++i) {
    if (!host_out[i]) return set_error(NERF_E_INVALID, "nerf_trainer_read: null buffer %d", i);
    std::memcpy(host_out[i], host.data() + param_offset(i), sizeof(float) * param_count(i));
  }
  return NERF_OK;
}

int nerf_trainer_write_grads(nerf_trainer* tr, int net, const float* const* grads, int n_params) {
  if (!tr || !grads) return set_error(NERF_E_INVALID, "nerf_trainer_write_grads: null argument");
  if (net != NERF_NET_COARSE && net != NERF_NET_FINE) return set_error(NERF_E_INVALID, "bad net %d", net);
  if (n_params != NERF_N_PARAMS) return set_error(NERF_E_INVALID, "expected %d tensors", NERF_N_PARAMS);
  std::vector<float> host(kNetFloats);
  for (int i = 0; i < NERF_N_PARAMS; ++i) {
    if (!grads[i]) return set_error(NERF_E_INVALID, "nerf_trainer_write_grads: null tensor %d", i);
    std::memcpy(host.data() + param_offset(i), grads[i], sizeof(float) * param_count(i));
  }
  DeviceGuardT dg(tr->device);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(tr->grads + net * kNetFloats, host.data(), sizeof(float) * kNetFloats, hipMemcpyHostToDevice));
  return NERF_OK;
}

int nerf_trainer_write(nerf_trainer* tr, int what, int net, const float* const* host_in, int n_params) {
  if (!tr || !host_in) return set_error(NERF_E_INVALID, "nerf_trainer_write: null argument");
  if (net != NERF_NET_COARSE && net != NERF_NET_FINE) return set_error(NERF_E_INVALID, "bad net %d", net);
  if (n_params != NERF_N_PARAMS) return set_error(NERF_E_INVALID, "expected %d tensors", NERF_N_PARAMS);
  float* dst = what == NERF_TR_PARAMS ? tr->params : what == NERF_TR_GRADS ? tr->grads
             : what == NERF_TR_EXP_AVG ? tr->m : what == NERF_TR_EXP_AVG_SQ ? tr->v : nullptr;
  if (!dst) return set_error(NERF_E_INVALID, "nerf_trainer_write: bad state %d", what);
  std::vector<float> host(kNetFloats);
  for (int i = 0; i < NERF_N_PARAMS; ++i) {
    if (!host_in[i]) return set_error(NERF_E_INVALID, "nerf_trainer_write: null tensor %d", i);
    std::memcpy(host.data() + param_offset(i), host_in[i], sizeof(float) * param_count(i));
  }
  DeviceGuardT dg(tr->device);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(dst + net * kNetFloats, host.data(), sizeof(float) * kNetFloats, hipMemcpyHostToDevice));
  if (what == NERF_TR_PARAMS) {   // the kernels' operand copies of the weights
    HIP_TRY(pack_operands(tr, 0));
    HIP_TRY(hipDeviceSynchronize());
  }
  return NERF_OK;
}

int nerf_trainer_set_schedule(nerf_trainer* tr, long steps, double lr) {
  if (!tr) return set_error(NERF_E_INVALID, "null trainer");
  if (steps < 0 || !(lr >= 0.0)) return set_error(NERF_E_INVALID, "nerf_trainer_set_schedule: steps %ld, lr %g", steps, lr);
  tr->steps = steps;
  tr->lr = lr;
  return NERF_OK;
}

int nerf_trainer_set_precision(nerf_trainer* tr, int precision) {
  if (!tr) return set_error(NERF_E_INVALID, "null trainer");
  if (precision != NERF_FP32 && precision != NERF_BF16X3)
    return set_error(NERF_E_INVALID, "nerf_trainer_set_precision: %d (NERF_FP32 or NERF_BF16X3)", precision);
  DeviceGuardT dg(tr->device);
  HIP_TRY(hipDeviceSynchronize());
  tr->fwd_x3 = precision == NERF_BF16X3;
  HIP_TRY(pack_operands(tr, 0));
  HIP_TRY(hipDeviceSynchronize());
  return NERF_OK;
}

double nerf_trainer_lr(const nerf_trainer* tr) { return tr ? tr->lr : 0.0; }
long nerf_trainer_steps(const nerf_trainer* tr) { return tr ? tr->steps : 0; }
double nerf_trainer_gemm_flops(const nerf_trainer* tr) { return tr ? tr->gemm_flops : 0.0; }

int nerf_trainer_set_profiling(nerf_trainer* tr, int enable) {
  if (!tr) return set_error(NERF_E_INVALID, "null trainer");
  tr->profiling = enable != 0;
  return NERF_OK;
}

int nerf_trainer_stage_ms(nerf_trainer* tr, float* ms_out) {
  if (!tr || !ms_out) return set_error(NERF_E_INVALID, "null argument");
  for (int i = 0; i < NERF_TRAIN_N_STAGES; ++i) ms_out[i] = 0.0f;
  if (!tr->have_times) return NERF_OK;
  DeviceGuardT dg(tr->device);
  HIP_TRY(hipEventSynchronize(tr->ev[13]));
  // event order: 0 | encode c | 1 | fwd c | 2 | render c | 3 | bwd-data c | 4 | wgrad c | 5 | reduce c | 6 |
  //              encode f | 7 | fwd f | 8 | render f | 9 | bwd-data f | 10 | wgrad f | 11 | reduce f | 12 |
  //              update | 13
  static const int stage_of[13] = {0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4, 5, 5};
  for (int i = 0; i < 13; ++i) {
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, tr->ev[i], tr->ev[i + 1]));
    ms_out[stage_of[i]] += ms;
  }
  return NERF_OK;
}

}  // extern "C"
