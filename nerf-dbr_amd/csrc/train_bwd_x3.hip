// The training step's backward-data chain on the split-bf16 MFMA (trainer precision
// NERF_BF16X3; train.hip's train_bwd_kernel is the fp32 form).
//
// Replaces the autograd of NeRFModel.forward's data path (src/models/nerf.py:104-121,
// driven by src/training/trainer.py:117-126): dZ_{l-1} = (W_l^T dZ_l) * bit(H_{l-1}) for the
// colour-0 layer into H_7 and trunk layers 7..1, every dZ row written for the weight
// gradients.  Each product W^T.dZ is split as in mlp_x3.h, A_hi.B_hi + A_hi.B_lo + A_lo.B_hi
// on v_mfma_f32_32x32x16_bf16 with fp32 accumulation (bf16 halves: gradients span more
// binades than fp16 holds), so a layer's error is ~2^-17 relative, the forward split path's.
//
// Structure: mlp_x3.h's, run over the backward layers of train_x3_layout.h -- one wave per
// SIMD, 32 samples per wave, a layer's 8 accumulator tiles issued as 4 quarters, the
// accumulators of one layer masked, split and kept as the next layer's B fragments, the
// weight stream through a 4-slot LDS ring (NERF_BWD_X3_SLOTS) filled by LDS-DMA (one barrier per 16 KiB chunk,
// the stream running on across persistent tiles).  What differs:
//   * no biases, encodings or heads: the colour-0 layer's inputs are the dZ rows of the
//     head backward (dhc [P][132]), read at the top of the tile; the density row's term
//     w_sigma . dsigma is the accumulators' initial value in the first layer (fp32);
//   * the ReLU of the forward is the mask of the stored bits (v_bfe_i32 of the bit, AND);
//   * each layer's masked accumulators also leave as the fp32 dZ rows [P][256];
//   * a layer's mask words (32 B per sample, 1 KiB per wave) arrive by one LDS-DMA piece
//     issued at the previous layer's first seam, so the seams' counted vmcnt covers them and
//     no compiler-counted global load waits for the weight stream inside the loop.
#include "nerf_asm.h"
#include "nerf_device.h"
#include "nerf_internal.h"
#include "train_x3_layout.h"

namespace nerf {
namespace {

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kSamplesPerBlock = kWaves * kSamplesPerWave;            // 128
constexpr int kUnits = kBwdX3Units;                                   // 480
constexpr int kUnitB = kBwdX3UnitBytes;                               // hi 2 KiB, lo 2 KiB
constexpr int kChunkUnits = kBwdX3ChunkUnits;
constexpr int kChunkB = kChunkUnits * kUnitB;                         // 16 KiB
constexpr int kTotalChunks = kUnits / kChunkUnits;                    // 120
// 4 ring slots, each chunk staged 2 seams before it is needed: a seam's counted wait then
// leaves the row stores of two chunk periods in flight (kVm); 3 slots left one
#ifndef NERF_BWD_X3_SLOTS
#define NERF_BWD_X3_SLOTS 4
#endif
constexpr int kSlots = NERF_BWD_X3_SLOTS;
constexpr int kPf = 3;                                                // fragment prefetch distance (units)
constexpr int kRing = kPf + 1;
constexpr int kGldsPerStage = kChunkB / (kThreads * 16);              // 4 pieces per wave per chunk
static_assert(kTotalChunks % kSlots == 0, "the stream runs on into the next tile: chunk g always uses slot g % kSlots");
static_assert(kSlots * kChunkB <= 65536, "ring offsets fit the ds_read offset field");
constexpr int kLdsMaskOff = kSlots * kChunkB;                         // [wave][buffer 2][1 KiB]
// dZ row staging: a tile pair's masked values, [sample 32][64 floats] per wave, rows padded
// to 272 B so the 16-B writes of a lane-half hit distinct banks
constexpr int kRowPitch = 272;
constexpr int kLdsRowOff = kLdsMaskOff + kWaves * 2 * 1024;
constexpr int kLdsRowWaveB = kSamplesPerWave * kRowPitch;              // 8.5 KiB
constexpr int kLdsBytes = kLdsRowOff + kWaves * kLdsRowWaveB;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
constexpr int kHeadLd = 132;                                          // dhc rows: colour-0 (128), density
constexpr int kRows = 256;                                            // dZ row length (floats)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

NL_HD bool is_seam(int n) { return (n + kPf) % kChunkUnits == 0 && n + kPf < kUnits && n + kPf != 0; }
// the first seam inside backward layer b (where the next layer's mask words are requested)
NL_HD int first_seam_unit(int b) {
  int n = bwd_x3_unit_base(b);
  while (!is_seam(n)) ++n;
  return n;
}

// Conversion schedule of mlp_x3.h: one dword per unit.
NL_HD int dword_unit_out(int ku, int m) { return ku >= 16 ? 2 + (m * (ku - 2)) / 16 : m / 4; }
NL_HD int dword_unit_in(int m) { return 2 + (m * 10) / 16; }

// Counted seam waits.  Inside the loop a wave issues three kinds of vector-memory op: the
// weight stream's LDS-DMA pieces (at seams), one mask-word piece per layer (after the
// layer's first seam) and its dZ row stores (one per converted dword pair).  vmcnt retires
// them in issue order (CDNA4 counts stores too), so a seam needs only the pieces staged at
// the previous seam: it waits until no more than the ops issued after them -- that interval's
// mask piece and stores -- are outstanding, and a row store gets a whole chunk to complete
// instead of stalling the next seam (vmcnt(0) there made the chain wait for HBM writes).
#ifndef NERF_BWD_X3_ABLATE_NOSTORE
constexpr int kFlushStores = kSamplesPerWave * 256 / (64 * 16);       // 8 row stores per tile pair
#else   // the timing-only build stores no rows: the table must count only what is issued
constexpr int kFlushStores = 0;
#endif
struct VmTable {
  int ops[kUnits];      // vector-memory ops unit body n issues after its seam
  int younger[kUnits];  // at the seam of body n: ops issued since the previous seam's stage
};
constexpr VmTable make_vm_table() {
  VmTable t{};
  for (int n = 0; n < kUnits; ++n) {
    int b = 0;
    while (b + 1 < kBwdX3Layers && bwd_x3_unit_base(b + 1) <= n) ++b;
    const int ku = bwd_x3_ksteps(b), r = n - bwd_x3_unit_base(b), q = r / ku, u = r % ku;
    int c = 0;
    if (b != 0 && q == 0 && u == dword_unit_in(15)) c += kFlushStores;    // the previous layer's tiles 6, 7
    if (q >= 1 && u == dword_unit_out(ku, 15)) c += kFlushStores;          // this layer's tiles 2q-2, 2q-1
    int first = bwd_x3_unit_base(b);
    while (!is_seam(first)) ++first;
    if (b + 1 < kBwdX3Layers && n == first) ++c;                        // the next layer's mask words
    t.ops[n] = c;
  }
  // A tile's stage events: the tile top stages chunk kSlots-2 (chunks below it have landed:
  // the top drains vmcnt), seam j stages chunk j + kSlots - 1; seam k needs chunk k + 1.
  int seams[kUnits] = {};
  int ns = 0;
  for (int n = 0; n < kUnits; ++n)
    if (is_seam(n)) seams[ns++] = n;
  for (int k = 0; k < ns; ++k) {
    const int j = k + 1 - (kSlots - 1);     // the seam that staged chunk k+1 (< 0: the tile top)
    const int from = j < 0 ? 0 : seams[j];  // the bodies after that stage
    // stages issued after it: the seams between; from the top, seams 0..k-1, and the top's own
    // when chunk k+1 had landed before it
    const int stages = j < 0 ? k + (k + 1 < kSlots - 2 ? 1 : 0) : k - j - 1;
    int y = kGldsPerStage * stages;
    for (int m = from; m < seams[k]; ++m) y += t.ops[m];
    t.younger[seams[k]] = y;
  }
  return t;
}
constexpr VmTable kVm = make_vm_table();

struct Ctx {
  const char* blob;
  unsigned lds_base;               // LDS byte address of the ring (lds[0])
  int wave_u, lane, h;
  unsigned ring_addr, mask_addr;   // mask_addr: this wave's 2 x 1 KiB of mask words + (lane & 31) * 32
  unsigned mask_dma;               // LDS byte address of this wave's mask buffers
  unsigned row_w;                  // this lane's sample row in the wave's dZ staging block
  unsigned row_r;                  // the flush's read address: sample lane / 16, piece lane % 16
};

// LDS destinations as integer LDS addresses (a generic char* destination costs a 64-bit
// register pair per piece and a null check on the cast)
__device__ __forceinline__ void stage_chunk(const char* __restrict__ blob, int g, unsigned lds_base, int wave_u,
                                            int lane) {
  const unsigned dst = lds_base + unsigned((g % kSlots) * kChunkB + wave_u * 1024);
#pragma unroll
  for (int i = 0; i < kGldsPerStage; ++i)
    lds_dma_16_s(blob + size_t(g) * kChunkB + i * kThreads * 16, unsigned(wave_u * 1024 + lane * 16),
                 dst + unsigned(i * kThreads * 16));
}

// Seam before the prefetch reaches chunk g+1: the wave's pieces of g+1 landed (counted:
// kVm), the barrier publishes g+1 and frees chunk g+2-kSlots's slot, which takes g+kSlots-1
// (every wave finished reading that chunk: its last unit was consumed before this seam).
__device__ __forceinline__ void seam_before(const Ctx& cx, int n) {
  if (!is_seam(n)) return;
  const int g = (n + kPf) / kChunkUnits - 1;
  wait_vmcnt_exact(kVm.younger[n]);
  compiler_fence();
  __builtin_amdgcn_s_barrier();
  compiler_fence();
  stage_chunk(cx.blob, (g + kSlots - 1) % kTotalChunks, cx.lds_base, cx.wave_u, cx.lane);
}

// Reads of unit n into ring entry n % kRing: A_hi and A_lo of the unit's two tiles.
__device__ __forceinline__ void read_unit(const Ctx& cx, int n, bf16x8 (&ra)[kRing][4]) {
  const int off = ((n / kChunkUnits) % kSlots) * kChunkB + (n % kChunkUnits) * kUnitB;
#pragma unroll
  for (int f = 0; f < 4; ++f) ra[n % kRing][f] = ds_read_b128<bf16x8>(cx.ring_addr, off + f * 1024);
}

// One LDS-DMA piece per wave: the 8 mask words of the wave's 32 samples (lane l: words
// 4(l & 1)..+3 of sample l >> 1, clamped into the array) into buffer `buf`.
__device__ __forceinline__ void request_masks(const Ctx& cx, const unsigned* __restrict__ mb, long p_first,
                                              long n_points, int buf) {
  long s = p_first + (cx.lane >> 1);
  s = s < n_points ? s : n_points - 1;
  lds_dma_16_s(mb, unsigned((s * 8 + 4 * (cx.lane & 1)) * 4), cx.mask_dma + unsigned(buf * 1024));
}
__device__ __forceinline__ void read_masks(const Ctx& cx, int buf, u32x4 (&w)[2]) {
  w[0] = ds_read_b128<u32x4>(cx.mask_addr, buf * 1024);
  w[1] = ds_read_b128<u32x4>(cx.mask_addr, buf * 1024 + 16);
}

__device__ __forceinline__ void split_pair(float a, float b, unsigned& hi, unsigned& lo) {
  hi = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));
  const float ha = __builtin_bit_cast(float, hi << 16), hb = __builtin_bit_cast(float, hi & 0xFFFF0000u);
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{__fsub_rn(a, ha), __fsub_rn(b, hb)}, bf16x2));
}
template <int N>
__device__ __forceinline__ void split8(const float (&v)[N], int o, u32x4& hi, u32x4& lo) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    unsigned h2, l2;
    split_pair(v[o + 2 * d], v[o + 2 * d + 1], h2, l2);
    hi[d] = h2;
    lo[d] = l2;
  }
}

__device__ __forceinline__ f32x16 mfma3(const bf16x8& ahi, const bf16x8& alo, const bf16x8& bhi, const bf16x8& blo,
                                        f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, bhi, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, blo, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo, bhi, acc, 0, 0, 0);
}

// Register r of a tile holds feature 32t + acc_row(r, h); its bit in the tile's word,
// shifted right by 4h (ws), is at (r & 3) + 8 (r >> 2).
__device__ __forceinline__ float masked(float v, unsigned ws, int r) {
  const int m = __builtin_amdgcn_sbfe(int(ws), (r & 3) + 8 * (r >> 2), 1);   // 0 or -1
  return __builtin_bit_cast(float, __builtin_bit_cast(int, v) & m);
}

// Dword pr (registers 2pr, 2pr+1) of output tile t: masked, split into the next layer's
// fragments (k-step 2t + (pr >> 2), dword pr & 3), and -- with the previous dword's pair --
// written as one 16-B piece of the sample's dZ row into the wave's LDS staging block
// (registers 4j..4j+3 are features 32t + 8j + 4h + 0..3; the block holds the tile pair
// t & ~1, t | 1).  flush_rows then stores the block as whole 256-B row segments.
struct Keep {
  float v[2];
};
__device__ __forceinline__ void lds_store16(unsigned addr, f32x4 v) {
  *(__attribute__((address_space(3))) f32x4*)(uintptr_t)addr = v;
}
__device__ __forceinline__ void convert_dword(const f32x16& tile, int t, int pr, unsigned word, const Ctx& cx,
                                              u32x4& fhi, u32x4& flo, Keep& kp, bool split) {
  const unsigned ws = word >> (4 * cx.h);
  const float v0 = masked(tile[2 * pr], ws, 2 * pr), v1 = masked(tile[2 * pr + 1], ws, 2 * pr + 1);
  if (split) {
    unsigned hi, lo;
    split_pair(v0, v1, hi, lo);
    fhi[pr & 3] = hi;
    flo[pr & 3] = lo;
  }
  if (pr & 1) {
#ifndef NERF_BWD_X3_ABLATE_NOSTORE   // timing-only lab build (no dZ rows): what the row stores cost
    lds_store16(cx.row_w + unsigned(((t & 1) * 32 + 8 * (pr >> 1) + 4 * cx.h) * 4), f32x4{kp.v[0], kp.v[1], v0, v1});
#else
    asm volatile("" ::"v"(kp.v[0]), "v"(kp.v[1]), "v"(v0), "v"(v1));
#endif
  } else {
    kp.v[0] = v0;
    kp.v[1] = v1;
  }
}
// The staged tile pair (features f0 .. f0+63 of the wave's 32 samples) to the dZ rows: lane
// l stores 16 B of sample 4i + l / 16, so one instruction writes four whole 256-B segments.
// A sample past the last one is clamped to it (its values equal the last sample's).
__device__ __forceinline__ void flush_rows(const Ctx& cx, float* __restrict__ dz, long p_first, long n_points, int f0) {
#ifndef NERF_BWD_X3_ABLATE_NOSTORE
#pragma unroll
  for (int i = 0; i < kSamplesPerWave / 4; ++i) {
    const f32x4 v = ds_read_b128<f32x4>(cx.row_r, i * 4 * kRowPitch);
    long s = p_first + 4 * i + (cx.lane >> 4);
    s = s < n_points ? s : n_points - 1;
    // non-temporal: the rows are read once, by the weight-gradient GEMMs after this launch
    // (3.2 GB per step, far past L2); streaming stores ran the chain 10 % faster (685 -> 616
    // us per net pass) and the weight gradients 3 % faster
    __builtin_nontemporal_store(v, (f32x4*)(dz + s * kRows + f0 + 4 * (cx.lane & 15)));
  }
#endif
}

struct TileIo {
  long p_first, n_points;   // the wave's first sample, the launch's samples
  float dsig;               // this lane's density gradient (the head backward's row[128])
};

// Backward layer B: reads the previous layer's fragments (ih/il), fills the next's (oh/ol);
// its output is dZ of forward layer 7 - B, masked by bits(H_{7-B}) (words wc), the previous
// layer's tiles 6, 7 by wp.
template <int B>
__device__ __forceinline__ void layer_bwd(f32x16 (&acc)[8], u32x4 (&ih)[16], u32x4 (&il)[16], u32x4 (&oh)[16],
                                          u32x4 (&ol)[16], bf16x8 (&ra)[kRing][4], const Ctx& cx, const BwdX3Io& io,
                                          const TileIo& ti, const u32x4 (&wc)[2], const u32x4 (&wp)[2]) {
  constexpr int KU = bwd_x3_ksteps(B);
  constexpr int N0 = bwd_x3_unit_base(B);
  constexpr bool kConvertPrev = B != 0;
  constexpr bool kSplit = B != kBwdX3Layers - 1;     // the last layer's output feeds nothing
  Keep kp;                                           // a dword pair's values until the next (odd) dword
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int n = N0 + q * KU + u;
      seam_before(cx, n);
      if (B + 1 < kBwdX3Layers && n == first_seam_unit(B))   // the next layer's mask words
        request_masks(cx, io.mb[6 - B], ti.p_first, ti.n_points, (B + 1) & 1);
      if (u == 0) {
#pragma unroll
        for (int o2 = 0; o2 < 2; ++o2) {
          if (B == 0) {   // the density row's term w_sigma[f] * dsigma (nerf.py:114)
            const f32x4* ws = (const f32x4*)(io.wsig + (cx.h * 8 + 2 * q + o2) * 16);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const f32x4 w4 = ws[j];
#pragma unroll
              for (int i = 0; i < 4; ++i) acc[2 * q + o2][4 * j + i] = __fmul_rn(w4[i], ti.dsig);
            }
          } else {
            acc[2 * q + o2] = f32x16{};
          }
        }
      }
      if (n + kPf < kUnits) read_unit(cx, n + kPf, ra);
      wait_lgkm(0);
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8 bhi = __builtin_bit_cast(bf16x8, ih[u]), blo = __builtin_bit_cast(bf16x8, il[u]);
#pragma unroll
      for (int o2 = 0; o2 < 2; ++o2)
        acc[2 * q + o2] = mfma3(ra[n % kRing][o2], ra[n % kRing][2 + o2], bhi, blo, acc[2 * q + o2]);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int t = m >> 3, pr = m & 7;
        if (kConvertPrev && q == 0 && u == dword_unit_in(m)) {
          convert_dword(acc[6 + t], 6 + t, pr, wp[1][2 + t], cx, ih[2 * (6 + t) + (pr >> 2)],
                        il[2 * (6 + t) + (pr >> 2)], kp, true);
          if (m == 15) flush_rows(cx, io.dz[8 - B], ti.p_first, ti.n_points, 192);   // the previous layer's dZ
        }
        if (q >= 1 && u == dword_unit_out(KU, m)) {
          const int tt = 2 * q - 2 + t;
          convert_dword(acc[tt], tt, pr, wc[tt >> 2][tt & 3], cx, oh[2 * tt + (pr >> 2)], ol[2 * tt + (pr >> 2)], kp,
                        kSplit);
          if (m == 15) flush_rows(cx, io.dz[7 - B], ti.p_first, ti.n_points, 64 * (q - 1));
        }
      }
    }
  }
}

__global__ __launch_bounds__(kThreads, 1) void train_bwd_x3_kernel(const char* __restrict__ blob, long n_points,
                                                                   BwdX3Io io) {
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  const int lane = threadIdx.x & 63;
  const int wave_u = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5;
  const unsigned base = lds_addr(lds);
  const unsigned rows = base + kLdsRowOff + wave_u * kLdsRowWaveB;
  const Ctx cx0{blob, base, wave_u, lane, h, base + lane * 16,
                base + kLdsMaskOff + wave_u * 2048 + (lane & 31) * 32, base + kLdsMaskOff + wave_u * 2048,
                rows + (lane & 31) * kRowPitch, rows + (lane >> 4) * kRowPitch + (lane & 15) * 16};
  const long n_tiles = (n_points + kSamplesPerBlock - 1) / kSamplesPerBlock;

#pragma unroll
  for (int g = 0; g < kSlots - 2; ++g) stage_chunk(blob, g, base, wave_u, lane);

#pragma unroll 1
  for (long tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    Ctx cx = cx0;
    asm volatile("" : "+s"(cx.blob));   // keep the 120 chunk addresses out of SGPRs across tiles
    TileIo ti;
    ti.n_points = n_points;
    ti.p_first = (tile * kWaves + wave_u) * kSamplesPerWave;
    const long p = ti.p_first + (lane & 31);
    const long pc = p < n_points ? p : n_points - 1;
    // the colour-0 layer's inputs: the head backward's dZ rows, in the B fragments' k order
    // (k-step u, half h: features 16u + 4h + 0..3 and 16u + 8 + 4h + 0..3)
    u32x4 aH[16], aL[16], bH[16], bL[16];
    {
      const float* row = io.dhc + pc * kHeadLd;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const f32x4 x0 = *(const f32x4*)(row + 16 * u + 4 * h), x1 = *(const f32x4*)(row + 16 * u + 8 + 4 * h);
        const float v[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
        split8(v, 0, bH[u], bL[u]);
      }
      ti.dsig = row[128];
    }
    request_masks(cx, io.mb[7], ti.p_first, n_points, 0);
    // the tile's first seam: chunks 0 .. kSlots-3 (staged by the last tile's seams, or the
    // prologue), the mask words and the last tile's row stores landed; chunk kSlots-2 starts
    // into its slot
    wait_vmcnt(0);
    __syncthreads();
    stage_chunk(cx.blob, kSlots - 2, base, wave_u, lane);
    bf16x8 ra[kRing][4];
#pragma unroll
    for (int n = 0; n < kPf; ++n) read_unit(cx, n, ra);
    f32x16 acc[8];
    u32x4 w[2][2];
    read_masks(cx, 0, w[0]);
    layer_bwd<0>(acc, bH, bL, aH, aL, ra, cx, io, ti, w[0], w[1]);      // dZ_7 (mask: H_7)
    read_masks(cx, 1, w[1]);
    layer_bwd<1>(acc, aH, aL, bH, bL, ra, cx, io, ti, w[1], w[0]);      // dZ_6
    read_masks(cx, 0, w[0]);
    layer_bwd<2>(acc, bH, bL, aH, aL, ra, cx, io, ti, w[0], w[1]);      // dZ_5
    read_masks(cx, 1, w[1]);
    layer_bwd<3>(acc, aH, aL, bH, bL, ra, cx, io, ti, w[1], w[0]);      // dZ_4
    read_masks(cx, 0, w[0]);
    layer_bwd<4>(acc, bH, bL, aH, aL, ra, cx, io, ti, w[0], w[1]);      // dZ_3
    read_masks(cx, 1, w[1]);
    layer_bwd<5>(acc, aH, aL, bH, bL, ra, cx, io, ti, w[1], w[0]);      // dZ_2
    read_masks(cx, 0, w[0]);
    layer_bwd<6>(acc, bH, bL, aH, aL, ra, cx, io, ti, w[0], w[1]);      // dZ_1
    read_masks(cx, 1, w[1]);
    layer_bwd<7>(acc, aH, aL, bH, bL, ra, cx, io, ti, w[1], w[0]);      // dZ_0
    // the last layer's tiles 6, 7 (no next layer to convert them in)
    Keep kp;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int t = 6 + (m >> 3), pr = m & 7;
      convert_dword(acc[t], t, pr, w[1][1][t & 3], cx, aH[0], aL[0], kp, false);
    }
    flush_rows(cx, io.dz[0], ti.p_first, n_points, 192);
  }
  // the stream ran into a tile that does not exist: let it land before the LDS is released
  wait_vmcnt(0);
}

}  // namespace

hipError_t launch_train_bwd_x3(const void* blob, long n_points, const BwdX3Io& io, hipStream_t stream) {
  if (n_points <= 0) return hipSuccess;
  // request_masks forms a 32-bit byte offset (s * 8 + ...) * 4 into the mask words
  if (n_points >= (1L << 27)) return hipErrorInvalidValue;
  const long tiles = (n_points + kSamplesPerBlock - 1) / kSamplesPerBlock;
  const long blocks = tiles < current_device_cus() ? tiles : current_device_cus();   // one workgroup per CU
  hipLaunchKernelGGL(train_bwd_x3_kernel, dim3(unsigned(blocks)), dim3(kThreads), 0, stream, (const char*)blob,
                     n_points, io);
  return hipGetLastError();
}

}  // namespace nerf
