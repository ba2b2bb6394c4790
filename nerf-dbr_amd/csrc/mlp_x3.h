// Split-precision ("x3") NeRF MLP on gfx950: the parity-grade fast paths.
//
// Replaces NeRFModel.forward (src/models/nerf.py:92-131) fused with
// sample_points_on_rays (src/benchmark/base_renderer.py:260-281) and the
// positional encoding (nerf.py:24-45), like mlp_f32.hip, but on the 16-bit MFMA
// (v_mfma_f32_32x32x16_{bf16,f16}, 16x the f32 MFMA rate): every fp32 operand v
// is split into v_hi = T(v) and v_lo = T(v - v_hi), and each product is
//     W.X ~= W_hi.X_hi + W_hi.X_lo + W_lo.X_hi
// accumulated in fp32, three MFMAs per product.  Two operand types T:
//   * bf16 (NERF_BF16X3): the dropped terms are ~2^-17 relative;
//   * fp16 (NERF_F16X3): 11-bit halves, the dropped terms ~2^-22 relative (the
//     lo parts of small values are fp16 subnormals: absolute 2^-25), ten times
//     closer to fp32 than bf16x3 at the same MFMA count -- the margin the real
//     (Lego) checkpoint needs under the 1e-4 gate.  fp16's range
//     (65504) is checked on the weights at packing; activations of the NeRF MLP
//     stay far inside it (max 65 on Lego, 6 on the synthetic net).
//
// Structure: mlp_bf16.hip's (transposed Linear, accumulators become the next
// layer's B fragments, quarter schedule, LDS ring filled by LDS-DMA with one
// barrier per chunk, persistent tiles, compiler-counted fragment reads),
// with one wave per SIMD: a lane holds the layer's 8 accumulator tiles (128)
// and the previous and next layers' hi and lo fragments (4 x 64), which only
// fits in the 512-entry register file of a single wave (accumulators in AGPRs).
//   * 4 waves x 32 samples = 128 samples per workgroup tile;
//   * weight units of 4 KiB = the bf16 kernel's 2 KiB unit of W_hi, then W_lo
//     (nerf_pack_weights_bf16x3 / _f16x3), 4 units per 16 KiB chunk, 3-slot ring (4 in the split-bf16 unit: NERF_X3_SLOTS);
//   * encodings are the accurate fp32 ones (sincos_acc, as the fp32 path; the training kernels keep ocml sincosf), split
//     into hi and lo fragments in LDS;
//   * the ReLU'd fp32 activations are split as they are converted:
//     hi = T(relu x), lo = T(relu x - hi).
// Outputs (sigma, r, g, b) per sample, or -- render passes with S % 32 == 0 --
// the compositing fused into the epilogue: each wave's 32 samples are one
// segment of one ray and leave as one 32-B segment record (nerf_device.h
// seg_composite, chained by composite_segments_kernel), as mlp_bf16.hip does.
#pragma once
#include "nerf_asm.h"
#include "nerf_device.h"
#include "nerf_internal.h"

namespace nerf {
namespace {

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kSamplesPerBlock = kWaves * kSamplesPerWave;            // 128
constexpr int kUnits = kHeadUnitBase + kHeadUnits;                    // 516 layer units + 12 head units
constexpr int kUnitB = 2 * kUnitBytes;                                // 4 KiB: hi unit, lo unit
// Ring geometry (compile-time knobs, swept with tools/kernel_lab.py; make variant)
#ifndef NERF_X3_CHUNK_UNITS
#define NERF_X3_CHUNK_UNITS 4
#endif
#ifndef NERF_X3_SLOTS
#define NERF_X3_SLOTS 3
#endif
#ifndef NERF_X3_PF
#define NERF_X3_PF 3
#endif
// counted seam waits in the training forward (needs NERF_X3_SLOTS=4; mlp_bf16x3.hip)
#ifndef NERF_X3_TRAIN_COUNTED
#define NERF_X3_TRAIN_COUNTED 0
#endif
constexpr int kChunkUnits = NERF_X3_CHUNK_UNITS;
constexpr int kChunkB = kChunkUnits * kUnitB;                         // 16 KiB
constexpr int kTotalChunks = (kUnits + kChunkUnits - 1) / kChunkUnits;   // 132
constexpr int kSlots = NERF_X3_SLOTS;
constexpr int kPf = NERF_X3_PF;                                       // fragment prefetch distance (units)
static_assert(kSlots >= 3 && kPf <= kChunkUnits, "prefetch reaches at most one published chunk ahead");
constexpr int kRing = kPf + 1;
constexpr int kGldsPerStage = kChunkB / (kThreads * 16);              // 4 LDS-DMA pieces per wave per chunk
static_assert(kTotalChunks % kSlots == 0, "the stream runs on into the next tile: chunk g always uses slot g % kSlots");
static_assert(kTotalChunks * kChunkB <= kBf16x3BlobBytes, "device blob is padded for the chunk geometry");
static_assert(kGldsPerStage * kThreads * 16 == kChunkB, "stage geometry");
constexpr int kLdsParamOff = kSlots * kChunkB;
constexpr int kLdsPeOff = kLdsParamOff + ((kParamFloats * 4 + 1023) / 1024) * 1024;
constexpr int kPeWaveB = 2 * 4 * 1024;                                // hi, lo x 4 k-steps x 1 KiB
constexpr int kDeWaveB = 2 * 2 * 1024;                                // hi, lo x 2 k-steps x 1 KiB
constexpr int kLdsDeOff = kLdsPeOff + kWaves * kPeWaveB;
constexpr int kLdsSegOff = kLdsDeOff + kWaves * kDeWaveB;            // fused compositing: (dist, z) per sample
constexpr int kLdsBytes = kLdsSegOff + kWaves * kSamplesPerWave * 8;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
// Training forward only: a tile pair's ReLU'd rows staged per wave, [sample 32][64 floats] at
// a 272-B pitch (conflict-free 16-B writes), stored as whole 256-B row segments
constexpr int kRowPitch = 272;
constexpr int kLdsRowOff = kLdsBytes;
constexpr int kLdsBytesTrain = kLdsRowOff + kWaves * kSamplesPerWave * kRowPitch;
static_assert(kLdsBytesTrain <= 160 * 1024, "LDS budget (training forward)");
// ds_read offsets are 16 bits: slots below kLoSlots are read at ring_addr + offset,
// the rest at ring_hi_addr (= ring_addr + kLoSlots * kChunkB) + offset
constexpr int kLoSlots = 65536 / kChunkB < kSlots ? 65536 / kChunkB : kSlots;
static_assert(kChunkB <= 32768 && (kSlots - kLoSlots) * kChunkB <= 65536, "ds_read offsets");
static_assert(kGldsPerStage >= 1, "at least one LDS-DMA piece per wave per chunk");

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// The operand type: the MFMA and the fp32 -> (hi, lo) split of two values, packed.
struct OpBf16 {
  typedef bf16x8 frag;
  static __device__ __forceinline__ f32x16 mfma(const frag& a, const frag& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  // hi = bf16(v) (v_cvt_pk_bf16_f32), lo = bf16(v - hi); v - hi is exact in fp32
  static __device__ __forceinline__ void split_pair(float a, float b, unsigned& hi, unsigned& lo) {
    hi = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));
    const float ha = __builtin_bit_cast(float, hi << 16), hb = __builtin_bit_cast(float, hi & 0xFFFF0000u);
    lo = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{__fsub_rn(a, ha), __fsub_rn(b, hb)}, bf16x2));
  }
};
struct OpF16 {
  typedef f16x8 frag;
  static __device__ __forceinline__ f32x16 mfma(const frag& a, const frag& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  // hi = f16(v) (v_cvt_pk_f16_f32, round to nearest even), lo = f16(v - hi): one
  // v_fma_mix{lo,hi}_f16 per value computes fma(-f32(hi half), 1, v) -- the exact
  // difference -- and rounds it to f16 into its half (subnormal lo for |v| < 2^-3
  // keeps an absolute 2^-25); the compiler's form is two conversions back to f32,
  // a packed subtraction and a second packed conversion
  static __device__ __forceinline__ void split_pair(float a, float b, unsigned& hi, unsigned& lo) {
    hi = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, f16x2));
#ifdef NERF_X3_NO_MIX
    const f32x2 hf = __builtin_convertvector(__builtin_bit_cast(f16x2, hi), f32x2);
    lo = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{__fsub_rn(a, hf[0]), __fsub_rn(b, hf[1])}, f16x2));
#else
    unsigned l;
    asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "=&v"(l) : "v"(hi), "v"(a), "v"(b));
    lo = l;
#endif
  }
};

NL_HD bool is_seam(int n) { return (n + kPf) % kChunkUnits == 0 && n + kPf < kUnits && n + kPf != 0; }
// NERF_X3_REGSTAGE (lab knob): the weight stream is staged through registers instead of
// LDS-DMA -- each wave loads its pieces of a chunk into AGPRs at one seam
// (global_load_dwordx4) and writes them to the ring at the next (ds_write_b128), so the
// ds_writes join the LDS counts below.
#ifndef NERF_X3_REGSTAGE
#define NERF_X3_REGSTAGE 0
#endif
NL_HD int seam_writes(int m) { return NERF_X3_REGSTAGE && m >= 0 && m < kUnits && is_seam(m) ? kGldsPerStage : 0; }
// writes of the seams in bodies n-kPf+1 .. n: younger than unit n's reads (issued in body n-kPf)
NL_HD int seam_writes_since(int n) {
  int c = 0;
  for (int m = n - kPf + 1; m <= n; ++m) c += seam_writes(m);
  return c;
}

// ---- compile-time unit map, as a constexpr table (this kernel is large
// enough that the optimiser stops folding mlp_bf16.hip's loop-based map) ----
struct UnitInfo {
  int layer, kstep, extra, reads, lgkm;
  bool opens;
};
struct UnitTable {
  UnitInfo u[kUnits];
};
constexpr UnitTable make_unit_table(int skip = kSkipNeRFModel) {
  UnitTable t{};
  for (int n = 0; n < kUnits; ++n) {
    UnitInfo& x = t.u[n];
    if (n >= kHeadUnitBase) {
      x = UnitInfo{-1, n - kHeadUnitBase, 0, 4, 0, false};
      continue;
    }
    int l = 0;
    while (l + 1 < kNumMfmaLayers && bf16_unit_base(l + 1, skip) <= n) ++l;
    const int ks = (n - bf16_unit_base(l, skip)) % ksteps_bf16(l, skip);
    const int ex = ks < layer_shape(l, skip).hidden / 16 ? 0 : layer_shape(l, skip).extra;
    x = UnitInfo{l, ks, ex, 4 + (ex != 0 ? 2 : 0), 0, ks == 0};
  }
  constexpr int kBiasReads = 8;   // 2 tiles x 4 x 16 B
  // LDS reads younger than everything unit n consumes, at its wait: the issue
  // order per unit body m is [bias reads if m opens a quarter], reads of unit
  // m+kPf, wait, MFMAs (the prologue issued units 0..kPf-1)
  for (int n = 0; n < kUnits; ++n) {
    int c = 0;
    if (t.u[n].opens) {
      c = n + kPf < kUnits ? t.u[n + kPf].reads : 0;
    } else {
      for (int k = n + 1; k <= n + kPf; ++k) c += k < kUnits ? t.u[k].reads : 0;
      for (int m = n - kPf + 1; m <= n; ++m) c += (m >= 0 && t.u[m].opens ? kBiasReads : 0);
      c += seam_writes_since(n);
    }
    t.u[n].lgkm = c;
  }
  return t;
}
// per network layout (nerf_layout.h kSkip*: the layer that takes the position encoding again)
template <int kSkip>
constexpr UnitTable kTabT = make_unit_table(kSkip);
constexpr UnitTable kTab = kTabT<kSkipNeRFModel>;

struct Ctx {
  const char* blob;
  char* lds;
  int wave_u, lane, h;
  unsigned ring_addr, pe_addr, de_addr, bias_addr, ring_hi_addr;
  u32x4* stg;            // NERF_X3_REGSTAGE: this wave's pieces of the chunk in flight (AGPRs)
  unsigned stg_addr;     // NERF_X3_REGSTAGE: LDS address of this lane's 16 B in slot 0, piece 0
};

__device__ __forceinline__ void stage_piece(const char* __restrict__ blob, int g, char* lds, int wave_u, int lane,
                                            int i) {
#ifdef NERF_X3_ABLATE_NODMA   // timing-only lab build (wrong results): the weight stream is not restaged
  if (g >= kSlots) return;
#endif
  char* dst = lds + (g % kSlots) * kChunkB + wave_u * 1024;
  // the piece's offset rides in the scalar base, so every piece shares one address
  // VGPR (four per-piece VGPRs were spilled to AGPRs and reloaded before each piece:
  // 3 spills and ~370 v_accvgpr_read per tile; time-neutral, bit-identical)
  lds_dma_16_s(blob + size_t(g) * kChunkB + i * kThreads * 16, unsigned(wave_u * 1024 + lane * 16),
               lds_addr(dst + i * kThreads * 16));
}
__device__ __forceinline__ void stage_chunk(const char* __restrict__ blob, int g, char* lds, int wave_u, int lane) {
#pragma unroll
  for (int i = 0; i < kGldsPerStage; ++i) stage_piece(blob, g, lds, wave_u, lane, i);
}

// NERF_X3_REGSTAGE: chunk g's pieces -> this wave's staging AGPRs (vmcnt), and from
// them into ring slot g % kSlots (lgkmcnt).  The asm outputs count as written at
// issue; the seams wait vmcnt before the writes read them.
__device__ __forceinline__ void load_chunk_regs(const Ctx& cx, int g) {
#pragma unroll
  for (int i = 0; i < kGldsPerStage; ++i) {
    const unsigned long long sb = (unsigned long long)(cx.blob + size_t(g) * kChunkB + i * kThreads * 16);
    const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(sb)), hi = __builtin_amdgcn_readfirstlane(unsigned(sb >> 32));
    const unsigned long long s64 = (unsigned long long)lo | ((unsigned long long)hi << 32);
    asm volatile("global_load_dwordx4 %0, %1, %2" : "=a"(cx.stg[i]) : "v"(unsigned(cx.wave_u * 1024 + cx.lane * 16)),
                 "s"(s64) : "memory");
  }
}
__device__ __forceinline__ void write_chunk_regs(const Ctx& cx, int g) {
#pragma unroll
  for (int i = 0; i < kGldsPerStage; ++i)
    asm volatile("ds_write_b128 %0, %1 offset:%2" :: "v"(cx.stg_addr), "a"(cx.stg[i]),
                 "i"((g % kSlots) * kChunkB + i * kThreads * 16) : "memory");
}

template <class Op>
__device__ __forceinline__ void split8(const float* v, u32x4& hi, u32x4& lo) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    unsigned h2, l2;
    Op::split_pair(v[2 * d], v[2 * d + 1], h2, l2);
    hi[d] = h2;
    lo[d] = l2;
  }
}

// NERF_X3_ABLATE_NODIR (timing-only lab build, wrong results): C0's direction k-steps, their
// B-fragment reads and the per-sample direction encoding dropped -- the upper bound of
// computing Wc0[:, 256:283] . PE4(d) once per ray instead of per sample (VERDICT r5 next 5a:
// nerf.py:117-129 feeds one PE4(d) to all samples of a ray).
#ifdef NERF_X3_ABLATE_NODIR
constexpr bool kNoDir = true;
#else
constexpr bool kNoDir = false;
#endif

// Reads of unit n into ring entry n % kRing: A_hi and A_lo of the unit's two
// output tiles and, for encoding inputs, the B fragment's hi and lo.
template <class Op, int kSkip = kSkipNeRFModel, class F = typename Op::frag>
__device__ __forceinline__ void read_unit(const Ctx& cx, int n, F (&ra)[kRing][4], F (&rb)[kRing][2]) {
  constexpr UnitTable kTab = kTabT<kSkip>;
#ifdef NERF_X3_ABLATE_NOREAD   // timing-only lab build (wrong results): the ring's first fragments reused
  if (n >= kRing) return;
#endif
  const int slot = (n / kChunkUnits) % kSlots;
  const unsigned base = slot < kLoSlots ? cx.ring_addr : cx.ring_hi_addr;
  const int off = (slot < kLoSlots ? slot : slot - kLoSlots) * kChunkB + (n % kChunkUnits) * kUnitB;
#pragma unroll
  for (int f = 0; f < 4; ++f) ra[n % kRing][f] = ds_read_b128<F>(base, off + f * 1024);
  const int ex = kTab.u[n].extra;
  if (ex != 0 && !(kNoDir && ex == kDir)) {
    const int u = kTab.u[n].kstep - layer_shape(kTab.u[n].layer, kSkip).hidden / 16;
    if (ex == kPos) {
      rb[n % kRing][0] = ds_read_b128<F>(cx.pe_addr, u * 1024);
      rb[n % kRing][1] = ds_read_b128<F>(cx.pe_addr, 4096 + u * 1024);
    } else {
      rb[n % kRing][0] = ds_read_b128<F>(cx.de_addr, u * 1024);
      rb[n % kRing][1] = ds_read_b128<F>(cx.de_addr, 2048 + u * 1024);
    }
  }
}

constexpr int kDmaOutstandingAtSeam = kSlots - 3;
constexpr int kStageAhead = kSlots - 1;
// NERF_X3_SPREAD (lab knob): a seam stages only its first LDS-DMA piece and the next
// units one piece each, instead of all pieces back to back at the seam.
#ifndef NERF_X3_SPREAD
#define NERF_X3_SPREAD 0
#endif
static_assert(!NERF_X3_SPREAD || !NERF_X3_REGSTAGE, "one staging form");
static_assert(!NERF_X3_REGSTAGE || kSlots == 3, "register staging: chunk g+2 written at seam g into chunk g-1's slot");
static_assert(!NERF_X3_SPREAD || (kGldsPerStage <= kChunkUnits && kSlots >= 4),
              "spread pieces land within a chunk, and need one chunk of slack at the next seam");
// Training forward (kTrain): the seams' vmcnt waits are counted.  vmcnt retires vector-memory
// operations in issue order, LDS-DMA pieces and stores alike; the chunk a seam publishes
// (g + 1) was staged two seams earlier, so everything issued after that stage -- the
// stage at the seam between (kGldsPerStage pieces) and the sink's row and ReLU-bit stores
// of the bodies since -- may stay in flight.  A vmcnt(kGldsPerStage) wait (kSlots = 4)
// would also drain every store issued since the last stage.  The store counts per unit
// body mirror layer_x3 and the heads loop (every store is unconditional: samples past the
// last are clamped to it); the tile top waits vmcnt(0), so a tile's first two seams count
// from the tile top.
#ifndef NERF_X3_ABLATE_NOSTORE
constexpr int kFlushStores = kSamplesPerWave / 4;        // flush_rows: one 16-B store per 4 lanes' sample
constexpr int kMaskStores = 1;                           // the tile's ReLU-bit word
#else   // the timing-only build issues no row or bit stores: the tables must not count them
constexpr int kFlushStores = 0;
constexpr int kMaskStores = 0;
#endif
struct TrainVm {
  int stores[kUnits];                                    // global stores of unit body n (after its seam)
  int seam[kUnits];                                      // the seam wait before body n, if is_seam(n)
};
constexpr void add_sink_stores(TrainVm& t, int n, int l, int tile, int pr) {
  if (pr != 7) return;
  if (l < 8) t.stores[n] += kMaskStores;                 // the tile's ReLU-bit word
  if (tile & 1) t.stores[n] += kFlushStores;             // the tile pair's rows
}
constexpr int dword_unit_out_c(int ku, int m) { return ku >= 16 ? 2 + (m * (ku - 2)) / 16 : m / 4; }
constexpr int dword_unit_in_c(int m) { return 2 + (m * 10) / 16; }
constexpr TrainVm make_train_vm() {
  TrainVm t{};
  for (int L = 0; L < kNumMfmaLayers; ++L) {
    const int KU = ksteps_bf16(L), NQ = out_tiles(L) / 2, N0 = bf16_unit_base(L);
    for (int q = 0; q < NQ; ++q)
      for (int u = 0; u < KU; ++u)
        for (int m = 0; m < 16; ++m) {
          const int n = N0 + q * KU + u, tt = m >> 3, pr = m & 7;
          if (L != L0 && q == 0 && u == dword_unit_in_c(m)) add_sink_stores(t, n, L - 1, 6 + tt, pr);
          if (q >= 1 && u == dword_unit_out_c(KU, m)) add_sink_stores(t, n, L, 2 * q - 2 + tt, pr);
        }
  }
  for (int i = 0; i < kHeadUnits; ++i)
    for (int m = 0; m < 16; ++m)
      if (i < 8 && m / 2 == i) add_sink_stores(t, kHeadUnitBase + i, C0, 2 + (m >> 3), m & 7);
  for (int n = 0; n < kUnits; ++n) {
    if (!is_seam(n)) continue;
    const int g = (n + kPf) / kChunkUnits - 1;
    const int from = g >= 2 ? kChunkUnits * (g - 1) - kPf : 0;   // body of seam g - 2 (its stage precedes its stores)
    int c = kGldsPerStage;                                        // the stage at seam g - 1 (or the tile top)
    for (int k = from; k < n; ++k) c += t.stores[k];
    t.seam[n] = c;
  }
  return t;
}
constexpr TrainVm kTrainVm = make_train_vm();
static_assert(kSlots == 4 || !NERF_X3_TRAIN_COUNTED, "counted training seams: chunk g + 1 staged two seams ahead");

template <bool kTrain = false>
__device__ __forceinline__ void seam_before(const Ctx& cx, int n) {
  if (NERF_X3_SPREAD) {
#pragma unroll
    for (int i = 1; i < kGldsPerStage; ++i)
      if (n - i >= 0 && is_seam(n - i))
        stage_piece(cx.blob, ((n - i + kPf) / kChunkUnits - 1 + kStageAhead) % kTotalChunks, cx.lds, cx.wave_u,
                    cx.lane, i);
  }
  if (!is_seam(n)) return;
  const int g = (n + kPf) / kChunkUnits - 1;
  if (NERF_X3_REGSTAGE) {   // chunk g+2 (loaded at seam g-1) -> the slot chunk g-1 frees; load chunk g+3
    wait_vmcnt(0);
    compiler_fence();
    __builtin_amdgcn_s_barrier();
    compiler_fence();
    write_chunk_regs(cx, (g + kStageAhead) % kTotalChunks);
    load_chunk_regs(cx, (g + kStageAhead + 1) % kTotalChunks);
    return;
  }
  if (kTrain && NERF_X3_TRAIN_COUNTED) wait_vmcnt_exact(kTrainVm.seam[n]);
  else wait_vmcnt(kGldsPerStage * kDmaOutstandingAtSeam);
  compiler_fence();
#ifndef NERF_X3_ABLATE_NOBARRIER   // timing-only lab build (wrong results): no seam barriers
  __builtin_amdgcn_s_barrier();
#endif
  compiler_fence();
  if (NERF_X3_SPREAD) stage_piece(cx.blob, (g + kStageAhead) % kTotalChunks, cx.lds, cx.wave_u, cx.lane, 0);
  else stage_chunk(cx.blob, (g + kStageAhead) % kTotalChunks, cx.lds, cx.wave_u, cx.lane);
}

// Conversion schedule of mlp_bf16.hip: one dword (two values) per unit.
NL_HD int dword_unit_out(int ku, int m) { return ku >= 16 ? 2 + (m * (ku - 2)) / 16 : m / 4; }
NL_HD int dword_unit_in(int m) { return 2 + (m * 10) / 16; }
constexpr bool same_conversion_schedule() {   // make_train_vm's copies of the two maps
  for (int m = 0; m < 16; ++m) {
    if (dword_unit_in(m) != dword_unit_in_c(m)) return false;
    for (int ku = 1; ku <= 40; ++ku)
      if (dword_unit_out(ku, m) != dword_unit_out_c(ku, m)) return false;
  }
  return true;
}
static_assert(same_conversion_schedule(), "the counted seams mirror the conversion schedule");
// fp16 range contract (NERF_F16X3): an activation at or above 65520 converts to hi = +inf and
// lo = f16(x - inf) = -inf, so in the next layer every row of that sample's column takes
// w_hi.inf + w_hi.(-inf) (or 0.inf) = NaN.  One row per column is checked as each layer's
// output tile 0 is converted (pre-ReLU, so a NaN's sign does not matter), and the heads'
// accumulators at the end of the tile; a hit sets the caller's range flag (one vector store)
// and the host reports NERF_E_RANGE (nerf_ctx_range_status) instead of returning the image.
template <class Op>
__device__ __forceinline__ bool range_checked() { return __is_same(Op, OpF16); }

template <class Op>
__device__ __forceinline__ void convert_dword(const f32x16& tile, int pr, u32x4& fhi, u32x4& flo) {
#ifdef NERF_X3_ABLATE_NOCONV   // timing-only lab build (wrong results): accumulator bits as fragments
  fhi[pr & 3] = __builtin_bit_cast(unsigned, tile[2 * pr]);
  flo[pr & 3] = __builtin_bit_cast(unsigned, tile[2 * pr + 1]);
  return;
#endif
  unsigned h2, l2;
#ifdef NERF_X3_ABLATE_NORELU   // timing-only lab build (wrong results): the split without the ReLU
  Op::split_pair(tile[2 * pr], tile[2 * pr + 1], h2, l2);
#else
  Op::split_pair(relu(tile[2 * pr]), relu(tile[2 * pr + 1]), h2, l2);
#endif
  fhi[pr & 3] = h2;
  flo[pr & 3] = l2;
}

__device__ __forceinline__ void issue_bias(const Ctx& cx, int l, int q, f32x16 (&acc)[8]) {
#pragma unroll
  for (int o2 = 0; o2 < 2; ++o2) {
    const int off = 4 * (kBiasOff + 256 * l + (2 * q + o2) * 32);
    const f32x4 b0 = ds_read_b128<f32x4>(cx.bias_addr, off), b1 = ds_read_b128<f32x4>(cx.bias_addr, off + 16);
    const f32x4 b2 = ds_read_b128<f32x4>(cx.bias_addr, off + 32), b3 = ds_read_b128<f32x4>(cx.bias_addr, off + 48);
    acc[2 * q + o2] = f32x16{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3],
                             b2[0], b2[1], b2[2], b2[3], b3[0], b3[1], b3[2], b3[3]};
  }
}

template <class Op, class F = typename Op::frag>
__device__ __forceinline__ f32x16 mfma3(const F& ahi, const F& alo, const F& bhi, const F& blo, f32x16 acc) {
  acc = Op::mfma(ahi, bhi, acc);
  acc = Op::mfma(ahi, blo, acc);
  return Op::mfma(alo, bhi, acc);
}

// Training outputs (launch_mlp_bf16x3_train): as each accumulator tile is converted, its
// ReLU'd fp32 values also go out as the sample's row (one 16-B piece per two dwords:
// registers 4j..4j+3 are features 32t + 8j + 4h + 0..3) and, for trunk layers, its ReLU bits
// as one word per tile (bit acc_row(r, h) of register r), both halves merged by a lane swap.
struct TrainSink {
  X3TrainOut o;
  long p;
  bool valid;
  unsigned bits[2];
  long p_first;         // the wave's first sample
  long n_points;
  unsigned row_w;       // LDS: this lane's sample row in the wave's staging block
  unsigned row_r;       // LDS: the flush's read address (sample lane / 16, piece lane % 16)
  int lane;
  unsigned mb_off;      // byte offset of the (clamped) sample's ReLU-bit words: one 32-bit VGPR for every store
};
__device__ __forceinline__ void lds_store16(unsigned addr, f32x4 v) {
  *(__attribute__((address_space(3))) f32x4*)(uintptr_t)addr = v;
}
// The staged tile pair t0, t0+1 of layer l (features 32 t0 .. +63 of the wave's 32 samples)
// to the rows: lane l stores 16 B of sample 4i + l / 16, four whole 256-B segments per
// instruction, non-temporal for the 1-KiB h rows (read once, by the backward and the weight
// gradients); a sample past the last is clamped to it (its values equal the last sample's).
__device__ __forceinline__ void flush_rows(const TrainSink& sk, int l, int t0, int lane) {
#ifdef NERF_X3_ABLATE_NOSTORE   // timing-only lab build (no rows): what the training rows cost
  return;
#endif
#pragma unroll
  for (int i = 0; i < kSamplesPerWave / 4; ++i) {
    const f32x4 v = ds_read_b128<f32x4>(sk.row_r, i * 4 * kRowPitch);
    long s = sk.p_first + 4 * i + (lane >> 4);
    s = s < sk.n_points ? s : sk.n_points - 1;
    if (l < 8) __builtin_nontemporal_store(v, (f32x4*)(sk.o.h[l] + s * 256 + 32 * t0 + 4 * (lane & 15)));
    else *(f32x4*)(sk.o.hc + s * 132 + 32 * t0 + 4 * (lane & 15)) = v;
  }
}
template <bool kTrain>
__device__ __forceinline__ void sink_dword(TrainSink& sk, int l, int t, int slot, const f32x16& tile, int pr, int h) {
  if constexpr (kTrain) {
    if (l < 8) {
      const unsigned m = (tile[2 * pr] > 0.0f ? 1u : 0u) << acc_row(2 * pr, h) |
                         (tile[2 * pr + 1] > 0.0f ? 1u : 0u) << acc_row(2 * pr + 1, h);
      sk.bits[slot] = (pr == 0 ? 0u : sk.bits[slot]) | m;
      if (pr == 7) {
        const auto sw = __builtin_amdgcn_permlane32_swap(sk.bits[slot], sk.bits[slot], false, false);
#ifndef NERF_X3_ABLATE_NOSTORE
        // counted seams: every lane stores (both halves hold the merged word, and a sample
        // past the last is clamped to it, the same word) -- no exec branch, one store per tile
        if (NERF_X3_TRAIN_COUNTED) *(unsigned*)((char*)sk.o.mb[l] + sk.mb_off + 4 * t) = unsigned(sw[0]) | unsigned(sw[1]);
        else if (sk.valid && h == 0) sk.o.mb[l][sk.p * 8 + t] = unsigned(sw[0]) | unsigned(sw[1]);
#endif
      }
    }
    if (pr & 1) {   // registers 4j..4j+3 are features 32t + 8j + 4h + 0..3: into the staging block
      const int j = pr >> 1;
      lds_store16(sk.row_w + unsigned(((t & 1) * 32 + 8 * j + 4 * h) * 4),
                  f32x4{relu(tile[4 * j]), relu(tile[4 * j + 1]), relu(tile[4 * j + 2]), relu(tile[4 * j + 3])});
      if (pr == 7 && (t & 1)) flush_rows(sk, l, t - 1, sk.lane);   // the pair's last dword
    }
  }
}

// NERF_X3_SCHED (lab knob): an explicit issue pattern for a unit body's scheduling region
// (sched_group_barrier), so that the region's VALU (conversions) and LDS reads sit between the
// MFMAs instead of where the compiler's scheduler clumps them (one wave per SIMD hides ~5
// single-issue instructions per 32-cycle MFMA gap, MI355X_MICROARCH.md constants table).
//   1: per MFMA: 1 MFMA, 1 DS read, 2 VALU;   2: per MFMA: 1 MFMA, 2 VALU, 1 DS read;
//   3: per MFMA: 1 MFMA, 1 VALU, 1 DS read, 1 VALU.
#ifndef NERF_X3_SCHED
#define NERF_X3_SCHED 0
#endif
__device__ __forceinline__ void sched_unit_pattern() {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    if (NERF_X3_SCHED == 1) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
    } else if (NERF_X3_SCHED == 2) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    } else if (NERF_X3_SCHED == 3) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    }
  }
}

// One layer: reads the previous layer's fragments (ih/il), fills the next's (oh/ol).
template <int L, bool kTrain, class Op, int kSkip = kSkipNeRFModel, class F = typename Op::frag>
__device__ __forceinline__ void layer_x3(f32x16 (&acc)[8], u32x4 (&ih)[16], u32x4 (&il)[16], u32x4 (&oh)[16],
                                         u32x4 (&ol)[16], F (&ra)[kRing][4], F (&rb)[kRing][2],
                                         const Ctx& cx, TrainSink& sk, bool& nan_seen) {
  constexpr LayerShape sh = layer_shape(L, kSkip);
  constexpr UnitTable kTab = kTabT<kSkip>;
  constexpr int KH = sh.hidden / 16;
  constexpr int KU = ksteps_bf16(L, kSkip);
  constexpr int NQ = out_tiles(L) / 2;
  constexpr int N0 = bf16_unit_base(L, kSkip);
  constexpr bool kConvert = L != L0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int n = N0 + q * KU + u;
      seam_before<kTrain>(cx, n);
      if (u == 0) issue_bias(cx, L, q, acc);
      if (n + kPf < kUnits) read_unit<Op, kSkip>(cx, n + kPf, ra, rb);
      wait_lgkm(kTab.u[n].lgkm);
      __builtin_amdgcn_sched_barrier(0);
      const bool hid = u < KH;
      const F bhi = hid ? __builtin_bit_cast(F, ih[hid ? u : 0]) : rb[n % kRing][0];
      const F blo = hid ? __builtin_bit_cast(F, il[hid ? u : 0]) : rb[n % kRing][1];
      if (!(kNoDir && L == C0 && !hid))
#pragma unroll
        for (int o2 = 0; o2 < 2; ++o2)
          acc[2 * q + o2] = mfma3<Op>(ra[n % kRing][o2], ra[n % kRing][2 + o2], bhi, blo, acc[2 * q + o2]);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int t = m >> 3, pr = m & 7;
        if (kConvert && q == 0 && u == dword_unit_in(m)) {
          convert_dword<Op>(acc[6 + t], pr, ih[2 * (6 + t) + (pr >> 2)], il[2 * (6 + t) + (pr >> 2)]);
          sink_dword<kTrain>(sk, L > 0 ? L - 1 : 0, 6 + t, t, acc[6 + t], pr, cx.h);
        }
        if (q >= 1 && u == dword_unit_out(KU, m)) {
          if (!kTrain && range_checked<Op>() && q == 1 && t == 0 && pr == 0)
            nan_seen |= __builtin_isnan(acc[0][0]);
          convert_dword<Op>(acc[2 * q - 2 + t], pr, oh[2 * (2 * q - 2 + t) + (pr >> 2)], ol[2 * (2 * q - 2 + t) + (pr >> 2)]);
          sink_dword<kTrain>(sk, L, 2 * q - 2 + t, t, acc[2 * q - 2 + t], pr, cx.h);
        }
      }
      if (NERF_X3_SCHED && !kTrain) sched_unit_pattern();
    }
  }
}

// seg != nullptr (render passes, S % 32 == 0): one segment record per wave's 32
// samples instead of out's (sigma, r, g, b).
// kOrig: the original NeRF implementation's network (NERF_LAYOUT_ORIGINAL_NERF, render and
// query only): position encoding again at layer 5, encodings without pi, view directions
// normalised before their encoding (mlp_f32.hip, nerf_layout.h).
template <bool kExplicit, bool kTrain, class Op, bool kOrig = false>
__global__ __launch_bounds__(kThreads, 1) void mlp_x3_kernel(const char* __restrict__ blob,
                                                             const float* __restrict__ prm_g, SampleSrc src,
                                                             long n_points, f32x4* __restrict__ out,
                                                             f32x4* __restrict__ seg, X3TrainOut tro,
                                                             int* __restrict__ range_flag) {
  typedef typename Op::frag F;
  static_assert(!(kOrig && kTrain), "the original-NeRF layout renders only");
  constexpr int S = kOrig ? kSkipOriginal : kSkipNeRFModel;
  __shared__ __attribute__((aligned(16))) char lds[kTrain ? kLdsBytesTrain : kLdsBytes];
  const int lane = threadIdx.x & 63;
  const int wave_u = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5;
  const unsigned lds_base = lds_addr(lds);
  u32x4 stg[kGldsPerStage];
  const Ctx cx0{blob, lds, wave_u, lane, h, lds_base + lane * 16, lds_base + kLdsPeOff + wave_u * kPeWaveB + lane * 16,
                lds_base + kLdsDeOff + wave_u * kDeWaveB + lane * 16, lds_base + kLdsParamOff + h * 64,
                lds_base + kLoSlots * kChunkB + lane * 16, stg, lds_base + wave_u * 1024 + lane * 16};
  const long n_tiles = (n_points + kSamplesPerBlock - 1) / kSamplesPerBlock;
  const bool fused = !kExplicit && !kTrain && seg != nullptr;
  char* seg_slot = lds + kLdsSegOff + (wave_u * kSamplesPerWave + (lane & 31)) * 8;

  if (NERF_X3_REGSTAGE) {   // chunk 0 written now, chunk 1 loaded (written at the tile top)
    load_chunk_regs(cx0, 0);
    wait_vmcnt(0);
    write_chunk_regs(cx0, 0);
    load_chunk_regs(cx0, 1);
  } else {
#pragma unroll
    for (int g = 0; g < kSlots - 2; ++g) stage_chunk(blob, g, lds, wave_u, lane);
  }
  for (int i = threadIdx.x; i < kParamFloats / 4; i += kThreads)
    ((f32x4*)(lds + kLdsParamOff))[i] = ((const f32x4*)prm_g)[i];
  const float* prm = (const float*)(lds + kLdsParamOff);

  f32x4 res = {};
  long res_p0 = -1;
  // the previous tile's results, stored after the next tile's first wait (vmcnt
  // counts stores and LDS-DMA together, in issue order)
  auto store = [&]() {
    if (kTrain || res_p0 < 0) return;
    if (fused) {
      const long first = res_p0 - (lane & 31);                     // the segment's first sample
      if (first < n_points && lane < 2) seg[(first / kSamplesPerWave) * 2 + lane] = res;
    } else if (res_p0 < n_points && lane < 32) {
      out[res_p0] = res;
    }
  };
#pragma unroll 1
  for (long tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const long p0 = (tile * kWaves + wave_u) * kSamplesPerWave + (lane & 31);
    Ctx cx = cx0;
    asm volatile("" : "+s"(cx.blob));   // keep the 132 chunk addresses out of SGPRs across tiles
    const unsigned rows = lds_base + kLdsRowOff + wave_u * kSamplesPerWave * kRowPitch;
    TrainSink sk{tro, p0, p0 < n_points, {0u, 0u}, (tile * kWaves + wave_u) * kSamplesPerWave, n_points,
                 rows + (lane & 31) * kRowPitch, rows + (lane >> 4) * kRowPitch + (lane & 15) * 16, lane,
                 unsigned(p0 < n_points ? p0 : n_points - 1) * 32u};
#ifdef NERF_X3_ABLATE_PE_ONCE   // timing-only lab build (wrong results): encodings of the first tile reused
    if (tile == blockIdx.x)
#endif
    {
      float x[3], d[3], pef[32], def[16];
      const long pc = p0 < n_points ? p0 : n_points - 1;
      if (fused) {
        float dist, zz;
        fetch_render_sample(src, pc, n_points <= 0xFFFFFFFFL, true, x, d, dist, zz);
        if (h == 0) *(f32x2_t*)seg_slot = f32x2_t{dist, zz};
      } else {
        fetch_sample<kExplicit>(src, pc, x, d);
      }
      pos_encode<false, kTrain, kOrig>(x[0], x[1], x[2], h, pef);    // accurate sin/cos, as the fp32 path
      if (kOrig) {   // the original's viewdirs = rays_d / |rays_d| (its encoding input)
        const float nd = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(d[0], d[0]), __fmul_rn(d[1], d[1])),
                                              __fmul_rn(d[2], d[2])));
#pragma unroll
        for (int c = 0; c < 3; ++c) d[c] = __fdiv_rn(d[c], nd);
      }
      if (!kNoDir) dir_encode<false, kTrain, kOrig>(d[0], d[1], d[2], h, def);
      char* pe_dst = lds + kLdsPeOff + wave_u * kPeWaveB + lane * 16;
      char* de_dst = lds + kLdsDeOff + wave_u * kDeWaveB + lane * 16;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        u32x4 hi, lo;
        split8<Op>(pef + 8 * u, hi, lo);
        *(u32x4*)(pe_dst + u * 1024) = hi;
        *(u32x4*)(pe_dst + 4096 + u * 1024) = lo;
      }
#pragma unroll
      for (int u = 0; u < (kNoDir ? 0 : 2); ++u) {
        u32x4 hi, lo;
        split8<Op>(def + 8 * u, hi, lo);
        *(u32x4*)(de_dst + u * 1024) = hi;
        *(u32x4*)(de_dst + 2048 + u * 1024) = lo;
      }
    }
    if (kTrain && NERF_X3_TRAIN_COUNTED) wait_vmcnt(0);   // the seams below count from here
    else wait_vmcnt(kGldsPerStage * kDmaOutstandingAtSeam);
    __syncthreads();
    if (NERF_X3_REGSTAGE) {
      write_chunk_regs(cx, kStageAhead - 1);
      load_chunk_regs(cx, kStageAhead);
    } else {
      stage_chunk(cx.blob, kStageAhead - 1, lds, wave_u, lane);
    }
    store();
    F ra[kRing][4], rb[kRing][2];
    f32x16 acc[8];
#pragma unroll
    for (int n = 0; n < kPf; ++n) read_unit<Op, S>(cx, n, ra, rb);

    u32x4 aH[16], aL[16], bH[16], bL[16];
    bool nan_seen = false;
    layer_x3<L0, kTrain, Op, S>(acc, bH, bL, aH, aL, ra, rb, cx, sk, nan_seen);
    layer_x3<L1, kTrain, Op, S>(acc, aH, aL, bH, bL, ra, rb, cx, sk, nan_seen);
    layer_x3<L2, kTrain, Op, S>(acc, bH, bL, aH, aL, ra, rb, cx, sk, nan_seen);
    layer_x3<L3, kTrain, Op, S>(acc, aH, aL, bH, bL, ra, rb, cx, sk, nan_seen);
    layer_x3<L4, kTrain, Op, S>(acc, bH, bL, aH, aL, ra, rb, cx, sk, nan_seen);   // skip: [x, pe] (nerf.py:109-110)
    layer_x3<L5, kTrain, Op, S>(acc, aH, aL, bH, bL, ra, rb, cx, sk, nan_seen);
    layer_x3<L6, kTrain, Op, S>(acc, bH, bL, aH, aL, ra, rb, cx, sk, nan_seen);
    layer_x3<L7, kTrain, Op, S>(acc, aH, aL, bH, bL, ra, rb, cx, sk, nan_seen);
    layer_x3<C0, kTrain, Op, S>(acc, bH, bL, aH, aL, ra, rb, cx, sk, nan_seen);   // [x, PE4(d)] (nerf.py:117-121)

    // Heads (nerf.py:114, 123-129): one tile, density row 3 over L7's fragments
    // (bH/bL, C0's input, k-steps 0..15), colour rows 0-2 over C0's output
    // (aH/aL: tiles 0, 1 converted in C0's quarter 1, tiles 2, 3 below).
    f32x16 hacc = f32x16{};
    if (h == 0) {
      hacc[0] = prm[kC1B];
      hacc[1] = prm[kC1B + 1];
      hacc[2] = prm[kC1B + 2];
      hacc[3] = prm[kSigB];
    }
#pragma unroll
    for (int i = 0; i < kHeadUnits; ++i) {
      const int n = kHeadUnitBase + i;
      seam_before<kTrain>(cx, n);
      if (n + kPf < kUnits) read_unit<Op, S>(cx, n + kPf, ra, rb);
      wait_lgkm(4 * (kUnits - 1 - n < kPf ? kUnits - 1 - n : kPf) + seam_writes_since(n));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int k = 2 * i + s2;
        const F bhi = __builtin_bit_cast(F, k < 16 ? bH[k < 16 ? k : 0] : aH[k >= 16 ? k - 16 : 0]);
        const F blo = __builtin_bit_cast(F, k < 16 ? bL[k < 16 ? k : 0] : aL[k >= 16 ? k - 16 : 0]);
        hacc = mfma3<Op>(ra[n % kRing][s2], ra[n % kRing][2 + s2], bhi, blo, hacc);
      }
#pragma unroll
      for (int m = 0; m < 16; ++m)
        if (i < 8 && m / 2 == i)
          {
          convert_dword<Op>(acc[2 + (m >> 3)], m & 7, aH[2 * (2 + (m >> 3)) + ((m & 7) >> 2)],
                            aL[2 * (2 + (m >> 3)) + ((m & 7) >> 2)]);
          sink_dword<kTrain>(sk, C0, 2 + (m >> 3), m >> 3, acc[2 + (m >> 3)], m & 7, h);
        }
    }
    if (!kTrain && range_checked<Op>()) {
      // the heads' inputs (L7's and C0's outputs) and their accumulators: rows 0-3 sit in lanes 0-31
      nan_seen |= h == 0 && !(__builtin_isfinite(hacc[0]) && __builtin_isfinite(hacc[1]) &&
                              __builtin_isfinite(hacc[2]) && __builtin_isfinite(hacc[3]));
      if (nan_seen && range_flag != nullptr) *range_flag = 1;
    }
    res = f32x4{relu(hacc[3]), sigmoid_ref(hacc[0]), sigmoid_ref(hacc[1]), sigmoid_ref(hacc[2])};
    if constexpr (kTrain) {
      if (sk.valid && lane < 32) {
        ((f32x4*)tro.rgbs)[p0] = f32x4{res[1], res[2], res[3], res[0]};
        tro.hc[p0 * 132 + 128] = res[0];
      }
    } else {
      if (fused) {
        const f32x2_t in = *(const f32x2_t*)seg_slot;
        float wl;
        res = seg_composite(res, in[0], in[1], lane, wl);
      }
      res_p0 = p0;
    }
  }
  store();
  wait_vmcnt(0);   // the stream ran into a tile that does not exist: let it land
}

// NERF_X3_LAB (timing builds of make variant_x3 only): instantiate just the f16
// render-pass kernel, so a variant compiles in a fifth of the time.
template <class Op>
hipError_t launch_x3(const void* blob, const float* params, const SampleSrc& src, long n_points, float* out,
                     bool explicit_points, hipStream_t stream, float* seg, int* range_flag, int layout = 0) {
#ifdef NERF_X3_LAB
  if (explicit_points || !__is_same(Op, OpF16)) return hipErrorNotSupported;
#endif
  if (n_points <= 0) return hipSuccess;
  if (seg != nullptr && (explicit_points || src.n_samples % kSamplesPerWave != 0)) return hipErrorInvalidValue;
  const long tiles = (n_points + kSamplesPerBlock - 1) / kSamplesPerBlock;
  const long blocks = tiles < current_device_cus() ? tiles : current_device_cus();   // one workgroup per CU
  const dim3 grid{unsigned(blocks), 1, 1}, block{kThreads, 1, 1};
  if (layout != 0) {   // NERF_LAYOUT_ORIGINAL_NERF: the split-fp16 unit only
#ifndef NERF_X3_LAB
    if constexpr (__is_same(Op, OpF16)) {
      if (layout != 1) return hipErrorInvalidValue;
      if (explicit_points)
        hipLaunchKernelGGL((mlp_x3_kernel<true, false, Op, true>), grid, block, 0, stream, (const char*)blob, params,
                           src, n_points, (f32x4*)out, (f32x4*)nullptr, X3TrainOut{}, range_flag);
      else
        hipLaunchKernelGGL((mlp_x3_kernel<false, false, Op, true>), grid, block, 0, stream, (const char*)blob, params,
                           src, n_points, (f32x4*)out, (f32x4*)seg, X3TrainOut{}, range_flag);
      return hipGetLastError();
    }
#endif
    return hipErrorNotSupported;
  }
#ifndef NERF_X3_LAB
  if (explicit_points)
    hipLaunchKernelGGL((mlp_x3_kernel<true, false, Op>), grid, block, 0, stream, (const char*)blob, params, src,
                       n_points, (f32x4*)out, (f32x4*)nullptr, X3TrainOut{}, range_flag);
  else
#endif
    hipLaunchKernelGGL((mlp_x3_kernel<false, false, Op>), grid, block, 0, stream, (const char*)blob, params, src,
                       n_points, (f32x4*)out, (f32x4*)seg, X3TrainOut{}, range_flag);
  return hipGetLastError();
}

}  // namespace
}  // namespace nerf
