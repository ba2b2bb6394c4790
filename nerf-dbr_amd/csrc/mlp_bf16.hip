// bf16 NeRF MLP on gfx950 (v_mfma_f32_32x32x16_bf16, fp32 accumulate): the
// throughput path.
//
// Replaces NeRFModel.forward (src/models/nerf.py:92-131) fused with
// sample_points_on_rays (src/benchmark/base_renderer.py:260-281) and the
// positional encoding (nerf.py:24-45).  Activations and weights are rounded to
// bf16 (RNE) at MFMA inputs; accumulation, bias, ReLU and everything outside the
// MLP stay fp32.  The density and colour heads run on the MFMA too, as one extra
// 32-row tile after C0 (nerf_layout.h kHeadUnits): their fp32 VALU form was
// ~450 instructions per wave, and this kernel's time tracks its VALU count.
//
// Geometry: workgroups of 256 samples.  The shipped build (round 5, Makefile:
// NERF_BF16_WAVES=4, VGPR-form, NERF_BF16_SCHED=2) runs 4 waves, one per SIMD, each
// owning two 32-sample column tiles, so every A fragment read from LDS feeds both
// columns' MFMAs; a lane keeps both columns' accumulator tiles (VGPRs) and B fragments
// (AGPRs), 442 registers, no scratch.  The source default (NERF_BF16_WAVES=8) is the
// rounds 1-4 form: 8 waves, two per SIMD, one column each (128 accumulator + 64
// fragment VGPRs).  Activations never leave registers (nerf_layout.h); the position and
// direction encodings wait in LDS for the layers that take them.  Timing ablations and
// the other lab variants of round 1 are not part of this source.
//
// Quarter schedule.  Each layer is issued in quarters of two output tiles.
// A layer's output tiles are converted to the next layer's bf16 fragments
// (ReLU'd) while the layer is still running: tiles 2q-2, 2q-1 during quarter
// q, tiles 6-7 in the next layer's quarter 0, one dword (two values) per unit,
// so the conversion is about one VALU per MFMA to issue under the other MFMAs
// (see layer_bf16).
//
// Weight stream.  The packed blob is a sequence of 2 KiB units (layer, quarter,
// k-step) cut into 16 KiB chunks.  A 3-slot LDS ring is filled by
// global_load_lds_dwordx4 (lane-linear 1 KiB pieces, issued from inline asm)
// two chunks ahead.  One raw s_barrier per chunk, placed where the fragment
// prefetch first reaches into the next chunk, both publishes that chunk (after
// a counted vmcnt for this wave's own pieces) and frees the slot of the chunk
// before, which is restaged right away.  Fragments are prefetched two units
// ahead through a 3-entry register ring; every LDS read in the loop is inline
// asm, and each unit waits once, with a compile-time lgkmcnt, for exactly the
// reads its MFMAs consume.
//
// Persistent tiles.  One workgroup per CU loops over 256-sample tiles.  The
// weight stream never stops: a tile's last seams stage the next tile's first
// chunks (the stream length is a multiple of the ring, so chunk g always uses
// slot g % kSlots), so the ring does not refill per tile, the parameters are
// copied once, and no workgroup launch gap remains.  Each wave re-encodes its
// own samples into its own LDS slots at the top of a tile; one barrier there
// publishes chunk 0.
#include "nerf_asm.h"
#include "nerf_device.h"
#include "nerf_internal.h"

namespace nerf {
namespace {

#ifndef NERF_BF16_WAVES
#define NERF_BF16_WAVES 8            // 8: two waves per SIMD, 32 samples each; 4: one per SIMD, 64 each
#endif
constexpr int kWaves = NERF_BF16_WAVES;
constexpr int kThreads = 64 * kWaves;
constexpr int kCols = 8 / kWaves;                                     // column tiles per wave
static_assert(kCols == 1 || kCols == 2, "4 or 8 waves");
constexpr int kSamplesPerBlock = kWaves * kCols * kSamplesPerWave;    // 256
// Ring geometry (compile-time knobs, swept with tools/kernel_lab.py).
#ifndef NERF_BF16_CHUNK_UNITS
#define NERF_BF16_CHUNK_UNITS 8      // 2 KiB units per LDS chunk (one barrier per chunk)
#endif
#ifndef NERF_BF16_SLOTS
#define NERF_BF16_SLOTS 3            // chunk slots in the LDS ring (chunks in flight: kSlots - 1)
#endif
#ifndef NERF_BF16_PF
#define NERF_BF16_PF 2               // fragment prefetch distance (units)
#endif
constexpr int kUnits = kHeadUnitBase + kHeadUnits;                   // 516 layer units + 12 head units
constexpr int kChunkUnits = NERF_BF16_CHUNK_UNITS;
constexpr int kChunkB = kChunkUnits * kUnitBytes;
constexpr int kTotalChunks = (kUnits + kChunkUnits - 1) / kChunkUnits;
constexpr int kSlots = NERF_BF16_SLOTS;
constexpr int kPf = NERF_BF16_PF;
constexpr int kRing = kPf + 1;
constexpr int kGldsPerStage = kChunkB / (kThreads * 16);              // LDS-DMA pieces per wave per chunk
constexpr int kLdsParamOff = kSlots * kChunkB;
static_assert(kSlots >= 3 && kPf <= kChunkUnits, "prefetch reaches at most one published chunk ahead");
static_assert(kTotalChunks % kSlots == 0, "the stream runs on into the next tile: chunk g of every tile uses slot g % kSlots");
static_assert(kTotalChunks * kChunkB <= kBf16BlobBytes, "device blob is padded for every chunk geometry");
constexpr int kLdsPeOff = kLdsParamOff + ((kParamFloats * 4 + 1023) / 1024) * 1024;
constexpr int kLdsDeOff = kLdsPeOff + kWaves * kCols * 4 * 1024;
constexpr int kLdsSegOff = kLdsDeOff + kWaves * kCols * 2 * 1024;       // fused compositing: (dist, z) per sample
constexpr int kLdsBytes = kLdsSegOff + kWaves * kCols * kSamplesPerWave * 8;
static_assert(kLdsParamOff % 16 == 0 && kLdsPeOff % 16 == 0, "LDS carve must stay 16-B aligned");
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
static_assert(kGldsPerStage * kThreads * 16 == kChunkB, "stage geometry");

typedef __attribute__((address_space(3))) void lds_void;
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// ---- compile-time unit map (constant-folded after unrolling) ----
NL_HD int unit_layer(int n) {
  int l = 0;
  while (l + 1 < kNumMfmaLayers && bf16_unit_base(l + 1) <= n) ++l;
  return l;
}
NL_HD bool unit_is_head(int n) { return n >= kHeadUnitBase; }
NL_HD int unit_kstep(int n) { return (n - bf16_unit_base(unit_layer(n))) % ksteps_bf16(unit_layer(n)); }
NL_HD int unit_extra(int n) {   // 0: B from hidden fragments (or head units); else the Extra kind
  if (unit_is_head(n)) return 0;
  const int l = unit_layer(n);
  return unit_kstep(n) < layer_shape(l).hidden / 16 ? 0 : layer_shape(l).extra;
}

// Chunk g -> ring slot g % kSlots.  Each wave moves its share as lane-linear
// 1 KiB LDS-DMA pieces (destination = wave-uniform base + lane*16).
__device__ __forceinline__ void stage_chunk(const char* __restrict__ blob, int g, char* lds, int wave_u, int lane) {
  char* dst = lds + (g % kSlots) * kChunkB + wave_u * 1024;
#pragma unroll
  for (int i = 0; i < kGldsPerStage; ++i) {
    // issued from inline asm (nerf_asm.h): the builtin makes hipcc emit lgkmcnt(0)
    // before every fragment use; completion is tracked by counted vmcnt + barrier
    lds_dma_16_s(blob + size_t(g) * kChunkB, unsigned(wave_u * 1024 + lane * 16 + i * kThreads * 16),
                 lds_addr(dst + i * kThreads * 16));
  }
}

__device__ __forceinline__ bf16x8 pack8(const float* v) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
  return r;
}

// ReLU after rounding, on the packed bf16 words: RNE rounding preserves sign
// and order, so relu(bf16(x)) == bf16(relu(x)) bit for bit, and a bf16 is
// negative exactly when its bit pattern is a negative int16 -> v_pk_max_i16
// with 0 (one instruction per two values, no fp32 canonicalisation).
__device__ __forceinline__ unsigned cvt_relu_pair(float lo, float hi) {
  const bf16x2 p = __builtin_convertvector(f32x2{lo, hi}, bf16x2);                    // v_cvt_pk_bf16_f32
  const i16x2 m = __builtin_elementwise_max(__builtin_bit_cast(i16x2, p), i16x2(0));   // v_pk_max_i16
  return __builtin_bit_cast(unsigned, m);
}


struct Ctx {
  const char* blob;
  char* lds;
  int wave_u, lane, h;
  // LDS byte addresses of this lane's 16 B in the ring, in this wave's position /
  // direction encodings, and of this lane half's bias rows (asm reads add an
  // immediate offset)
  unsigned ring_addr, pe_addr, de_addr, bias_addr;
  u32x4* stg;            // NERF_BF16_REGSTAGE: this wave's pieces of the chunk in flight (VGPRs)
  unsigned stg_addr;     // NERF_BF16_REGSTAGE: LDS address of this lane's 16 B in slot 0, piece 0
};

// NERF_BF16_REGSTAGE: chunk g's pieces -> this wave's staging VGPRs (vmcnt), and from
// them into ring slot g % kSlots (lgkmcnt).  The asm outputs count as written at
// issue; the seams wait vmcnt before the writes read them.
__device__ __forceinline__ void load_chunk_regs(const Ctx& cx, int g) {
#pragma unroll
  for (int i = 0; i < kGldsPerStage; ++i) {
    const unsigned long long sb = (unsigned long long)(cx.blob + size_t(g) * kChunkB + i * kThreads * 16);
    const unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(sb)), hi = __builtin_amdgcn_readfirstlane(unsigned(sb >> 32));
    const unsigned long long s64 = (unsigned long long)lo | ((unsigned long long)hi << 32);
    asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(cx.stg[i]) : "v"(unsigned(cx.wave_u * 1024 + cx.lane * 16)),
                 "s"(s64) : "memory");
  }
}
__device__ __forceinline__ void write_chunk_regs(const Ctx& cx, int g) {
#pragma unroll
  for (int i = 0; i < kGldsPerStage; ++i)
    asm volatile("ds_write_b128 %0, %1 offset:%2" :: "v"(cx.stg_addr), "v"(cx.stg[i]),
                 "i"((g % kSlots) * kChunkB + i * kThreads * 16) : "memory");
}

// ---- LDS fragment reads from inline asm with counted waits.  Left to itself
// hipcc puts an s_waitcnt in front of almost every MFMA (one per fragment);
// here each unit waits once, for exactly the reads it consumes: everything the
// loop reads from LDS (fragments, encodings, biases) is issued below, so the
// count of younger reads is known at compile time.  An asm destination counts
// as written at the asm statement, so each wait is followed by a
// sched_barrier that keeps the consuming MFMAs behind it (§5.7 rule 18).
NL_HD int unit_reads(int n) { return n < 0 || n >= kUnits ? 0 : 2 + (unit_extra(n) != 0 ? kCols : 0); }

// Issue order per unit body m: [bias reads if m opens a quarter], reads of unit
// m+kPf, wait, MFMAs of unit m (the prologue issued units 0..kPf-1).
NL_HD bool unit_opens_quarter(int n) {
  if (unit_is_head(n)) return false;
  const int l = unit_layer(n);
  return (n - bf16_unit_base(l)) % ksteps_bf16(l) == 0;
}
// NERF_BF16_REGSTAGE (lab knob): the weight stream is staged through registers instead
// of LDS-DMA -- each wave loads its pieces of a chunk into VGPRs at one seam
// (global_load_dwordx4) and writes them to the ring at the next (ds_write_b128), so
// those ds_writes join the LDS counts.
#ifndef NERF_BF16_REGSTAGE
#define NERF_BF16_REGSTAGE 0
#endif
NL_HD bool is_seam(int n) { return (n + kPf) % kChunkUnits == 0 && n + kPf < kUnits && n + kPf != 0; }
NL_HD int seam_writes(int m) { return NERF_BF16_REGSTAGE && m >= 0 && m < kUnits && is_seam(m) ? kGldsPerStage : 0; }
// writes of the seams in bodies n-kPf+1 .. n: younger than unit n's reads (issued in body n-kPf)
NL_HD int seam_writes_since(int n) {
  int c = 0;
  for (int m = n - kPf + 1; m <= n; ++m) c += seam_writes(m);
  return c;
}
constexpr int kBiasReads = 8 * kCols;   // 2 tiles x 4 x 16 B, per column
NL_HD int bias_reads(int m) { return m >= 0 && m < kUnits && unit_opens_quarter(m) ? kBiasReads : 0; }
// LDS reads younger than everything unit n consumes, at its wait
NL_HD int lgkm_for_unit(int n) {
  if (unit_opens_quarter(n)) return unit_reads(n + kPf);      // this body's bias is the youngest need
  int c = 0;
  for (int k = n + 1; k <= n + kPf; ++k) c += unit_reads(k);
  for (int m = n - kPf + 1; m <= n; ++m) c += bias_reads(m);
  return c + seam_writes_since(n);
}

// Reads of unit n into ring entry n % kRing: two A fragments (output tiles of
// the unit's quarter) and, for encoding inputs, the two columns' B fragments.
__device__ __forceinline__ void read_unit(const Ctx& cx, int n, bf16x8 (&ra)[kRing][2], bf16x8 (&rb)[kRing][kCols]) {
  static_assert(kSlots * kChunkB <= 65536, "ring offsets must fit the ds_read offset field");
  const int slot_off = ((n / kChunkUnits) % kSlots) * kChunkB + (n % kChunkUnits) * kUnitBytes;
  ra[n % kRing][0] = ds_read_b128<bf16x8>(cx.ring_addr, slot_off);
  ra[n % kRing][1] = ds_read_b128<bf16x8>(cx.ring_addr, slot_off + 1024);
  const int ex = unit_extra(n);
  if (ex != 0) {
    const int u = unit_kstep(n) - layer_shape(unit_layer(n)).hidden / 16;
#pragma unroll
    for (int c = 0; c < kCols; ++c)
      rb[n % kRing][c] = ex == kPos ? ds_read_b128<bf16x8>(cx.pe_addr, (4 * c + u) * 1024)
                                    : ds_read_b128<bf16x8>(cx.de_addr, (2 * c + u) * 1024);
  }
}

// Seam E_g, at the top of unit n when its prefetch (unit n+kPf) is the first
// unit of chunk g+1.  Every read of chunk g-1 was consumed by MFMAs of earlier
// units (so no lgkmcnt wait), so after the barrier its slot is free:
//   (1) own LDS-DMA pieces of chunk g+1 landed (counted vmcnt; chunk g+1 was
//       staged kSlots-2 seams earlier, and kSlots-3 younger stages are in flight),
//   (2) s_barrier: chunk g+1 is published and every wave is past chunk g-1,
//   (3) stage chunk g+kSlots-1 into chunk g-1's slot -- past the end of the
//       tile, the next tile's chunk of the same slot.
// The top of a tile is seam E_-1 (tile_top).
constexpr int kDmaOutstandingAtSeam = kSlots - 3;
constexpr int kStageAhead = kSlots - 1;   // seam g stages chunk g + kStageAhead
static_assert(!NERF_BF16_REGSTAGE || kSlots == 3, "register staging: chunk g+2 written at seam g into chunk g-1's slot");
__device__ __forceinline__ void seam_before(const Ctx& cx, int n) {
  if (!is_seam(n)) return;
  const int g = (n + kPf) / kChunkUnits - 1;
  if (NERF_BF16_REGSTAGE) {   // chunk g+2 (loaded at seam g-1) -> the slot chunk g-1 frees; load chunk g+3
    wait_vmcnt(0);
    compiler_fence();
    __builtin_amdgcn_s_barrier();
    compiler_fence();
    write_chunk_regs(cx, (g + kStageAhead) % kTotalChunks);
    load_chunk_regs(cx, (g + kStageAhead + 1) % kTotalChunks);
    return;
  }
  wait_vmcnt(kGldsPerStage * kDmaOutstandingAtSeam);
  compiler_fence();
  __builtin_amdgcn_s_barrier();
  compiler_fence();
  stage_chunk(cx.blob, (g + kStageAhead) % kTotalChunks, cx.lds, cx.wave_u, cx.lane);
}
// Conversion schedule (default): layer L's output tiles 2q-2, 2q-1 become final
// at the end of its quarter q-1 and are converted to the next layer's B
// fragments (bout) in four half-tile slices during quarter q = 1..3; tiles 6, 7
// follow in the next layer's quarter 0 (into its bin, before k-step 12 reads
// them).  Two tiles per quarter, nothing exposed at the layer boundary, and each
// fp32 tile dies as soon as it is packed.
// Slice j (0..3) of a quarter runs at unit kSlicePos(KU, j).
NL_HD int slice_pos(int ku, int j) { return ku >= 12 ? 2 + 3 * j : j; }
// Finer still for the layers without a density head: one dword (two values,
// one v_cvt_pk_bf16_f32 + one v_pk_max_i16) per unit, so each wave has about
// one conversion instruction per MFMA to issue under the other MFMAs instead
// of a 16-instruction burst.  Dword m (0..15) of a tile pair: tile m>>3,
// register pair m&7 -> fragment (m&7)>>2, dword m&3.
NL_HD int dword_unit_out(int ku, int m) { return ku >= 16 ? 2 + (m * (ku - 2)) / 16 : m / 4; }   // quarters 1..3
NL_HD int dword_unit_in(int m) { return 2 + (m * 10) / 16; }                                     // quarter 0, < 12
__device__ __forceinline__ void convert_dword(const f32x16& tile, int pr, u32x4& frag) {
  frag[pr & 3] = cvt_relu_pair(tile[2 * pr], tile[2 * pr + 1]);
}

// Bias pre-load of quarter q of layer l (tiles 2q, 2q+1), straight into the
// accumulators (param blob [layer][tile][half][16]); l, q constant after unrolling.
__device__ __forceinline__ void issue_bias(const Ctx& cx, int l, int q, f32x16 (&acc)[kCols][8]) {
#pragma unroll
  for (int o2 = 0; o2 < 2; ++o2)
#pragma unroll
    for (int c = 0; c < kCols; ++c) {
      const int off = 4 * (kBiasOff + 256 * l + (2 * q + o2) * 32);
      const f32x4 b0 = ds_read_b128<f32x4>(cx.bias_addr, off), b1 = ds_read_b128<f32x4>(cx.bias_addr, off + 16);
      const f32x4 b2 = ds_read_b128<f32x4>(cx.bias_addr, off + 32), b3 = ds_read_b128<f32x4>(cx.bias_addr, off + 48);
      acc[c][2 * q + o2] = f32x16{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3],
                                  b2[0], b2[1], b2[2], b2[3], b3[0], b3[1], b3[2], b3[3]};
    }
}

// NERF_BF16_SCHED (lab knob): an explicit issue pattern for a unit body's scheduling region
// (sched_group_barrier), per MFMA: 1: 1 MFMA, 1 DS read, 1 VALU; 2: 1 MFMA, 2 VALU, 1 DS read;
// 3: 1 MFMA, 3 VALU, 1 DS read; 4: 1 MFMA, 1 VALU, 1 DS read, 1 VALU.
#ifndef NERF_BF16_SCHED
#define NERF_BF16_SCHED 0
#endif
__device__ __forceinline__ void sched_unit_pattern() {
#pragma unroll
  for (int i = 0; i < 2 * kCols; ++i) {
    if (NERF_BF16_SCHED == 1) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    } else if (NERF_BF16_SCHED == 2) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    } else if (NERF_BF16_SCHED == 3) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    } else if (NERF_BF16_SCHED == 4) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
    }
  }
}

template <int L>
__device__ __forceinline__ void layer_bf16(f32x16 (&acc)[kCols][8], u32x4 (&bh)[kCols][16], u32x4 (&bout)[kCols][16],
                                           bf16x8 (&ra)[kRing][2], bf16x8 (&rb)[kRing][kCols], const Ctx& cx) {
  constexpr LayerShape sh = layer_shape(L);
  constexpr int KH = sh.hidden / 16;
  constexpr int KU = ksteps_bf16(L);
  constexpr int NQ = out_tiles(L) / 2;
  constexpr int N0 = bf16_unit_base(L);
  constexpr bool kConvert = L != L0;          // B fragments come from the previous layer
  // outputs feed another MFMA layer: the next layer, or (C0) the heads' tile;
  // C0 has two quarters, so its tiles 2, 3 are converted in the head loop
  constexpr bool kConvertOut = true;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int n = N0 + q * KU + u;
      seam_before(cx, n);
      if (u == 0) issue_bias(cx, L, q, acc);   // this quarter's bias (waited with its first unit)
      if (n + kPf < kUnits) read_unit(cx, n + kPf, ra, rb);
      wait_lgkm(lgkm_for_unit(n));
      // keep the prefetch reads here: left alone, the scheduler sinks them next
      // to their MFMAs and every unit then waits out the LDS latency
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 b[kCols];
#pragma unroll
      for (int c = 0; c < kCols; ++c)
        b[c] = u < KH ? __builtin_bit_cast(bf16x8, bh[c][u < KH ? u : 0]) : rb[n % kRing][c];
#pragma unroll
      for (int o2 = 0; o2 < 2; ++o2)
#pragma unroll
        for (int c = 0; c < kCols; ++c)
          acc[c][2 * q + o2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[n % kRing][o2], b[c], acc[c][2 * q + o2],
                                                                      0, 0, 0);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int t = m >> 3, pr = m & 7;
        if (kConvert && q == 0 && u == dword_unit_in(m))
#pragma unroll
          for (int c = 0; c < kCols; ++c) convert_dword(acc[c][6 + t], pr, bh[c][2 * (6 + t) + (pr >> 2)]);
        if (kConvertOut && q >= 1 && u == dword_unit_out(KU, m))
#pragma unroll
          for (int c = 0; c < kCols; ++c)
            convert_dword(acc[c][2 * q - 2 + t], pr, bout[c][2 * (2 * q - 2 + t) + (pr >> 2)]);
      }
      if (NERF_BF16_SCHED) sched_unit_pattern();
    }
  }
}

// (sigma, r, g, b) of a tile's samples, or with fused compositing (seg) each
// column's segment record (nerf_device.h SegRecord, lanes 0 and 1); p0 < 0:
// nothing pending
__device__ __forceinline__ void store_results(const f32x4 (&res)[kCols], const float (&wl)[kCols], long p0,
                                              long n_points, int lane, f32x4* __restrict__ out,
                                              f32x4* __restrict__ seg, float* __restrict__ wloc) {
  if (p0 < 0) return;
#pragma unroll
  for (int c = 0; c < kCols; ++c) {
    const long p = p0 + c * kSamplesPerWave;
    if (seg) {
      const long first = p - (lane & 31);                 // the segment's first sample
      if (first < n_points && lane < 2) seg[(first / kSamplesPerWave) * 2 + lane] = res[c];
      if (wloc != nullptr && p < n_points && lane < 32) wloc[p] = wl[c];
    } else if (p < n_points && lane < 32) {
      out[p] = res[c];
    }
  }
}

template <bool kExplicit>
__global__ __launch_bounds__(kThreads, 1) void mlp_bf16_kernel(const char* __restrict__ blob,
                                                               const float* __restrict__ prm_g, SampleSrc src,
                                                               long n_points, f32x4* __restrict__ out,
                                                               f32x4* __restrict__ seg, float* __restrict__ wloc) {
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  const int lane = threadIdx.x & 63;
  const int wave_u = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5;
  const unsigned lds_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)lds;
  u32x4 stg[kGldsPerStage];
  const Ctx cx0{blob, lds, wave_u, lane, h, lds_base + lane * 16,
               lds_base + kLdsPeOff + wave_u * kCols * 4096 + lane * 16,
               lds_base + kLdsDeOff + wave_u * kCols * 2048 + lane * 16,
               lds_base + kLdsParamOff + h * 64, stg, lds_base + wave_u * 1024 + lane * 16};
  const long n_tiles = (n_points + kSamplesPerBlock - 1) / kSamplesPerBlock;

  // Start the weight stream (chunks 0 .. kSlots-3; each tile's top stages one
  // more) and copy the parameters, once per workgroup.
  if (NERF_BF16_REGSTAGE) {   // chunk 0 written now, chunk 1 loaded (written at the tile top)
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

  // A tile's results are stored at the top of the next tile, after its seam:
  // vmcnt counts stores with the LDS-DMA in issue order, so a store issued last
  // would make the next tile's first wait also wait out the store.
  f32x4 res[kCols];
  float wl[kCols];
  long res_p0 = -1;

#pragma unroll 1
  for (long tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const long p0 = (tile * kWaves + wave_u) * (kCols * kSamplesPerWave) + (lane & 31);
    // an opaque copy of the stream base per tile: otherwise the 66 chunk
    // addresses (blob + constant) are hoisted out of the tile loop and held in
    // SGPRs (spilling); recomputing each is one scalar add pair at its stage
    Ctx cx = cx0;
    asm volatile("" : "+s"(cx.blob));
    // This tile's encodings, into this wave's own LDS slots (its reads of the
    // previous tile's were waited for before their MFMAs).
#pragma unroll 1
    for (int c = 0; c < kCols; ++c) {
      const long p = p0 + c * kSamplesPerWave;
      float x[3], d[3], pef[32], def[16];
      float dist = 0.0f, zz = 0.0f;
      if (kExplicit) fetch_sample<true>(src, p < n_points ? p : n_points - 1, x, d);
      else fetch_render_sample(src, p < n_points ? p : n_points - 1, n_points <= 0xFFFFFFFFL, seg != nullptr, x, d, dist, zz);
      pos_encode<true>(x[0], x[1], x[2], h, pef);
      dir_encode<true>(d[0], d[1], d[2], h, def);
      char* pe_dst = lds + kLdsPeOff + (wave_u * kCols + c) * 4096 + lane * 16;
      char* de_dst = lds + kLdsDeOff + (wave_u * kCols + c) * 2048 + lane * 16;
#pragma unroll
      for (int u = 0; u < 4; ++u) *(bf16x8*)(pe_dst + u * 1024) = pack8(pef + 8 * u);
      *(bf16x8*)(de_dst) = pack8(def);
      *(bf16x8*)(de_dst + 1024) = pack8(def + 8);
      if (!kExplicit && seg != nullptr) {   // the integral's network-independent inputs (nerf_device.h)
        if (h == 0) *(f32x2_t*)(lds + kLdsSegOff + ((wave_u * kCols + c) * kSamplesPerWave + (lane & 31)) * 8) = f32x2_t{dist, zz};
      }
    }

    // Seam E_-1: chunk 0 landed (own pieces) and is published, parameters too
    // on the first tile; chunk kSlots-2 starts loading into its slot, whose
    // previous chunk every wave finished with the last tile.
    wait_vmcnt(kGldsPerStage * kDmaOutstandingAtSeam);
    __syncthreads();
    if (NERF_BF16_REGSTAGE) {
      write_chunk_regs(cx, kStageAhead - 1);
      load_chunk_regs(cx, kStageAhead);
    } else {
      stage_chunk(cx.blob, kStageAhead - 1, lds, wave_u, lane);
    }
    store_results(res, wl, res_p0, n_points, lane, out, seg, wloc);
    bf16x8 ra[kRing][2], rb[kRing][kCols];
    f32x16 acc[kCols][8];
#pragma unroll
    for (int n = 0; n < kPf; ++n) read_unit(cx, n, ra, rb);

    // two B-fragment sets: layer l reads one while it fills the other for l+1
    u32x4 bA[kCols][16], bB[kCols][16];
    layer_bf16<L0>(acc, bB, bA, ra, rb, cx);
    layer_bf16<L1>(acc, bA, bB, ra, rb, cx);
    layer_bf16<L2>(acc, bB, bA, ra, rb, cx);
    layer_bf16<L3>(acc, bA, bB, ra, rb, cx);
    layer_bf16<L4>(acc, bB, bA, ra, rb, cx);   // skip: [x, pe] (nerf.py:109-110)
    layer_bf16<L5>(acc, bA, bB, ra, rb, cx);
    layer_bf16<L6>(acc, bB, bA, ra, rb, cx);
    layer_bf16<L7>(acc, bA, bB, ra, rb, cx);
    layer_bf16<C0>(acc, bB, bA, ra, rb, cx);   // [x, PE4(d)] (nerf.py:117-121)

    // Heads (nerf.py:114, 123-129) as one MFMA tile: rows 0-2 colour, row 3
    // density; k-steps 0..15 over L7's fragments (bB, C0's input), 16..23 over
    // C0's output (bA[0..3] converted in C0's quarter 1, bA[4..7] below).
    f32x16 hacc[kCols];
#pragma unroll
    for (int c = 0; c < kCols; ++c) {
      hacc[c] = f32x16{};
      if (h == 0) {
        hacc[c][0] = prm[kC1B];
        hacc[c][1] = prm[kC1B + 1];
        hacc[c][2] = prm[kC1B + 2];
        hacc[c][3] = prm[kSigB];
      }
    }
#pragma unroll
    for (int i = 0; i < kHeadUnits; ++i) {
      const int n = kHeadUnitBase + i;
      seam_before(cx, n);
      if (n + kPf < kUnits) read_unit(cx, n + kPf, ra, rb);
      // head units read two fragments each and no bias: the younger reads are
      // those of the next min(kPf, units left) units (spelled out so it folds)
      wait_lgkm(2 * (kUnits - 1 - n < kPf ? kUnits - 1 - n : kPf) + seam_writes_since(n));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int k = 2 * i + s2;
#pragma unroll
        for (int c = 0; c < kCols; ++c) {
          const bf16x8 b = __builtin_bit_cast(bf16x8, k < 16 ? bB[c][k < 16 ? k : 0] : bA[c][k >= 16 ? k - 16 : 0]);
          hacc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ra[n % kRing][s2], b, hacc[c], 0, 0, 0);
        }
      }
      // C0's tiles 2, 3 -> colour k-steps 20..23 (bA[4..7]), two dwords per unit
#pragma unroll
      for (int m = 0; m < 16; ++m)
        if (i < 8 && m / 2 == i)
#pragma unroll
          for (int c = 0; c < kCols; ++c) convert_dword(acc[c][2 + (m >> 3)], m & 7, bA[c][2 * (2 + (m >> 3)) + ((m & 7) >> 2)]);
    }
#pragma unroll
    for (int c = 0; c < kCols; ++c) {
      res[c] = f32x4{relu(hacc[c][3]), sigmoid_ref(hacc[c][0]), sigmoid_ref(hacc[c][1]), sigmoid_ref(hacc[c][2])};
      if (!kExplicit && seg != nullptr) {
        const f32x2_t in = *(const f32x2_t*)(lds + kLdsSegOff + ((wave_u * kCols + c) * kSamplesPerWave + (lane & 31)) * 8);
        res[c] = seg_composite(res[c], in[0], in[1], lane, wl[c]);
      }
    }
    res_p0 = p0;
  }
  store_results(res, wl, res_p0, n_points, lane, out, seg, wloc);
  // the stream ran kSlots-2 chunks into a tile that does not exist: let them
  // land before the workgroup's LDS is released
  wait_vmcnt(0);
}

}  // namespace

hipError_t launch_mlp_bf16(const void* blob, const float* params, const SampleSrc& src, long n_points, float* out,
                           bool explicit_points, hipStream_t stream, float* seg, float* wloc) {
  if (n_points <= 0) return hipSuccess;
  const long tiles = (n_points + kSamplesPerBlock - 1) / kSamplesPerBlock;
  const long blocks = tiles < current_device_cus() ? tiles : current_device_cus();   // one workgroup per CU
  if (blocks > 0x7FFFFFFFL) return hipErrorInvalidValue;
  const dim3 grid{unsigned(blocks), 1, 1}, block{kThreads, 1, 1};
  if (explicit_points)
    hipLaunchKernelGGL(mlp_bf16_kernel<true>, grid, block, 0, stream, (const char*)blob, params, src, n_points,
                       (f32x4*)out, (f32x4*)seg, wloc);
  else
    hipLaunchKernelGGL(mlp_bf16_kernel<false>, grid, block, 0, stream, (const char*)blob, params, src, n_points,
                       (f32x4*)out, (f32x4*)seg, wloc);
  return hipGetLastError();
}

}  // namespace nerf
