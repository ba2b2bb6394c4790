// fp8 (OCP e4m3) NeRF MLP on gfx950, mixed with bf16: the compressed-weights path
// (BASELINE config 5).  The reference's counterpart is the int8 CompressedNeRFRenderer
// (src/benchmark/compressed_renderer.py:89-211, 233-269), whose error against the
// reference's fp32 render is the bar this path has to clear.
//
// Round 5: L2, L3, L5, L6, L7 and L4's hidden k-steps run on the block-scaled fp8 MFMA
// (v_mfma_scale_f32_32x32x64_f8f6f4, e4m3 operands); L0 and L1 (the layers whose errors
// every later layer amplifies), L4's encoding k-steps, C0 and both heads on the bf16 MFMA
// (v_mfma_f32_32x32x16_bf16); all encodings are bf16.  On the Lego checkpoint this is the
// cheapest set of bf16 layers at which the render is at least as close to the reference's
// fp32 render as the reference's int8 renderer, in max and mean RGB (tools/fp8_mixed_lab.py;
// the all-fp8 network of rounds 1-4 was 1.9x / 1.2x further off than int8 on Lego).  74.5 %
// of the MACs stay fp8: the ceiling for this mix is 3.98 PFLOP/s (the fp8 part at 5, the
// bf16 part at 2.5).
//
// Same orientation and schedule as mlp_bf16.hip (nerf_layout.h): H^T = W . X^T on 32x32
// tiles, the accumulator of one layer is the B operand of the next, 8 waves x 32 samples,
// quarter schedule, an LDS ring filled by LDS-DMA with one barrier per chunk,
// compiler-counted fragment reads; waves 4-7 run one chunk behind waves 0-3 (the wave lag
// below), and one workgroup per CU loops over the tiles with the weight stream running on.
// The stream is 4 KiB units (nerf_layout.h "fp8, mixed"): an fp8 unit is one 64-wide
// k-step of a quarter (two 64-cycle MFMAs), a bf16 unit two 16-wide k-steps (four 32-cycle
// MFMAs), a head unit four k-steps of the head tile -- 128 MFMA cycles each.
//   * fp8 weights are e4m3 with a power-of-two (E8M0) scale per output row, chosen at
//     packing so that no row saturates; the MFMA applies it (scale_a operand);
//   * fp8 activations (the ReLU'd fp32 outputs) are e4m3 at scale 1, saturated: one
//     v_med3_f32(x, 0, 448) per value is the ReLU and the clamp (e4m3fn has no infinity and
//     the conversion does not saturate), then v_cvt_pk_fp8_f32 per two values; the MFMA's B
//     scale is 1 (E8M0 127);
//   * bf16 activations: v_cvt_pk_bf16_f32, then the ReLU as v_pk_max_i16 on the words;
//   * a layer's output tiles are converted while it still runs (tiles 2q-2, 2q-1 in quarter
//     q, tiles 6, 7 in the next layer's quarter 0) into the next layer's operand type: one
//     bf16 fragment set (64 VGPRs: L0 -> L1, L7 -> C0 and the density head), two fp8 sets
//     (32 each) between the fp8 layers, the colour set (C0 -> the colour head).
// Bias, ReLU and everything outside the MLP stay fp32.
#include "nerf_asm.h"
#include "nerf_device.h"
#include "nerf_internal.h"

namespace nerf {
namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

static_assert(!NERF_ASM_LDS_READS, "the mixed fp8 kernel reads LDS with compiler-counted loads only");

// NERF_FP8_WAVES: 8 (rounds 1-5) -- two waves per SIMD, one 32-sample column each, waves 4-7
// one chunk behind (the wave lag below); 4 (round 6) -- one wave per SIMD owning two columns,
// so every A fragment read from LDS feeds both columns' MFMAs (the bf16 headline's form)
#ifndef NERF_FP8_WAVES
#define NERF_FP8_WAVES 8
#endif
constexpr int kWaves = NERF_FP8_WAVES;
constexpr int kCols = 8 / kWaves;                                    // column tiles per wave
static_assert(kCols == 1 || kCols == 2, "4 or 8 waves");
constexpr bool kLag = kWaves == 8;                                   // a lagging half of the waves
constexpr int kThreads = 64 * kWaves;
constexpr int kSamplesPerBlock = kWaves * kCols * kSamplesPerWave;   // 256
constexpr int kUnitB = kFp8UnitBytes;                                // 4 KiB
constexpr int kUnits = kMixUnits;                                    // 168
constexpr int kChunkUnits = 4;                                       // 4 KiB units per LDS chunk (one barrier per chunk)
constexpr int kChunkB = kChunkUnits * kUnitB;                        // 16 KiB
constexpr int kTotalChunks = (kUnits + kChunkUnits - 1) / kChunkUnits;   // 42
constexpr int kSlots = 4;
// Wave lag: waves 4-7 run one chunk behind waves 0-3, so the two waves of a SIMD reach
// their layer boundaries (conversions, nothing for the MFMA pipe) at different times.  The
// ring holds one chunk more for the lagging half: every wave stages one chunk ahead of the
// chunk it publishes, and the lagging half's seam for chunk c is barrier instance c + 1 (one
// extra barrier at its start, one at the leading half's end).  (-1.6 % kernel time in round
// 1, bit-identical output.)
//
// Persistent tiles: one workgroup per CU loops over 256-sample tiles and the weight stream
// runs on across them -- a tile's last seams stage the next tile's first chunks -- so the
// ring is never refilled, the parameters and row scales are copied once per workgroup, and
// no workgroup is relaunched.  A tile is kTotalChunks = 42 chunks and 42 = 2 mod 4, so the
// ring slot of a tile's chunk c is (c + rot) mod 4 with rot = 2 * (tile iteration mod 2),
// known only at run time: a fragment read of chunk c uses base ring_lo (= ring + rot slots)
// for c mod 4 in {0, 1} and ring_hi (= ring - rot slots) for {2, 3} with the immediate offset
// of rotation 0 (the ring sits 2 slots above the LDS base, so ring_hi stays a valid
// address), and a stage's LDS slot is a scalar (c + rot) & 3.
constexpr int kGldsPerStage = kChunkB / (kThreads * 16);
// NERF_FP8_AHEAD (4 waves only): a seam stages the chunk 1 (default) or 2 ahead of the one it
// publishes; with 2, the seam waits for its chunk with the next one still in flight.  The
// 4-slot ring has room: at seam c every wave's reads of chunk c - 2 have completed (its MFMAs
// consumed them before the wave reached the seam), so chunk c + 2 takes that slot.
#ifndef NERF_FP8_AHEAD
#define NERF_FP8_AHEAD 1
#endif
constexpr int kAhead = NERF_FP8_AHEAD;
static_assert(kAhead == 1 || (kAhead == 2 && !kLag), "two chunks ahead: the one-wave-per-SIMD form");
#ifndef NERF_FP8_PF
#define NERF_FP8_PF 1
#endif
constexpr int kPf = NERF_FP8_PF;                                     // fragment prefetch distance (units)
constexpr int kRing = kPf + 1;
static_assert(kUnits % kChunkUnits == 0 && kUnits % kRing == 0, "the next tile's unit n uses ring entry n % kRing");
static_assert(kTotalChunks % 2 == 0 && kTotalChunks % kSlots == 2,
              "the ring rotation assumes an even chunk count of 2 mod 4 per tile in a 4-slot ring");
static_assert(kTotalChunks * kChunkB <= kFp8ScaleOff, "ring reads stay inside the padded fragment area");
constexpr int kLdsParamOff = 0;
constexpr int kLdsScaleOff = ((kParamFloats * 4 + 1023) / 1024) * 1024;
constexpr int kLdsRingOff = kLdsScaleOff + kFp8ScaleBytes;
static_assert(kLdsRingOff >= 2 * kChunkB, "ring_hi = ring - 2 slots must stay a valid LDS address");
static_assert(kLdsRingOff % 16 == 0 && kSlots * kChunkB <= 65536, "ring offsets fit the ds_read offset field");
// per wave: the position encoding's 4 bf16 k-steps, then the direction encoding's 2 ([k][lane][16 B])
constexpr int kEncWaveB = 6 * 1024;
constexpr int kDirEncOff = 4 * 1024;
constexpr int kLdsEncOff = kLdsRingOff + kSlots * kChunkB;
constexpr int kLdsSegOff = kLdsEncOff + kWaves * kCols * kEncWaveB;   // fused compositing: (dist, z) per sample
// NERF_FP8_PIPE_ENC (lab knob, 4 waves): the next tile's samples are fetched and encoded during
// this tile's head units (their MFMAs hide the encoding VALU; the tile top then only seams),
// the (dist, z) slots double-buffered by tile parity.  Unit of the head loop that fetches, and
// the two that encode column 0 and 1:
#ifndef NERF_FP8_PIPE_ENC
#define NERF_FP8_PIPE_ENC 0
#endif
#ifndef NERF_FP8_PIPE_FETCH_UNIT
#define NERF_FP8_PIPE_FETCH_UNIT 0
#endif
static_assert(!NERF_FP8_PIPE_ENC || kCols == 2, "the pipelined encodings assume the two-column form");
constexpr int kSegBufB = kWaves * kCols * kSamplesPerWave * 8;
constexpr int kLdsBytes = kLdsSegOff + (NERF_FP8_PIPE_ENC ? 2 : 1) * kSegBufB;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
static_assert(kFp8ScaleBytes % 16 == 0 && kLdsScaleOff % 16 == 0, "16-B aligned carve");

// ---- compile-time unit map, a constexpr table (inside the tile loop LLVM stops
// constant-folding a loop-based map at this body size) ----
enum UnitKind { kUF8 = 0, kUB16 = 1, kUHead = 2 };
struct UnitInfo {
  int layer, kind, q, iu;   // iu: index within the quarter
  int enc, enc_ks;          // B units on an encoding: its kind and first k-step there
};
struct UnitTable {
  UnitInfo u[kUnits];
};
constexpr UnitTable make_unit_table() {
  UnitTable t{};
  for (int n = 0; n < kUnits; ++n) {
    UnitInfo& x = t.u[n];
    if (n >= kMixLayerUnits) {
      x = UnitInfo{-1, kUHead, 0, n - kMixLayerUnits, 0, 0};
      continue;
    }
    int l = 0;
    while (l + 1 < kNumMfmaLayers && mix_unit_base(l + 1) <= n) ++l;
    const int upq = mix_units_per_quarter(l), r = n - mix_unit_base(l);
    const int q = r / upq, iu = r % upq, nf = mix_f8_units(l);
    x = UnitInfo{l, iu < nf ? kUF8 : kUB16, q, iu, 0, 0};
    if (iu >= nf) {
      const int ks = mix_b_kstep(l, iu - nf, 0), kh = layer_shape(l).hidden / 16;
      if (ks >= kh) {
        x.enc = layer_shape(l).extra;
        x.enc_ks = ks - kh;
      }
    }
  }
  return t;
}
constexpr UnitTable kTab = make_unit_table();

struct Ctx {
  const char* blob;
  char* lds;
  unsigned lds_base;                                 // LDS byte address of lds[0]
  int wave_u, lane, h;
  unsigned ring_lo, ring_hi, enc_addr, bias_addr, scale_addr;
  int rot;                                           // ring rotation of this tile (0 or 2), wave-uniform
  int lag;                                           // 1: this wave runs a chunk behind
};

// Stage this wave's pieces of the tile's chunk c (a constant after unrolling; c >= 42 is
// the next tile's chunk c - 42, whose slot the same rotation gives).
// NERF_FP8_ABLATE_* (timing-only lab builds, wrong results): NODMA -- the
// stream is not restaged after the ring's first fill; NOBARRIER -- no seam barriers; NOREAD --
// the ring's first fragments reused; NOCONV -- accumulator bits as the next layer's operands;
// PE_ONCE -- the first tile's encodings reused.
__device__ __forceinline__ void stage_piece(const Ctx& cx, int c, int i) {
#ifdef NERF_FP8_ABLATE_NODMA
  if (c >= kSlots) return;
#endif
  const int slot = (c + cx.rot) & (kSlots - 1);
  const unsigned dst = cx.lds_base + unsigned(kLdsRingOff + slot * kChunkB + cx.wave_u * 1024);
  const int src = c < kTotalChunks ? c : c - kTotalChunks;
  lds_dma_16_s(cx.blob + size_t(src) * kChunkB, unsigned(cx.wave_u * 1024 + cx.lane * 16 + i * kThreads * 16),
               dst + unsigned(i * kThreads * 16));
}
__device__ __forceinline__ void stage_chunk(const Ctx& cx, int c) {
#pragma unroll
  for (int i = 0; i < kGldsPerStage; ++i) stage_piece(cx, c, i);
}
// NERF_FP8_SPREAD (with NERF_FP8_AHEAD=2): a seam stages the first LDS-DMA piece of its chunk and
// the next units one piece each, instead of all of the wave's pieces back to back at the seam.
#ifndef NERF_FP8_SPREAD
#define NERF_FP8_SPREAD 0
#endif
static_assert(!NERF_FP8_SPREAD || (kAhead == 2 && kGldsPerStage <= kChunkUnits),
              "spread pieces land within the chunk after the next seam");

// Seam before this wave's first read of the tile's chunk c: its own pieces of c landed
// (nothing younger is in flight: vmcnt(0)), the barrier publishes c to every wave and frees
// the slot of chunk c - 3 (the lagging half finished it a barrier ago), which takes chunk
// c + 1 (leading half) or c + 2 (lagging half): at barrier instance k both halves stage
// global chunk k + 1.
__device__ __forceinline__ void seam(const Ctx& cx, int c) {
  wait_vmcnt(kAhead == 2 ? kGldsPerStage : 0);
  compiler_fence();
#ifndef NERF_FP8_ABLATE_NOBARRIER
  __builtin_amdgcn_s_barrier();
#endif
  compiler_fence();
  if (NERF_FP8_SPREAD) stage_piece(cx, c + kAhead, 0);
  else stage_chunk(cx, c + kAhead + cx.lag);
}
// The seam inside the unit sequence: before unit body n when its prefetch (unit n + kPf)
// is the first unit of a chunk.
NL_HD bool seam_unit(int m) { return m >= 0 && (m + kPf) % kChunkUnits == 0 && m + kPf < kUnits; }
__device__ __forceinline__ void seam_before(const Ctx& cx, int n) {
  if (NERF_FP8_SPREAD) {   // the pieces 1.. of the chunk the seam i units back staged (-1: the tile top)
#pragma unroll
    for (int i = 1; i < kGldsPerStage; ++i) {
      const int m = n - i;
      if (m == -1) stage_piece(cx, kAhead, i);
      else if (seam_unit(m)) stage_piece(cx, (m + kPf) / kChunkUnits + kAhead, i);
    }
  }
  if ((n + kPf) % kChunkUnits != 0 || n + kPf >= kUnits) return;
  seam(cx, (n + kPf) / kChunkUnits);
}

__device__ __forceinline__ i32x8 join(i32x4 lo, i32x4 hi) {
  return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
__device__ __forceinline__ bf16x8 half8(const i32x8& v, int hi) {
  return __builtin_bit_cast(bf16x8, hi ? i32x4{v[4], v[5], v[6], v[7]} : i32x4{v[0], v[1], v[2], v[3]});
}

// Unit n -> ring entry n % kRing: the unit's 4 KiB as two lane-linear 32-B A operands
// (fp8: tile o2; bf16: k-step parity s, tiles in the halves; head: k-steps 2s, 2s+1 in the
// halves) and, for a bf16 unit on an encoding, its two bf16 B fragments.
__device__ __forceinline__ void read_unit(const Ctx& cx, int n, i32x8 (&ra)[kRing][2], i32x8 (&rb)[kRing][kCols]) {
#ifdef NERF_FP8_ABLATE_NOREAD
  if (n >= kRing) return;
#endif
  const int s0 = (n / kChunkUnits) % kSlots;                   // the slot at rotation 0
  const unsigned addr = s0 < 2 ? cx.ring_lo : cx.ring_hi;
  const int off = s0 * kChunkB + (n % kChunkUnits) * kUnitB;
#pragma unroll
  for (int o2 = 0; o2 < 2; ++o2)
    ra[n % kRing][o2] = join(ds_read_b128<i32x4>(addr, off + o2 * 2048),
                             ds_read_b128<i32x4>(addr, off + o2 * 2048 + 1024));
  const UnitInfo x = kTab.u[n];
  if (x.enc != 0) {
    const int eo = (x.enc == kPos ? 0 : kDirEncOff) + x.enc_ks * 1024;
#pragma unroll
    for (int c = 0; c < kCols; ++c)
      rb[n % kRing][c] = join(ds_read_b128<i32x4>(cx.enc_addr, c * kEncWaveB + eo),
                              ds_read_b128<i32x4>(cx.enc_addr, c * kEncWaveB + eo + 1024));
  }
}

// Four e4m3 bytes from four fp32 values (RNE), low byte first.
__device__ __forceinline__ int cvt4(float a, float b, float c, float d) {
  // the low-word convert preserves the high word, which the second convert overwrites:
  // seed it with the bits of b (dying here) so the tied destination takes b's register
  // instead of a copy of a zero
  const int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, __builtin_bit_cast(int, b), false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}
// ReLU and saturation in one instruction: v_med3_f32(x, 0, 448).
__device__ __forceinline__ float relu_sat(float x) { return __builtin_amdgcn_fmed3f(x, 0.0f, kFp8Max); }
// an accumulator tile -> half of an fp8 B operand (hid_fp8_feature order)
__device__ __forceinline__ void convert_tile(const f32x16& t, i32x8& b, int off) {
#ifdef NERF_FP8_ABLATE_NOCONV
#pragma unroll
  for (int d = 0; d < 4; ++d) b[off + d] = __builtin_bit_cast(int, t[4 * d]);
  return;
#endif
#pragma unroll
  for (int d = 0; d < 4; ++d)
    b[off + d] = cvt4(relu_sat(t[4 * d]), relu_sat(t[4 * d + 1]), relu_sat(t[4 * d + 2]), relu_sat(t[4 * d + 3]));
}
// one quarter of that (dword d of the B operand half)
__device__ __forceinline__ void convert_piece(const f32x16& t, i32x8& b, int off, int d) {
#ifdef NERF_FP8_ABLATE_NOCONV
  b[off + d] = __builtin_bit_cast(int, t[4 * d]);
  return;
#endif
  b[off + d] = cvt4(relu_sat(t[4 * d]), relu_sat(t[4 * d + 1]), relu_sat(t[4 * d + 2]), relu_sat(t[4 * d + 3]));
}
// NERF_FP8_CONV (lab knob): 1 (default) spreads each conversion over the units of its quarter
// and never converts a tile in the unit right after the MFMA that finished it; 0 converts a whole
// fp8 tile per unit (units 1, 2) and starts the bf16 conversions at unit 0.
#ifndef NERF_FP8_CONV
#define NERF_FP8_CONV 1
#endif
// ReLU after rounding, on the packed bf16 words (RNE keeps sign and order): v_cvt_pk_bf16_f32,
// then v_pk_max_i16 with 0.
__device__ __forceinline__ unsigned cvt_relu_pair(float lo, float hi) {
  const bf16x2 p = __builtin_convertvector(f32x2{lo, hi}, bf16x2);
  const i16x2 m = __builtin_elementwise_max(__builtin_bit_cast(i16x2, p), i16x2(0));
  return __builtin_bit_cast(unsigned, m);
}
// dword m (0..15) of the tile pair (t, t+1) -> bf16 B fragments (hid_bf16_feature order:
// k-step 2 tile + s takes registers 8s..8s+7 of the tile)
template <int N>
__device__ __forceinline__ void bf16_dword(const f32x16 (&acc)[8], int t, int m, u32x4 (&f)[N]) {
  const int tile = t + (m >> 3), pr = m & 7;
#ifdef NERF_FP8_ABLATE_NOCONV
  f[2 * tile + (pr >> 2)][pr & 3] = __builtin_bit_cast(unsigned, acc[tile][2 * pr]);
  return;
#endif
  f[2 * tile + (pr >> 2)][pr & 3] = cvt_relu_pair(acc[tile][2 * pr], acc[tile][2 * pr + 1]);
}

// NERF_FP8_SCHED (lab knob): an explicit issue pattern for a unit body's scheduling region
// (sched_group_barrier), per MFMA: 1: 1 MFMA, 2 VALU, 1 DS read; 2: 1 MFMA, 1 DS read, 3 VALU;
// 3: 1 MFMA, 1 DS read, 6 VALU; 4: 1 MFMA, 3 VALU, 1 DS read, 3 VALU.
#ifndef NERF_FP8_SCHED
#define NERF_FP8_SCHED 0
#endif
__device__ __forceinline__ void sched_unit_pattern(int n_mfma) {
#pragma unroll
  for (int i = 0; i < n_mfma; ++i) {
    if (NERF_FP8_SCHED == 1) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    } else if (NERF_FP8_SCHED == 2) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
    } else if (NERF_FP8_SCHED == 3) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
    } else if (NERF_FP8_SCHED == 4) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
    }
  }
}

// Output conversion of a layer: into the fp8 set, the bf16 set, or C0's colour set.
enum OutKind { kOutF8 = 0, kOutB16 = 1, kOutColour = 2 };
NL_HD int out_kind(int l) { return l == C0 ? kOutColour : (l == L0 || l == L7) ? kOutB16 : kOutF8; }
NL_HD bool in_b16(int l) { return l == L1 || l == C0; }     // hidden input from the bf16 set
NL_HD bool in_f8(int l) { return !mix_bf16_layer(l); }      // hidden input from an fp8 set

template <int L>
__device__ __forceinline__ void layer_mix(f32x16 (&acc)[kCols][8], i32x8 (&b8in)[kCols][4], i32x8 (&b8out)[kCols][4],
                                          u32x4 (&b16)[kCols][16], u32x4 (&hb)[kCols][8], i32x8 (&ra)[kRing][2],
                                          i32x8 (&rb)[kRing][kCols], const Ctx& cx) {
  constexpr int UPQ = mix_units_per_quarter(L);
  constexpr int NF = mix_f8_units(L);
  constexpr int NQ = out_tiles(L) / 2;
  constexpr int N0 = mix_unit_base(L);
  constexpr int OUT = out_kind(L);
  static_assert(OUT != kOutF8 || UPQ >= 3, "tiles of an fp8 output are converted at units 1 and 2");
  static_assert(!in_f8(L) || NF == 4, "the previous layer's tiles 6, 7 are converted before k-step 3 reads them");
  int sa0 = 127, sa1 = 127;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
#pragma unroll
    for (int u = 0; u < UPQ; ++u) {
      const int n = N0 + q * UPQ + u;
      seam_before(cx, n);
      if (u == 0) {
#pragma unroll
        for (int o2 = 0; o2 < 2; ++o2) {
          const int off = 4 * (kBiasOff + 256 * L + (2 * q + o2) * 32);
          const f32x4 b0 = ds_read_b128<f32x4>(cx.bias_addr, off), b1 = ds_read_b128<f32x4>(cx.bias_addr, off + 16);
          const f32x4 b2 = ds_read_b128<f32x4>(cx.bias_addr, off + 32), b3 = ds_read_b128<f32x4>(cx.bias_addr, off + 48);
          const f32x16 bias = f32x16{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3],
                                     b2[0], b2[1], b2[2], b2[3], b3[0], b3[1], b3[2], b3[3]};
#pragma unroll
          for (int c = 0; c < kCols; ++c) acc[c][2 * q + o2] = bias;
        }
        if (NF > 0) {
          const u32x2 sc = ds_read_b64(cx.scale_addr, (L * 4 + q) * 512);
          sa0 = int(sc[0]);
          sa1 = int(sc[1]);
        }
      }
      if (n + kPf < kUnits) read_unit(cx, n + kPf, ra, rb);
      wait_lgkm(0);
      if (u < NF) {                                   // fp8 k-step u over the fp8 set
#pragma unroll
        for (int c = 0; c < kCols; ++c)
          acc[c][2 * q] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ra[n % kRing][0], b8in[c][u < NF ? u : 0],
                                                                       acc[c][2 * q], 0, 0, 0, sa0, 0, 127);
#pragma unroll
        for (int c = 0; c < kCols; ++c)
          acc[c][2 * q + 1] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ra[n % kRing][1], b8in[c][u < NF ? u : 0],
                                                                           acc[c][2 * q + 1], 0, 0, 0, sa1, 0, 127);
      } else {                                        // two bf16 k-steps
        const int b = u - NF;
        const bool enc = kTab.u[n].enc != 0;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int ks = 2 * b + s;                   // hidden k-step (bf16 layers' hidden units)
#pragma unroll
          for (int o2 = 0; o2 < 2; ++o2)
#pragma unroll
            for (int c = 0; c < kCols; ++c) {
              const bf16x8 bf = enc ? half8(rb[n % kRing][c], s) : __builtin_bit_cast(bf16x8, b16[c][ks < 16 ? ks : 0]);
              acc[c][2 * q + o2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(half8(ra[n % kRing][s], o2), bf,
                                                                          acc[c][2 * q + o2], 0, 0, 0);
            }
        }
      }
      // the previous layer's tiles 6, 7 -> this layer's input, before its unit reads them
      if (q == 0 && in_f8(L)) {
        if (NERF_FP8_CONV) {   // 8 pieces over units 1, 2 (unit 3 reads them)
#pragma unroll
          for (int pc = 0; pc < 8; ++pc)
            if (1 + pc / 4 == u)
#pragma unroll
              for (int c = 0; c < kCols; ++c) convert_piece(acc[c][6 + (pc >> 2)], b8in[c][3], 4 * (pc >> 2), pc & 3);
        } else {
#pragma unroll
          for (int c = 0; c < kCols; ++c) {
            if (u == 1) convert_tile(acc[c][6], b8in[c][3], 0);
            if (u == 2) convert_tile(acc[c][7], b8in[c][3], 4);
          }
        }
      }
      if (q == 0 && in_b16(L)) {
#pragma unroll
        for (int m = 0; m < 16; ++m)   // k-steps 12..15 are read by unit 6
          if ((NERF_FP8_CONV ? 1 + (m * 5) / 16 : (m * 6) / 16) == u)
#pragma unroll
            for (int c = 0; c < kCols; ++c) bf16_dword(acc[c], 6, m, b16[c]);
      }
      // this layer's final tiles 2q-2, 2q-1 -> the next layer's operand type
      if (q >= 1) {
        if (OUT == kOutF8) {
          if (NERF_FP8_CONV) {   // 8 pieces over units 1 .. UPQ-1
#pragma unroll
            for (int pc = 0; pc < 8; ++pc)
              if (1 + (pc * (UPQ - 1)) / 8 == u)
#pragma unroll
                for (int c = 0; c < kCols; ++c)
                  convert_piece(acc[c][2 * q - 2 + (pc >> 2)], b8out[c][q >= 1 ? q - 1 : 0], 4 * (pc >> 2), pc & 3);
          } else {
#pragma unroll
            for (int c = 0; c < kCols; ++c) {
              if (u == 1) convert_tile(acc[c][2 * q - 2], b8out[c][q >= 1 ? q - 1 : 0], 0);
              if (u == 2) convert_tile(acc[c][2 * q - 1], b8out[c][q >= 1 ? q - 1 : 0], 4);
            }
          }
        } else if (OUT == kOutB16) {
#pragma unroll
          for (int m = 0; m < 16; ++m)
            if ((NERF_FP8_CONV ? (UPQ - 1) - ((15 - m) * (UPQ - 1)) / 16 : (m * UPQ) / 16) == u)
#pragma unroll
              for (int c = 0; c < kCols; ++c) bf16_dword(acc[c], 2 * q - 2, m, b16[c]);
        } else {   // C0's tiles 0, 1 -> colour k-steps 16..19 (its tiles 2, 3 in the head units)
#pragma unroll
          for (int m = 0; m < 16; ++m)
            if ((NERF_FP8_CONV ? 1 + (m * (UPQ - 1)) / 16 : (m * UPQ) / 16) == u)
#pragma unroll
              for (int c = 0; c < kCols; ++c) bf16_dword(acc[c], 0, m, hb[c]);
        }
      }
      if (NERF_FP8_SCHED) sched_unit_pattern(kCols * (u < NF ? 2 : 4));
    }
  }
}

// A sample's network inputs, and for fused compositing the integral's network-independent ones.
struct SampleIn {
  float x[3], d[3], dist, zz;
};
template <bool kExplicit>
__device__ __forceinline__ void fetch_in(const SampleSrc& src, long p, long n_points, bool fused, SampleIn& si) {
  si.dist = 0.0f;
  si.zz = 0.0f;
  if (kExplicit) fetch_sample<true>(src, p < n_points ? p : n_points - 1, si.x, si.d);
  else fetch_render_sample(src, p < n_points ? p : n_points - 1, n_points <= 0xFFFFFFFFL, fused, si.x, si.d, si.dist, si.zz);
}
// -> the encodings in the wave's own LDS slots of column col (bf16), (dist, z) into seg buffer sb
template <bool kExplicit>
__device__ __forceinline__ void encode_write(const Ctx& cx, const SampleIn& si, bool fused, int col, int sb) {
  float pef[32], def[16];
  pos_encode<true>(si.x[0], si.x[1], si.x[2], cx.h, pef);
  dir_encode<true>(si.d[0], si.d[1], si.d[2], cx.h, def);
  const int slot = cx.wave_u * kCols + col;                 // the column's encoding and segment slots
  char* dst = cx.lds + kLdsEncOff + slot * kEncWaveB + cx.lane * 16;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)pef[8 * u + j];
    *(bf16x8*)(dst + u * 1024) = v;
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)def[8 * u + j];
    *(bf16x8*)(dst + kDirEncOff + u * 1024) = v;
  }
  if (!kExplicit && fused && cx.h == 0)
    *(f32x2_t*)(cx.lds + kLdsSegOff + sb * kSegBufB + (slot * kSamplesPerWave + (cx.lane & 31)) * 8) =
        f32x2_t{si.dist, si.zz};
}
// This tile's sample inputs -> its encodings (and (dist, z)), at the tile top.
template <bool kExplicit>
__device__ __forceinline__ void encode_tile(const Ctx& cx, const SampleSrc& src, long p, long n_points, bool fused,
                                            int col, int sb) {
  SampleIn si;
  fetch_in<kExplicit>(src, p, n_points, fused, si);
  encode_write<kExplicit>(cx, si, fused, col, sb);
}

// A tile's outputs, stored after the next tile's first seam: vmcnt counts stores together
// with the LDS-DMA in issue order, so a store issued at the tile's end would make that
// seam's vmcnt(0) wait for it as well.
struct Pending {
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};   // (sigma, r, g, b) or half of a segment record
  long idx = -1;                          // into out, or into seg (as f32x4); -1: none
  float wl = 0.f;
  long widx = -1;                         // into wloc; -1: none
};
__device__ __forceinline__ void store_pending(const Pending& pd, f32x4* out, float* wloc) {
  if (pd.idx >= 0) out[pd.idx] = pd.v;
  if (pd.widx >= 0) wloc[pd.widx] = pd.wl;
}

template <bool kExplicit>
__global__ __launch_bounds__(kThreads, 1) void mlp_fp8_kernel(const char* __restrict__ blob,
                                                              const float* __restrict__ prm_g, SampleSrc src,
                                                              long n_points, f32x4* __restrict__ out,
                                                              f32x4* __restrict__ seg, float* __restrict__ wloc) {
  __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
  const int lane = threadIdx.x & 63;
  const int wave_u = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5;
  const unsigned base = lds_addr(lds);
  const long n_tiles = (n_points + kSamplesPerBlock - 1) / kSamplesPerBlock;
  const bool fused = !kExplicit && seg != nullptr;
  f32x4* const dst = fused ? seg : out;
  Ctx cx0{blob, lds, base, wave_u, lane, h,
          base + kLdsRingOff + lane * 16, base + kLdsRingOff + lane * 16,
          base + kLdsEncOff + wave_u * kCols * kEncWaveB + lane * 16,
          base + kLdsParamOff + h * 64,
          base + kLdsScaleOff + lane * 8,
          0, kLag && wave_u >= kWaves / 2 ? 1 : 0};

  // The stream's first two chunks, and the parameters and row scales, once per workgroup.
  stage_chunk(cx0, 0);
  stage_chunk(cx0, 1);
  for (int i = threadIdx.x; i < kParamFloats / 4; i += kThreads)
    ((f32x4*)(lds + kLdsParamOff))[i] = ((const f32x4*)prm_g)[i];
  for (int i = threadIdx.x; i < kFp8ScaleBytes / 16; i += kThreads)
    ((f32x4*)(lds + kLdsScaleOff))[i] = ((const f32x4*)(blob + kFp8ScaleOff))[i];
  const float* prm = (const float*)(lds + kLdsParamOff);
  Pending pd[kCols];

#pragma unroll 1
  for (long tile = blockIdx.x, it = 0; tile < n_tiles; tile += gridDim.x, ++it) {
    // an opaque per-tile copy of the stream base: otherwise the 42 chunk addresses
    // (blob + constant) are hoisted out of the tile loop and held in SGPRs
    Ctx cx = cx0;
    asm volatile("" : "+s"(cx.blob));
    cx.rot = int(it & 1) * 2;
    cx.ring_lo = cx0.ring_lo + unsigned(cx.rot * kChunkB);
    cx.ring_hi = cx0.ring_hi - unsigned(cx.rot * kChunkB);
    const long p = (tile * kWaves + wave_u) * (kCols * kSamplesPerWave) + (lane & 31);
    // this tile's encodings into the wave's own slots (its reads of the previous tile's
    // were consumed by that tile's MFMAs)
    const int sb = NERF_FP8_PIPE_ENC ? int(it & 1) : 0;   // this tile's (dist, z) buffer
#ifdef NERF_FP8_ABLATE_PE_ONCE
    if (it == 0)
#endif
    if (!NERF_FP8_PIPE_ENC || it == 0)   // (pipelined: the previous tile's head units encoded this one)
#pragma unroll 1
      for (int c = 0; c < kCols; ++c) encode_tile<kExplicit>(cx, src, p + c * kSamplesPerWave, n_points, fused, c, sb);
    if (it == 0) {
      // barrier instance 0 publishes chunk 0 (and the parameters); the lagging half then
      // takes its seam for chunk 0 (instance 1, staging chunk 2)
      wait_vmcnt(kGldsPerStage);                     // own pieces of chunk 0 (chunk 1 may be in flight)
      __syncthreads();
      if (cx.lag) seam(cx, 0);
      if (kAhead == 2 && NERF_FP8_SPREAD) stage_piece(cx, 2, 0);   // what the tile-top seam stages later
      else if (kAhead == 2) stage_chunk(cx, 2);
    } else {
      seam(cx, 0);
#pragma unroll
      for (int c = 0; c < kCols; ++c) store_pending(pd[c], dst, wloc);   // the previous tile's outputs
    }
    i32x8 ra[kRing][2], rb[kRing][kCols];
#pragma unroll
    for (int n = 0; n < kPf; ++n) read_unit(cx, n, ra, rb);

    f32x16 acc[kCols][8];
    u32x4 b16[kCols][16], hb[kCols][8];
    i32x8 bA[kCols][4], bB[kCols][4];                // the fp8 sets: a layer reads one, fills the other
    layer_mix<L0>(acc, bA, bB, b16, hb, ra, rb, cx);   // bf16: PE -> b16
    layer_mix<L1>(acc, bB, bA, b16, hb, ra, rb, cx);   // bf16: b16 -> fp8 bA
    layer_mix<L2>(acc, bA, bB, b16, hb, ra, rb, cx);
    layer_mix<L3>(acc, bB, bA, b16, hb, ra, rb, cx);
    layer_mix<L4>(acc, bA, bB, b16, hb, ra, rb, cx);   // skip: [x, pe] (nerf.py:109-110), pe on bf16
    layer_mix<L5>(acc, bB, bA, b16, hb, ra, rb, cx);
    layer_mix<L6>(acc, bA, bB, b16, hb, ra, rb, cx);
    layer_mix<L7>(acc, bB, bA, b16, hb, ra, rb, cx);   // fp8 -> b16 (C0's input, the density head's)
    layer_mix<C0>(acc, bA, bB, b16, hb, ra, rb, cx);   // bf16: [x, PE4(d)] (nerf.py:117-121) -> hb

    // Heads (nerf.py:114, 123-129) as one bf16 MFMA tile: row 3 density over L7's output
    // (b16, k-steps 0..15), rows 0-2 colour over C0's output (hb, k-steps 16..23; C0's
    // tiles 2, 3 converted during the density units).
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
    const long next_tile = tile + gridDim.x;
    const bool has_next = NERF_FP8_PIPE_ENC && next_tile < n_tiles;   // wave-uniform
    SampleIn sn[kCols];
#pragma unroll
    for (int i = 0; i < kMixHeadUnits; ++i) {
      const int n = kMixLayerUnits + i;
      seam_before(cx, n);
      if (n + kPf < kUnits) read_unit(cx, n + kPf, ra, rb);
      if (NERF_FP8_PIPE_ENC && has_next) {
        const long pn = (next_tile * kWaves + wave_u) * (kCols * kSamplesPerWave) + (lane & 31);
        if (i == NERF_FP8_PIPE_FETCH_UNIT)
#pragma unroll
          for (int c = 0; c < kCols; ++c) fetch_in<kExplicit>(src, pn + c * kSamplesPerWave, n_points, fused, sn[c]);
        if (i == 2) encode_write<kExplicit>(cx, sn[0], fused, 0, sb ^ 1);
        if (i == 4) encode_write<kExplicit>(cx, sn[1], fused, 1, sb ^ 1);
      }
      wait_lgkm(0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ks = 4 * i + k;
#pragma unroll
        for (int c = 0; c < kCols; ++c) {
          const bf16x8 bf = __builtin_bit_cast(bf16x8, ks < 16 ? b16[c][ks < 16 ? ks : 0] : hb[c][ks >= 16 ? ks - 16 : 0]);
          hacc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(half8(ra[n % kRing][k >> 1], k & 1), bf, hacc[c], 0, 0, 0);
        }
      }
#pragma unroll
      for (int m = 0; m < 16; ++m)
        if (i < 4 && m / 4 == i)
#pragma unroll
          for (int c = 0; c < kCols; ++c) bf16_dword(acc[c], 2, m, hb[c]);   // C0's tiles 2, 3 -> k-steps 20..23
      if (NERF_FP8_SCHED) sched_unit_pattern(4 * kCols);
    }
    // the sample index again, from the lane id recounted by v_mbcnt: keeping the 64-bit p
    // (or the lane id) live through the layers costs a spill, and its reload a vmcnt(0)
    // drain of the weight stream
    const int lane_o = int(__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)));
#pragma unroll
    for (int c = 0; c < kCols; ++c) {
      const long p_o = (tile * kWaves + wave_u) * (kCols * kSamplesPerWave) + c * kSamplesPerWave + (lane_o & 31);
      const f32x4 res{relu(hacc[c][3]), sigmoid_ref(hacc[c][0]), sigmoid_ref(hacc[c][1]), sigmoid_ref(hacc[c][2])};
      pd[c] = Pending{};
      if (fused) {                                       // fused compositing: one record per segment
        const f32x2_t in = *(const f32x2_t*)(lds + kLdsSegOff + sb * kSegBufB +
                                             ((wave_u * kCols + c) * kSamplesPerWave + (lane_o & 31)) * 8);
        float wl;
        pd[c].v = seg_composite(res, in[0], in[1], lane_o, wl);
        const long first = p_o - (lane_o & 31);
        if (first < n_points && lane_o < 2) pd[c].idx = (first / kSamplesPerWave) * 2 + lane_o;
        if (wloc != nullptr && p_o < n_points && h == 0) {
          pd[c].wl = wl;
          pd[c].widx = p_o;
        }
      } else if (p_o < n_points && h == 0) {
        pd[c].v = res;
        pd[c].idx = p_o;
      }
    }
  }
  // the leading half's matching barrier for the lagging half's last seam
  if (kLag && !cx0.lag) {
    compiler_fence();
    __builtin_amdgcn_s_barrier();
    compiler_fence();
  }
#pragma unroll
  for (int c = 0; c < kCols; ++c) store_pending(pd[c], dst, wloc);
  // the stream ran two chunks into a tile that does not exist: let them land before the
  // workgroup's LDS is released
  wait_vmcnt(0);
}

}  // namespace

hipError_t launch_mlp_fp8(const void* blob, const float* params, const SampleSrc& src, long n_points, float* out,
                          bool explicit_points, hipStream_t stream, float* seg, float* wloc) {
  if (n_points <= 0) return hipSuccess;
  const long tiles = (n_points + kSamplesPerBlock - 1) / kSamplesPerBlock;
  const long blocks = tiles < current_device_cus() ? tiles : current_device_cus();   // one workgroup per CU
  if (blocks > 0x7FFFFFFFL) return hipErrorInvalidValue;
  const dim3 grid{unsigned(blocks), 1, 1}, block{kThreads, 1, 1};
  if (explicit_points)
    hipLaunchKernelGGL(mlp_fp8_kernel<true>, grid, block, 0, stream, (const char*)blob, params, src, n_points,
                       (f32x4*)out, (f32x4*)seg, wloc);
  else
    hipLaunchKernelGGL(mlp_fp8_kernel<false>, grid, block, 0, stream, (const char*)blob, params, src, n_points,
                       (f32x4*)out, (f32x4*)seg, wloc);
  return hipGetLastError();
}

}  // namespace nerf
