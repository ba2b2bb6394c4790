// Shared host/device description of the NeRF MLP as the gfx950 kernels see it.
//
// The network is the reference NeRFModel (src/models/nerf.py:48-131).  Kernels
// compute every Linear in the transposed orientation
//     H^T[out_feature, sample] = W[out, k] . X^T[k, sample]
// with 32x32 MFMA tiles: output features on the accumulator's ROW axis, samples
// on its COLUMN (lane) axis.  The accumulator of layer l is then already the
// B operand of layer l+1 (the contraction runs over its row index), so
// activations never leave registers; only the weights (the A operand) stream
// through LDS / L2.  The price is a fixed permutation of each layer's input
// (k) order, which is absorbed into the host-side weight packing below.
//
// Accumulator map of v_mfma_f32_32x32x{16_bf16,2_f32} (same on gfx950):
//     lane l, register r  ->  row (r&3) + 8*(r>>2) + 4*(l>>5),  column l&31.
#pragma once

#ifdef __HIPCC__
#define NL_HD __host__ __device__ constexpr
#else
#define NL_HD constexpr
#endif

namespace nerf {

constexpr int kHidden = 256;
constexpr int kPosL = 10, kDirL = 4;
constexpr int kPosDim = 3 + 6 * kPosL;   // 63
constexpr int kDirDim = 3 + 6 * kDirL;   // 27
constexpr int kColorHidden = 128;
constexpr int kSamplesPerWave = 32;      // one 32-column MFMA tile per wave

// Per-sample positional-encoding slots.  The two lane halves of a column share
// one sample; half h computes 32 of the 64 (63 + 1 pad) position features and
// 16 of the 32 (27 + 5 pad) direction features.  The split is chosen so that
// every half evaluates whole sin/cos pairs: half 0 owns frequencies 0-4 plus
// x0,x1; half 1 owns frequencies 5-9 plus x2.  Returned index is the feature's
// position in the reference's encoding ([x, sin f0, cos f0, sin f1, ...],
// nerf.py:40-45), or -1 for padding.
NL_HD int pe_slot_feature(int h, int q) {   // q in [0, 32)
  if (q < 30) return 3 + 6 * (5 * h + q / 6) + (q % 6);
  if (h == 0) return q - 30;                // x0, x1
  return q == 30 ? 2 : -1;                  // x2, pad
}
NL_HD int dpe_slot_feature(int h, int q) {  // q in [0, 16)
  if (q < 12) return 3 + 6 * (2 * h + q / 6) + (q % 6);
  if (h == 0) return q < 14 ? q - 12 : -1;  // d0, d1, pad, pad
  return q == 12 ? 2 : -1;                  // d2, pad x3
}

NL_HD int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// f32 MFMA (32x32x2): k-step u feeds one value per lane half.  Hidden k-steps
// come straight from the previous accumulator: tile u>>4, register u&15.
NL_HD int hid_f32_feature(int u, int h) { return 32 * (u >> 4) + acc_row(u & 15, h); }
// bf16 MFMA (32x32x16): k-step u (16 k) takes registers 8s..8s+7 of tile u>>1,
// s = u&1, converted pairwise to bf16.  Element j of lane half h is row
// 16s + 8(j>>2) + 4h + (j&3) of that tile.
NL_HD int hid_bf16_feature(int u, int h, int j) {
  return 32 * (u >> 1) + 16 * (u & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
}

// MFMA layers (density head and the last colour layer run on the VALU).
enum LayerId { L0 = 0, L1, L2, L3, L4, L5, L6, L7, C0, kNumMfmaLayers };
enum Extra { kNone = 0, kPos = 1, kDir = 2 };

struct LayerShape {
  int out;        // output features
  int in;         // reference in_features
  int hidden;     // leading hidden inputs (0 or 256)
  int extra;      // Extra kind appended after the hidden inputs
};

// The trunk layer whose input carries the position encoding again: NeRFModel's skip feeds
// layers[4] with cat([x, pe]) (nerf.py:109-110); the original NeRF implementation's feeds its
// layer 5 with cat([pe, h]) (data/lego_example_weights, args.txt), which the
// host re-orders to [h, pe] so that one k map serves both (nerf_amd/weights.py).
constexpr int kSkipNeRFModel = L4, kSkipOriginal = L5;

NL_HD LayerShape layer_shape(int l, int skip = kSkipNeRFModel) {
  if (l == L0) return {kHidden, kPosDim, 0, kPos};
  if (l == skip) return {kHidden, kHidden + kPosDim, kHidden, kPos};
  if (l == C0) return {kColorHidden, kHidden + kDirDim, kHidden, kDir};
  return {kHidden, kHidden, kHidden, kNone};
}
NL_HD int extra_slots(int kind) { return kind == kPos ? 32 : kind == kDir ? 16 : 0; }
NL_HD int out_tiles(int l) { return layer_shape(l).out / 32; }
NL_HD int ksteps_f32(int l, int skip = kSkipNeRFModel) {
  LayerShape s = layer_shape(l, skip);
  return s.hidden / 2 + extra_slots(s.extra);
}
NL_HD int ksteps_bf16(int l, int skip = kSkipNeRFModel) {
  LayerShape s = layer_shape(l, skip);
  return s.hidden / 16 + extra_slots(s.extra) / 8;
}

// Reference column index of the weight that multiplies the value lane half h
// supplies at (k-step u, element j) -- or -1 for padding.
NL_HD int f32_k_col(int l, int u, int h, int skip = kSkipNeRFModel) {
  LayerShape s = layer_shape(l, skip);
  int nh = s.hidden / 2;
  if (u < nh) return hid_f32_feature(u, h);
  int q = u - nh;
  int f = s.extra == kPos ? pe_slot_feature(h, q) : dpe_slot_feature(h, q);
  return f < 0 ? -1 : s.hidden + f;
}
NL_HD int bf16_k_col(int l, int u, int h, int j, int skip = kSkipNeRFModel) {
  LayerShape s = layer_shape(l, skip);
  int nh = s.hidden / 16;
  if (u < nh) return hid_bf16_feature(u, h, j);
  int q = 8 * (u - nh) + j;
  int f = s.extra == kPos ? pe_slot_feature(h, q) : dpe_slot_feature(h, q);
  return f < 0 ? -1 : s.hidden + f;
}

// ---------------------------------------------------------------- packing --
// f32 A blob, per layer: [u/4][tile o][lane 64][4 floats]  (one float4 per lane
//   covers four consecutive k-steps).
// bf16 A blob: a stream of 2 KiB "units", one per (layer, quarter q, k-step u):
//   per layer [q][u][tile-in-quarter o2 (2)][lane 64][8 bf16], where quarter q
//   holds output tiles 2q and 2q+1 (4 quarters for 256-wide layers, 2 for C0).
//   Issuing a layer quarter by quarter lets the previous layer's accumulator
//   tiles 2..7 be converted while quarter 0 computes (mlp_bf16.hip).  The
//   stream is cut into 16 KiB chunks (8 units) consumed in order; the tail is
//   zero-padded to a whole chunk.
// Params blob (fp32, shared by both precisions), in floats:
//   bias[layer l][tile o][half h][16]  at  kBiasOff + 256*l (C0: 128 used)
//   density weight [h][tile t][16] at kSigW, density bias at kSigB
//   colour-1 weight [c][h][t 0..3][16] at kC1W, colour-1 bias [3] at kC1B
constexpr int kChunkBytes = 16384;
constexpr int kBiasOff = 0;
constexpr int kSigW = 256 * kNumMfmaLayers;         // 2304
constexpr int kSigB = kSigW + 256;
constexpr int kC1W = kSigB + 4;                     // 16-B aligned
constexpr int kC1B = kC1W + 3 * 128;
constexpr int kParamFloats = kC1B + 4;              // 2952

constexpr int kUnitBytes = 2048;                    // one k-step of one quarter
constexpr int kUnitsPerChunk = kChunkBytes / kUnitBytes;

NL_HD int f32_layer_floats(int l, int skip = kSkipNeRFModel) { return ksteps_f32(l, skip) * out_tiles(l) * 64; }
NL_HD int bf16_layer_units(int l, int skip = kSkipNeRFModel) { return (out_tiles(l) / 2) * ksteps_bf16(l, skip); }
NL_HD int bf16_unit_base(int l, int skip = kSkipNeRFModel) {   // first unit of layer l
  int n = 0;
  for (int i = 0; i < l; ++i) n += bf16_layer_units(i, skip);
  return n;
}
NL_HD int f32_blob_floats() {
  int n = 0;
  for (int l = 0; l < kNumMfmaLayers; ++l) n += f32_layer_floats(l);
  return n;
}
NL_HD int bf16_blob_chunks() {
  return (bf16_unit_base(kNumMfmaLayers) + kUnitsPerChunk - 1) / kUnitsPerChunk;
}
// Output heads of the bf16 path on the MFMA (one 32-row tile): rows 0-2 the
// colour-1 layer (nerf.py:123-127) over C0's 128 outputs, row 3 the density
// head (nerf.py:114) over L7's 256 outputs, other rows zero.  24 k-steps of 16:
// k-steps 0..15 density (the L7 fragments C0 also reads), 16..23 colour (C0's
// output as bf16 fragments, hid_bf16_feature order).  Streamed after C0 as 12
// units of two k-steps each: unit i = [k-step 2i][lane 64][8 bf16],
// [k-step 2i+1][lane 64][8 bf16].
constexpr int kHeadKsteps = 24;
constexpr int kHeadUnits = kHeadKsteps / 2;
constexpr int kHeadUnitBase = bf16_unit_base(kNumMfmaLayers);           // 516
NL_HD int head_k_row_col(int u, int row, int h, int j, int* spec_is_density) {
  // returns the input feature the (k-step u, row, half h, element j) weight
  // multiplies, or -1 for a zero weight; *spec_is_density selects the tensor
  if (u < 16) {
    *spec_is_density = 1;
    return row == 3 ? hid_bf16_feature(u, h, j) : -1;
  }
  *spec_is_density = 0;
  return row < 3 ? hid_bf16_feature(u - 16, h, j) : -1;
}

// Packed bf16 blob size: units rounded up to a multiple of 32 (zero padding),
// so any kernel chunk geometry of up to 32 units reads inside the buffer.
constexpr int kBf16BlobBytes = ((kHeadUnitBase + kHeadUnits + 31) / 32) * 32 * kUnitBytes;
// Split-bf16 blob (mlp_bf16x3.hip): for each bf16 unit, its W_hi = bf16(W) unit
// then its W_lo = bf16(W - W_hi) unit (4 KiB per unit, same padding).
constexpr int kBf16x3BlobBytes = 2 * kBf16BlobBytes;

// ------------------------------------------------------------------ fp8 --
// v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 A and B (OCP e4m3fn).  Lane half h
// supplies 32 bytes of a k-step of 64; byte j of A (row r) and byte j of B
// (column c) carry the same k (pinned on hardware, tools/probes).  A hidden
// k-step u takes accumulator tiles 2u and 2u+1 of the previous layer: byte j
// of lane half h is register j&15 of tile 2u + (j>>4), i.e. row
// 32(2u + (j>>4)) + acc_row(j&15, h).  An encoding k-step takes the 32 slots
// of pe_slot_feature / dpe_slot_feature (direction: slots 16..31 padding).
// Scales are E8M0 bytes: weights per output row (fixed at packing), the
// previous layer's activations per sample (computed in the kernel).
NL_HD int hid_fp8_feature(int u, int h, int j) { return 32 * (2 * u + (j >> 4)) + acc_row(j & 15, h); }
NL_HD int ksteps_fp8(int l) { LayerShape s = layer_shape(l); return s.hidden / 64 + (s.extra != kNone ? 1 : 0); }
NL_HD int fp8_k_col(int l, int u, int h, int j) {
  LayerShape s = layer_shape(l);
  int nh = s.hidden / 64;
  if (u < nh) return hid_fp8_feature(u, h, j);
  int f = s.extra == kPos ? pe_slot_feature(h, j) : (j < 16 ? dpe_slot_feature(h, j) : -1);
  return f < 0 ? -1 : s.hidden + f;
}
// ------------------------------------------------------ fp8, mixed (round 5) --
// Config 5's network as the fp8 kernel runs it since round 5: L2, L3, L5, L6, L7 and L4's
// hidden k-steps on the fp8 MFMA; L0, L1, L4's encoding k-steps, C0 and both heads on the
// bf16 MFMA (v_mfma_f32_32x32x16_bf16); every encoding bf16.  That is the cheapest set of
// bf16 layers that puts the Lego render at least as close to the reference's fp32 render as
// the reference's own int8 compressed renderer, in max and mean RGB (tools/fp8_mixed_lab.py,
// DESIGN.md section 4); the all-fp8 form of rounds 1-4 was 1.9x / 1.2x further off.
//
// The stream is 4 KiB units, 4 per 16 KiB chunk, per layer [quarter q][unit], a quarter's
// fp8 units (k-steps) first, then its bf16 units (two k-steps each), then the head units:
//   F unit (fp8 k-step u):   [tile-in-quarter o2][half p][lane 64][16 B e4m3]; byte 16p + i of
//                             lane l is the weight of row 32(2q+o2) + (l&31) at
//                             fp8_k_col(l, u, l>>5, 16p + i), scaled by the row's 2^-e;
//   B unit (bf16 k-steps 2b, 2b+1 of the layer's bf16 k-step list): [k-step parity s][o2]
//                             [lane 64][8 bf16] at bf16_k_col(l, mix_b_kstep(l, b, s), h, j);
//   H unit (head k-steps 4i..4i+3): [k 4][lane 64][8 bf16] at head_k_row_col (nerf_layout's
//                             bf16 heads: density over L7's fragments, colour over C0's).
// Each unit is 128 MFMA cycles either way (2 fp8 MFMAs of 64, or 4 bf16 MFMAs of 32).
// Then the E8M0 row scales of the fp8 layers: per layer [quarter 4][lane 64][o2 2] u32 whose
// low byte is the scale of row 32*(2q+o2) + (lane&31) (127 = 1 for the bf16 layers).
NL_HD bool mix_bf16_layer(int l) { return l == L0 || l == L1 || l == C0; }
NL_HD int mix_f8_units(int l) { return mix_bf16_layer(l) ? 0 : layer_shape(l).hidden / 64; }
NL_HD int mix_b_units(int l) {
  return mix_bf16_layer(l) ? ksteps_bf16(l) / 2 : extra_slots(layer_shape(l).extra) / 16;
}
NL_HD int mix_units_per_quarter(int l) { return mix_f8_units(l) + mix_b_units(l); }
NL_HD int mix_layer_units(int l) { return (out_tiles(l) / 2) * mix_units_per_quarter(l); }
NL_HD int mix_unit_base(int l) {
  int n = 0;
  for (int i = 0; i < l; ++i) n += mix_layer_units(i);
  return n;
}
// bf16 k-step (bf16_k_col numbering) of element s of B unit b of layer l
NL_HD int mix_b_kstep(int l, int b, int s) {
  return (mix_bf16_layer(l) ? 0 : layer_shape(l).hidden / 16) + 2 * b + s;
}
constexpr int kFp8UnitBytes = 4096;
constexpr int kMixLayerUnits = mix_unit_base(kNumMfmaLayers);                  // 162
constexpr int kMixHeadUnits = kHeadKsteps / 4;                                 // 6
constexpr int kMixUnits = kMixLayerUnits + kMixHeadUnits;                      // 168
constexpr int kFp8UnitsPadded = ((kMixUnits + 7) / 8) * 8;                     // 168
constexpr int kFp8ScaleOff = kFp8UnitsPadded * kFp8UnitBytes;                  // bytes
constexpr int kFp8ScaleBytes = (kNumMfmaLayers + 1) * 4 * 64 * 2 * 4;
constexpr int kFp8BlobBytes = kFp8ScaleOff + kFp8ScaleBytes;
constexpr float kFp8Max = 448.0f;                                              // largest finite e4m3fn

}  // namespace nerf
