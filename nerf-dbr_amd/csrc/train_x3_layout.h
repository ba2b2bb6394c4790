// Layout of the split-bf16 weight stream of the training backward-data chain
// (train_bwd_x3.hip), shared by its packer (train.hip, pack_bwd_x3_kernel).
//
// The chain dZ_{l-1} = (W_l^T dZ_l) * bit(H_{l-1}) runs as "backward layers" b: b = 0 is
// the colour-0 layer's data gradient into H_7 (k = its 128 output rows; the density row's
// rank-1 term is added on the VALU), b = 1..7 are trunk layers 7..1 (k = their 256 output
// rows).  Every backward layer has 256 outputs (the forward layer's hidden inputs) in 8
// tiles of 32, issued as 4 quarters of 2 tiles, k-step by k-step (16 k each) -- the
// forward split kernels' schedule (mlp_x3.h).  One unit = one (b, quarter q, k-step u):
//   [hi: tile-in-quarter o2 (2)][lane 64][8 bf16]  then  [lo: the same], 4 KiB,
// A[row = 32 (2q + o2) + lane % 32][k = 8 (lane / 32) + j] = W_l[hid_bf16_feature(u, lane / 32,
// j)][row]: the k order the previous backward layer's accumulators give as B fragments.
// Units are streamed in order in 16 KiB chunks of 4; the colour-0 layer's 8 k-steps make
// the stream 480 units = 120 chunks, a multiple of the 4-slot ring the kernel runs by
// default (NERF_BWD_X3_SLOTS; 3 slots also divide it), so that the stream runs on across
// tiles with chunk g always in slot g % slots.
#pragma once
#include "nerf_layout.h"

namespace nerf {

constexpr int kBwdX3Layers = 8;
NL_HD int bwd_x3_ksteps(int b) { return b == 0 ? 8 : 16; }
NL_HD int bwd_x3_unit_base(int b) {
  int n = 0;
  for (int i = 0; i < b; ++i) n += 4 * bwd_x3_ksteps(i);
  return n;
}
constexpr int kBwdX3Units = bwd_x3_unit_base(kBwdX3Layers);        // 480
constexpr int kBwdX3UnitBytes = 4096;
constexpr int kBwdX3ChunkUnits = 4;
constexpr long kBwdX3BlobBytes = long(kBwdX3Units) * kBwdX3UnitBytes;   // 1.97 MB per net
static_assert(kBwdX3Units % (3 * kBwdX3ChunkUnits) == 0 && kBwdX3Units % (4 * kBwdX3ChunkUnits) == 0,
              "whole chunks, a multiple of either ring size (3 or 4 slots)");
// the forward trunk layer whose weights backward layer b >= 1 transposes
NL_HD int bwd_x3_trunk_layer(int b) { return 8 - b; }

}  // namespace nerf
