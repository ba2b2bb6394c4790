// Internal declarations shared by the C ABI (capi.hip), the packer and the kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "nerf_mi355x.h"

// Record a failure for nerf_last_error() (thread-local) and return `code`.
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

namespace nerf {

struct SampleSrc;

// Element strides of a render's per-ray outputs: rgb at rgb*r (3: [R][3]; 4: the
// packed [R][4] band of nerf_render_band, depth then at offset 3), depth at depth*r.
struct OutStrides {
  int rgb = 3;
  int depth = 1;
};

// Compute units of the current device (cached per device): the grid of the
// persistent MLP kernels, one workgroup per CU.
int current_device_cus();

hipError_t launch_generate_rays(const float* c2w_rowmajor16, int width, int height, int row0, int row1,
                                float focal, float* rays_o, float* rays_d, hipStream_t stream);
// layout: 0 = NeRFModel (nerf.py), 1 = the original NeRF implementation's trunk (skip into
// layer 5, encodings without pi, normalised view directions; nerf_ctx_load_weights_layout)
hipError_t launch_mlp_f32(const float* blob, const float* params, const SampleSrc& src, long n_points,
                          float* out, bool explicit_points, hipStream_t stream, int layout = 0);
// seg (render passes with n_samples % 32 == 0 only): compositing fused into the
// epilogue, one 32-B SegRecord per 32-sample segment instead of out's (sigma, rgb);
// wloc (with seg): each sample's in-segment weight as well (hierarchical coarse pass)
hipError_t launch_mlp_bf16(const void* blob, const float* params, const SampleSrc& src, long n_points,
                           float* out, bool explicit_points, hipStream_t stream, float* seg = nullptr,
                           float* wloc = nullptr);
hipError_t launch_mlp_fp8(const void* blob, const float* params, const SampleSrc& src, long n_points,
                          float* out, bool explicit_points, hipStream_t stream, float* seg = nullptr,
                          float* wloc = nullptr);
// Split-bf16 parity-grade path (mlp_bf16x3.hip): (sigma, r, g, b) per sample.
hipError_t launch_mlp_bf16x3(const void* blob, const float* params, const SampleSrc& src, long n_points,
                             float* out, bool explicit_points, hipStream_t stream, float* seg = nullptr);
// Split-fp16 parity-grade path (the same kernel on the f16 MFMA, nerf_pack_weights_f16x3's blob).
// seg: the render pass's fused compositing (S % 32 == 0), one SegRecord per 32 samples.
// range_flag: set to 1 (device int) when a sample's activation overflowed fp16 (mlp_x3.h).
hipError_t launch_mlp_f16x3(const void* blob, const float* params, const SampleSrc& src, long n_points,
                            float* out, bool explicit_points, hipStream_t stream, float* seg = nullptr,
                            int* range_flag = nullptr, int layout = 0);
// The same kernel as the training forward (train.hip): per sample also every trunk layer's
// post-ReLU row h[l] [P][256] and ReLU bit words mb[l] [P][8], the colour-0 row and density
// hc [P][132], and (r, g, b, sigma) rgbs [P][4]; blob is the split-bf16 blob of the net's
// current weights (nerf_pack_weights_bf16x3's layout), params the params blob.
struct X3TrainOut {
  float* h[8];
  unsigned* mb[8];
  float* hc;
  float* rgbs;
};
hipError_t launch_mlp_bf16x3_train(const void* blob, const float* params, const SampleSrc& src, long n_points,
                                   const X3TrainOut& o, hipStream_t stream);
// The training backward-data chain on the split-bf16 MFMA (train_bwd_x3.hip): dZ_7 .. dZ_0
// rows from the head backward's rows, the stored ReLU bits and the packed transposed
// weights (train_x3_layout.h; packed from the flat parameters by train.hip).
struct BwdX3Io {
  const float* dhc;          // [P][132]: colour-0 pre-activation gradients (128), density (128)
  const float* wsig;         // density weights in accumulator order [h][tile 8][16] (params blob)
  const unsigned* mb[8];     // ReLU bits of H_0..H_7, [P][8]
  float* dz[8];              // out: dZ_0..dZ_7 rows [P][256]
};
hipError_t launch_train_bwd_x3(const void* blob, long n_points, const BwdX3Io& io, hipStream_t stream);
// Chains each ray's segment records into (rgb, depth) (nerf_device.h SegRecord).
hipError_t launch_composite_segments(const float* seg, int n_rays, int n_segments, float* rgb_out, float* depth_out,
                                     hipStream_t stream, OutStrides os = {});
hipError_t launch_composite(const float* sigma, int sigma_stride, const float* rgb, int rgb_stride,
                            const float* z, int z_ray_stride, const float* rays_d, int n_rays, int n_samples,
                            float* rgb_out, float* depth_out, float* acc_out, float* weights_out,
                            hipStream_t stream, OutStrides os = {});
// PositionalEncoding.encode (nerf.py:31-45) as the MLP kernels evaluate it:
// x [n][3] -> out [n][3 + 6*n_freqs] in the reference's channel order; fast =
// the bf16/fp8 kernels' reduced sin/cos with angle doubling, else accurate sincosf.
hipError_t launch_encode(const float* x, long n, int n_freqs, bool fast, float* out, hipStream_t stream);
hipError_t launch_sample(const float* z_tab, const float* t_rand, int n_rays, int n_samples, const float* rays_o,
                         const float* rays_d, float* z_out, float* points_out, hipStream_t stream);
// seg (optional): weights are in-segment weights of a fused coarse pass, scaled
// here by the product of the ray's earlier segment records' P
hipError_t launch_importance(const float* z_coarse, int z_ray_stride, const float* weights, const float* u,
                             int u_ray_stride, int n_rays, int n_coarse, int n_importance, float* z_fine,
                             hipStream_t stream, const float* seg = nullptr);

}  // namespace nerf
