/*
 * nerf_mi355x.h -- C ABI of the MI355X (gfx950) NeRF render path.
 *
 * One shared library, libnerf_mi355x.so, built from nerf-dbr_amd/csrc.  Plain
 * pointers and sizes only: no C++ types, no torch types, no exceptions cross
 * this boundary.  Every int-returning call returns NERF_OK (0) or a negative
 * NERF_E_* code; the message of the last failure on the calling thread is in
 * nerf_last_error().
 *
 * Device pointers are HIP device memory on the context's device; `stream` is a
 * hipStream_t (NULL = the legacy default stream).  Calls on one context are
 * serialised on the caller's stream; a render issued on a different stream than
 * the previous render waits (on the device) for that render to finish, since
 * both use the context's scratch.  The context owns its packed weights and its
 * scratch, the caller owns every input/output buffer.
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to dgsmith7/nerf-dbr).
 */
#ifndef NERF_MI355X_H
#define NERF_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NERF_ABI_VERSION 6

enum nerf_status {
  NERF_OK = 0,
  NERF_E_INVALID = -1,    /* bad argument (shape, pointer, enum)            */
  NERF_E_HIP = -2,        /* a HIP runtime call failed                      */
  NERF_E_NO_WEIGHTS = -3, /* the requested network has not been loaded      */
  NERF_E_NO_DEVICE = -4,  /* no gfx950 device at that ordinal               */
  NERF_E_RANGE = -5,      /* NERF_F16X3: an activation left fp16's range      */
};

enum nerf_precision {
  NERF_FP32 = 0, /* f32-in MFMA (v_mfma_f32_32x32x2_f32); the parity path   */
  NERF_BF16 = 1, /* bf16-in MFMA (v_mfma_f32_32x32x16_bf16), f32 accumulate */
  NERF_FP8 = 2,  /* fp8 mixed with bf16 (round 5): L2, L3, L5-L7 and L4's hidden inputs on
                    the e4m3 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4: per-row weight scales,
                    activations e4m3 at scale 1 saturated at 448), L0, L1, L4's encoding inputs,
                    C0, the heads and every encoding on the bf16 MFMA; f32 accumulate.  The
                    compressed-weights path (config 5; the reference's int8
                    CompressedNeRFRenderer, src/benchmark/compressed_renderer.py, is its error
                    bar: on the Lego checkpoint this path is the closer of the two to the fp32
                    render, in max and mean RGB, at 200x150x32 and on whole 800x600x128 frames
                    of suite view 0 and an off-axis pose) */
  NERF_BF16X3 = 3, /* split bf16 on the bf16 MFMA: W.X ~ Wh.Xh + Wh.Xl + Wl.Xh with
                      v = vh + vl, vh = bf16(v), vl = bf16(v - vh); f32 accumulate,
                      accurate encodings: a parity-grade fast path (RGB/depth
                      within the 1e-4 gate of the reference renderer) */
  NERF_F16X3 = 4,  /* the same split on the f16 MFMA (v_mfma_f32_32x32x16_f16):
                      11-bit halves, ~10x closer to fp32 than NERF_BF16X3 at the
                      same MFMA count; weights must lie in fp16's range (65504:
                      checked at load, the precision is then refused), and so must
                      every activation and encoding input (|x| < 65520): checked on the
                      device per sample, reported by nerf_ctx_range_status as
                      NERF_E_RANGE, never as an inf or NaN image */
};

enum nerf_net { NERF_NET_COARSE = 0, NERF_NET_FINE = 1 };

/* Number of parameter tensors of one NeRFModel, in state-dict order:
 * layers.0..7, density_head, color_layers.0, color_layers.1 -- (weight, bias)
 * each, weight in nn.Linear [out, in] row-major fp32 (src/models/nerf.py:72-90). */
#define NERF_N_PARAMS 22

typedef struct nerf_ctx nerf_ctx;

int nerf_abi_version(void);
const char* nerf_last_error(void);

/* Replaces: BaseUnifiedRenderer.__init__ device binding (src/benchmark/base_renderer.py:93-112). */
int nerf_ctx_create(int device, nerf_ctx** out);
void nerf_ctx_destroy(nerf_ctx* ctx);
int nerf_device_name(int device, char* buf, int buf_len);

/* Replaces: SharedNeRFModel.load_models (src/benchmark/base_renderer.py:28-78) --
 * the caller has already read the checkpoint; this packs the 22 host tensors
 * into the kernels' fragment layouts and uploads them once.  Host buffers may
 * be freed after the call returns. */
int nerf_ctx_load_weights(nerf_ctx* ctx, int net, const float* const* params, int n_params);

/* Network layouts ("optionally a second original-NeRF weight-layout loader").
 *   NERF_LAYOUT_NERFMODEL: the reference's NeRFModel (src/models/nerf.py:48-131), as above.
 *   NERF_LAYOUT_ORIGINAL_NERF: the original NeRF implementation's network, as the reference's
 *   bundled Lego weights hold it (data/lego_example_weights, args.txt: 8x256, multires 10 / 4):
 *   position encoding re-entering at layer 5 (cat([pe, h]) there), encodings sin(2^k x) without
 *   pi, view directions normalised before their encoding, a linear feature layer before the
 *   views layer.  The 22 tensors are passed in NeRFModel's order and [out, in] orientation with
 *   three changes the host makes (nerf_amd/weights.py original_nerf_tensors): layers.4 is
 *   [256, 256], layers.5 is [256, 319] with its columns re-ordered to [h, pe], and
 *   color_layers.0 is the views layer with the feature layer folded in (W_v[:, :256] W_f,
 *   bias W_v[:, :256] b_f + b_v, in float64).  Rendered on NERF_FP32 and NERF_F16X3 (the other
 *   precisions are refused for such a net). */
#define NERF_LAYOUT_NERFMODEL 0
#define NERF_LAYOUT_ORIGINAL_NERF 1
int nerf_ctx_load_weights_layout(nerf_ctx* ctx, int net, int layout, const float* const* params, int n_params);

/* Pure host helper (no device needed): packs one network into the three blobs
 * the kernels read.  Sizes in bytes via nerf_packed_sizes.  Used by the
 * loader above and by host-side layout tests. */
void nerf_packed_sizes(size_t* f32_blob, size_t* bf16_blob, size_t* param_blob);
int nerf_pack_weights(const float* const* params, int n_params, float* f32_blob, uint16_t* bf16_blob,
                      float* param_blob);
/* The f32, params and (optional, NULL to skip) NERF_F16X3 blobs of a network in either layout
 * (NERF_LAYOUT_*); NERF_E_INVALID if the f16x3 blob is asked for and a weight is outside fp16's
 * range. */
int nerf_pack_weights_layout(const float* const* params, int n_params, int layout, float* f32_blob,
                             float* param_blob, uint16_t* f16x3_blob);

/* Pure host helpers for the fp8 path: the packed mixed blob the fp8 kernel reads (the fp8
 * layers' e4m3 fragment units, the bf16 units of L0, L1, C0, L4's encoding inputs and the
 * heads, then the per-row E8M0 weight scales), and the f32 -> e4m3fn (OCP) rounding it uses
 * (round to nearest even; inputs must be within +-448). */
size_t nerf_fp8_blob_bytes(void);
int nerf_pack_weights_fp8(const float* const* params, int n_params, uint8_t* blob);
void nerf_f32_to_e4m3(const float* x, int n, uint8_t* out);

/* Pure host helper for the split-bf16 path: W_hi / W_lo fragment units the
 * NERF_BF16X3 kernel streams (nerf_layout.h kBf16x3BlobBytes). */
size_t nerf_bf16x3_blob_bytes(void);
int nerf_pack_weights_bf16x3(const float* const* params, int n_params, uint16_t* blob);
/* The NERF_F16X3 blob (nerf_bf16x3_blob_bytes() bytes, the same unit layout with fp16
 * halves: hi = f16(w), lo = f16(w - hi)); NERF_E_INVALID if a weight is outside fp16's range. */
int nerf_pack_weights_f16x3(const float* const* params, int n_params, uint16_t* blob);

/* Pure host helper: z = near*(1-t) + far*t in fp32, operation for operation
 * (src/benchmark/base_renderer.py:274-275). */
void nerf_uniform_z(const float* t_vals, int n, float near_, float far_, float* z_out);

/* Pure host helper: torch.linspace(0, 1, n) as torch's CPU kernel computes it, bit for bit
 * (the t table of src/utils/rendering.py:37 and base_renderer.py:274). */
void nerf_linspace01(int n, float* out);

/* Replaces: BaseUnifiedRenderer.generate_rays (src/benchmark/base_renderer.py:223-258)
 * for image rows [row0, row1).  c2w: 16 floats row-major [4][4] (host).  Outputs are
 * device [(row1-row0)*width][3] fp32. */
int nerf_generate_rays(nerf_ctx* ctx, const float* c2w, int width, int height, int row0, int row1,
                       float focal, float* rays_o, float* rays_d, void* stream);

/* Replaces: BaseUnifiedRenderer.sample_points_on_rays + query_nerf_networks +
 * NeRFModel.forward (base_renderer.py:165-188, 260-281; src/models/nerf.py:92-131)
 * fused: sample s of ray r sits at  o_r + d_r * z[r*z_ray_stride + s]  (z_ray_stride 0:
 * one shared [n_samples] table), is encoded, and runs through the whole MLP.
 * out: device [n_rays*n_samples][4] = (sigma, r, g, b). */
int nerf_mlp_forward(nerf_ctx* ctx, int net, int precision, const float* rays_o, const float* rays_d,
                     const float* z, int z_ray_stride, int n_rays, int n_samples, float* out,
                     void* stream);

/* Replaces: query_nerf_networks on explicit point/direction lists
 * (base_renderer.py:165-188): positions, directions device [n][3] ->
 * out device [n][4] = (sigma, r, g, b). */
int nerf_query(nerf_ctx* ctx, int net, int precision, const float* positions, const float* directions,
               int n, float* out, void* stream);

/* Replaces: PyTorchCPURenderer.execute_volume_rendering (src/benchmark/pytorch_renderers.py:105-125)
 * and VolumeRenderer.volume_render (src/utils/rendering.py:102-143).
 * sigma[(r*S+s)*sigma_stride], rgb[(r*S+s)*rgb_stride + c], z[r*z_ray_stride + s],
 * rays_d[r*3 + c].  Outputs device: rgb_out [n_rays][3], depth_out [n_rays]; acc_out
 * [n_rays] and weights_out [n_rays][S] may be NULL. */
int nerf_composite(const float* sigma, int sigma_stride, const float* rgb, int rgb_stride,
                   const float* z, int z_ray_stride, const float* rays_d, int n_rays, int n_samples,
                   float* rgb_out, float* depth_out, float* acc_out, float* weights_out, void* stream);

/* Replaces (and fixes): VolumeRenderer.importance_sample (src/utils/rendering.py:54-100),
 * which crashes at its gather (:89-90).  For each ray: pdf from weights+1e-5 (sequential
 * normaliser), cdf, inverse-cdf samples at u (u[r*u_ray_stride + k], ascending per ray),
 * then the sorted union with the coarse z.  z_fine: device [n_rays][n_coarse+n_importance]. */
int nerf_importance_sample(const float* z_coarse, int z_ray_stride, const float* weights,
                           const float* u, int u_ray_stride, int n_rays, int n_coarse,
                           int n_importance, float* z_fine, void* stream);

/* Replaces: PyTorchCPURenderer.render_image (src/benchmark/pytorch_renderers.py:127-154)
 * for rows [row0, row1) of a width x height image, the whole path in one call:
 * rays -> (coarse pass + importance samples if n_importance > 0) -> fine pass -> composite.
 * t_vals: host [n_samples] = torch.linspace(0,1,n_samples) bits (the reference's table).
 * u: host [n_importance] ascending draw shared by every ray (NULL: t-table style
 * linspace(0,1,n_importance) computed as (k/(n-1)) in fp32).  With n_importance > 0,
 * n_samples is the coarse count.  rgb_out device [(row1-row0)*width][3], depth_out
 * device [(row1-row0)*width]. */
int nerf_render(nerf_ctx* ctx, const float* c2w, int width, int height, int row0, int row1,
                float focal, float near_, float far_, const float* t_vals, int n_samples,
                int n_importance, const float* u, int precision, float* rgb_out, float* depth_out,
                void* stream);

/* nerf_render with the random draws injected per ray (the training-time sampling of
 * VolumeRenderer, src/utils/rendering.py:36-50 and :79):
 *   t_rand: device [(row1-row0)*width][n_samples] uniform draws that stratify the
 *           first-pass samples (rendering.py:42-47); NULL = the uniform table;
 *   u_rays: device [(row1-row0)*width][n_importance], ascending per ray, replaces the
 *           shared host u (rendering.py:79 draws one row per ray); NULL = as nerf_render.
 * nerf_render(...) is nerf_render_sampled(..., t_rand = NULL, u_rays = NULL, ...). */
int nerf_render_sampled(nerf_ctx* ctx, const float* c2w, int width, int height, int row0, int row1,
                        float focal, float near_, float far_, const float* t_vals, int n_samples,
                        int n_importance, const float* u, const float* t_rand, const float* u_rays,
                        int precision, float* rgb_out, float* depth_out, void* stream);

/* Replaces: PyTorchCPURenderer.render_image (src/benchmark/pytorch_renderers.py:127-154) for one
 * row band [row0, row1) of the frame, written as the packed tile the multi-GPU gather moves
 * (SURVEY §8e): rgbd_out device [(row1-row0)*width][4] = (r, g, b, depth).  Otherwise as
 * nerf_render. */
int nerf_render_band(nerf_ctx* ctx, const float* c2w, int width, int height, int row0, int row1,
                     float focal, float near_, float far_, const float* t_vals, int n_samples,
                     int n_importance, const float* u, int precision, float* rgbd_out, void* stream);

/* The fine-pass sample depths of the last hierarchical render on this context: the sorted
 * union of coarse and importance samples (the z_samples VolumeRenderer.importance_sample
 * returns, src/utils/rendering.py:54-100, merged with the coarse z), device
 * [n_rays][per_ray].  n_rays / per_ray must match that render; NERF_E_INVALID otherwise.
 * The copy is queued on `stream`. */
int nerf_ctx_last_fine_z(nerf_ctx* ctx, long n_rays, int per_ray, float* z_out, void* stream);

/* NERF_F16X3's range contract (no reference counterpart: the reference computes in fp32).
 * Synchronizes `stream`, then returns NERF_E_RANGE if any NERF_F16X3 launch on this context
 * since the last call met an activation or encoding input of magnitude >= 65520 (fp16's
 * overflow: the outputs of those launches are not valid), NERF_OK otherwise; clears the
 * flag.  The Python plugin calls it after every f16x3 render_image / query. */
int nerf_ctx_range_status(nerf_ctx* ctx, void* stream);

/* Replaces: PositionalEncoding.encode (src/models/nerf.py:31-45) for the model's two
 * encodings (n_freqs 10: positions, 4: directions): x device [n][3] -> out device
 * [n][3 + 6*n_freqs] = [x, sin(2^0 pi x), cos(2^0 pi x), sin(2^1 pi x), ...] -- the values
 * the MLP kernels of `precision` compute before rounding them to the MFMA's input type.
 * NERF_FP32 / NERF_BF16X3 / NERF_F16X3: accurate sin/cos of fl(2^k*pi)*x (sincos_acc:
 * 3-part Cody-Waite reduction by pi/2 and minimax polynomials, within 2 ulp of torch's CPU
 * sin/cos for |x| <= 1e3 and 3 ulp at 4e3 (the reduction's second step rounds at the reduced
 * argument's ulp), 76 % bit-exact; precondition |x| < 8192, so that the quotient of
 * fl(2^9*pi*x) by pi/2 is an fp32 integer); NERF_BF16 / NERF_FP8: one reduced sin/cos per
 * coordinate and lane half, then
 * angle doubling (nerf_device.h). */
int nerf_positional_encoding(int precision, const float* x, long n, int n_freqs, float* out, void* stream);

/* Replaces: BaseUnifiedRenderer.sample_points_on_rays (src/benchmark/base_renderer.py:260-281)
 * and, with t_rand, VolumeRenderer.sample_points_on_rays(perturb=True)
 * (src/utils/rendering.py:17-52) with torch.rand_like injected.  t_vals: host [n_samples]
 * linspace table; t_rand: device [n_rays][n_samples] or NULL.  Outputs device: z_out
 * [n_rays][n_samples]; points_out [n_rays][n_samples][3] = o + d*z (may be NULL, and then
 * rays_o / rays_d may be NULL too). */
int nerf_sample_points(nerf_ctx* ctx, const float* rays_o, const float* rays_d, int n_rays,
                       const float* t_vals, int n_samples, float near_, float far_,
                       const float* t_rand, float* z_out, float* points_out, void* stream);

/* Per-stage device time of the last nerf_render on this context, from HIP events
 * recorded on the caller's stream when profiling is on.  Stages:
 * 0 rays, 1 coarse MLP, 2 importance, 3 fine MLP, 4 composite. */
#define NERF_N_STAGES 5
int nerf_ctx_set_profiling(nerf_ctx* ctx, int enable);
int nerf_ctx_stage_ms(nerf_ctx* ctx, float* ms_out /* [NERF_N_STAGES] */);
/* The same for each of the last n renders (n <= 64, oldest first), so that a run of
 * back-to-back renders can be timed per stage without a host synchronisation per frame. */
int nerf_ctx_stage_ms_history(nerf_ctx* ctx, int n, float* ms_out /* [n][NERF_N_STAGES] */);

/* Context options (no reference counterpart: implementation switches of this library).
 *   NERF_OPT_FUSED_COMPOSITE, a bit mask (default 3): in nerf_render / nerf_render_sampled,
 *   bf16 and fp8 passes whose per-ray sample count is a multiple of 32 composite inside the
 *   MLP kernel (per-32-sample partial integrals, chained per ray; the same sums as
 *   execute_volume_rendering, src/benchmark/pytorch_renderers.py:105-125, regrouped).
 *   Bit 1: the rendered pass (uniform, or the hierarchical fine pass); bit 2: the
 *   hierarchical coarse pass, whose weights then come from the MLP epilogue. 0 writes
 *   (sigma, rgb) per sample and runs the sequential composite kernel for both. */
#define NERF_OPT_FUSED_COMPOSITE 1
/*   NERF_OPT_COARSE_PRECISION (default -1: the render's own precision): the precision of the
 *   hierarchical coarse pass (rendering.py:54-100's first network evaluation) when it should
 *   differ from the fine pass's, e.g. NERF_FP32 under an NERF_F16X3 render.  The importance
 *   sampler turns last-bit differences of the coarse weights into moved fine samples at a few
 *   hundred rays per 800x600 frame, so the coarse pass's accumulation sets how close a
 *   hierarchical render is to the float64 result of the same chain. */
#define NERF_OPT_COARSE_PRECISION 2
int nerf_ctx_set_option(nerf_ctx* ctx, int option, int value);

/* ---------------------------------------------------------------------------------------
 * Training: NeRFTrainer's step on the device, fp32 throughout
 * (f32-in MFMA GEMMs, exact fp32 fma chains).  A trainer owns both networks' fp32
 * parameters, their gradients, Adam's moment estimates and the lr schedule.
 * ------------------------------------------------------------------------------------- */

/* NeRFTrainer's configuration (src/training/trainer.py:25-81; main.py:25-61 defaults). */
typedef struct nerf_train_config {
  double lr;           /* optim.Adam lr (trainer.py:57)                                  */
  double beta1, beta2; /* Adam betas (torch defaults 0.9, 0.999)                          */
  double eps;          /* Adam eps (torch default 1e-8)                                   */
  double weight_decay; /* Adam L2 weight decay added to the gradient (trainer.py:58)      */
  double lr_gamma;     /* ExponentialLR gamma = lr_decay ** (1 / decay_steps) (:62-64)    */
  double grad_clip;    /* clip_grad_norm_ max_norm over both nets; <= 0: no clipping (:128-133) */
  int n_coarse;        /* stratified coarse samples per ray (:66, rendering.py:17-52)      */
  int n_fine;          /* uniform fine samples per ray (:67, trainer.py:307-309)          */
  float near_, far_;   /* scene bounds (:70-71)                                           */
} nerf_train_config;

typedef struct nerf_trainer nerf_trainer;

/* Replaces: NeRFTrainer.__init__ (trainer.py:25-81) with the state dicts loaded: coarse and
 * fine are the 22 host tensors of each NeRFModel in state-dict order (NERF_N_PARAMS). */
int nerf_trainer_create(int device, const nerf_train_config* cfg, const float* const* coarse,
                        const float* const* fine, int n_params, nerf_trainer** out);
void nerf_trainer_destroy(nerf_trainer* tr);

/* Replaces: NeRFTrainer.train_step (trainer.py:83-138) -- _get_rays (:271-292), the ray
 * selection (:106-114), _render_rays (:294-316: coarse samples stratified by
 * VolumeRenderer.sample_points_on_rays(perturb=True), rendering.py:17-52; fine samples uniform),
 * _query_network + volume_render (:318-351, rendering.py:102-143), the two MSE losses,
 * backward, clip_grad_norm_, Adam and ExponentialLR (:121-136).  The step's draws are inputs:
 *   image   device [height][width][3] target colours;
 *   c2w     host 16 floats row-major [4][4]; focal as the dataset's (loader.py:36);
 *   select  device int32 [n_rays] = torch.randperm(height*width)[:n_rays] (trainer.py:111);
 *   t_rand  device [n_rays][n_coarse] = the coarse pass's torch.rand_like (rendering.py:47).
 * loss_out (device [3], may be NULL): loss, coarse MSE, fine MSE.  flags: NERF_TRAIN_NO_UPDATE
 * stops after backward (gradients unclipped, no optimizer or schedule step).  Work is queued on
 * `stream`; a call on another stream than the trainer's previous call waits for that call's
 * work (the trainer's workspace and state are shared by all its calls). */
#define NERF_TRAIN_NO_UPDATE 1
int nerf_train_step(nerf_trainer* tr, const float* image, int height, int width, float focal,
                    const float* c2w, const int32_t* select, int n_rays, const float* t_rand, int flags,
                    float* loss_out, void* stream);

/* Data-parallel training (one process per GPU): the gradients of this rank's share
 * of a step's rays (select / t_rand rows of the share), with the MSE normalised by the whole
 * step's ray count (the mean over n_rays_total x 3, trainer.py:117-119), so that the sum over
 * ranks -- one all-reduce of the gradient store -- is the full step's gradient.  No update:
 * every rank then runs nerf_trainer_update on the reduced gradients and the replicas stay
 * identical.  loss_out (device [3], may be NULL): this share's part of each mean. */
int nerf_train_backward(nerf_trainer* tr, const float* image, int height, int width, float focal,
                        const float* c2w, const int32_t* select, int n_rays, int n_rays_total,
                        const float* t_rand, float* loss_out, void* stream);
/* Floats per net in the flat gradient / parameter order (state-dict order, 530,052). */
#define NERF_TRAIN_NET_FLOATS 530052
/* Makes a caller-owned device buffer of 2 * NERF_TRAIN_NET_FLOATS floats (coarse, then fine; each
 * net's 22 tensors in state-dict order, row-major) the trainer's gradient store -- e.g. a tensor
 * that torch.distributed all-reduces between nerf_train_backward and nerf_trainer_update.  The
 * current gradients are copied in; NULL returns to the trainer's own store. */
int nerf_trainer_set_grad_buffer(nerf_trainer* tr, float* grads_dev);

/* Reads one net's state into 22 host buffers (state-dict order and shapes; synchronous):
 * what = NERF_TR_PARAMS, NERF_TR_GRADS (the last step's gradients, clipped when that step
 * updated), NERF_TR_EXP_AVG or NERF_TR_EXP_AVG_SQ (Adam's moment estimates). */
enum nerf_train_state { NERF_TR_PARAMS = 0, NERF_TR_GRADS = 1, NERF_TR_EXP_AVG = 2, NERF_TR_EXP_AVG_SQ = 3 };
int nerf_trainer_read(nerf_trainer* tr, int what, int net, float* const* host_out, int n_params);
/* Overwrites one net's gradients (22 host tensors), e.g. to check clip + Adam on given grads. */
int nerf_trainer_write_grads(nerf_trainer* tr, int net, const float* const* grads, int n_params);
/* Resuming a run (NeRFTrainer.load_checkpoint, trainer.py:388-399): overwrite one net's state
 * (what as for nerf_trainer_read; NERF_TR_PARAMS also rewrites the kernels' operand copies)
 * from host tensors in state-dict order, and set Adam's step count and the current learning
 * rate (optimizer.state[p]['step'], param_groups[0]['lr']; ExponentialLR's last_epoch = steps). */
int nerf_trainer_write(nerf_trainer* tr, int what, int net, const float* const* host_in, int n_params);
int nerf_trainer_set_schedule(nerf_trainer* tr, long steps, double lr);
/* The forward's arithmetic (the reference trains in fp32; no reference counterpart):
 * NERF_FP32 (default) the f32 MFMA, gradients at the fp32 ReLU-flip floor of the reference's;
 * NERF_BF16X3 the split-bf16 MFMA for the forward (mlp_bf16x3.hip's kernel with the rows and
 * ReLU bits the backward reads) and, since round 4, the backward-data chain
 * (train_bwd_x3.hip), gradients as close to the float64 step's as the reference's own fp32
 * step (more ReLU flips against the fp32 reference, so further from it: DESIGN.md section
 * 10).  The weight gradients are split-bf16 in both. */
int nerf_trainer_set_precision(nerf_trainer* tr, int precision);
/* Clip + Adam + schedule on the gradients as they stand (the update half of train_step). */
int nerf_trainer_update(nerf_trainer* tr, void* stream);
/* The learning rate the next update uses (optimizer.param_groups[0]['lr']) and the steps taken. */
double nerf_trainer_lr(const nerf_trainer* tr);
long nerf_trainer_steps(const nerf_trainer* tr);

/* Per-stage device time of the last train_step (HIP events on the step's stream, profiling on):
 * 0 rays + sampling + encoding, 1 forward GEMMs (f32 MFMA), 2 colour head + volume render
 * fwd/bwd, 3 backward-data GEMMs (f32 MFMA) + the skinny head weight gradients, 4 weight-gradient
 * GEMMs (split-bf16 MFMA, HBM-bound), 5 gradient reduction + clip + Adam + weight relayout. */
#define NERF_TRAIN_N_STAGES 6
int nerf_trainer_set_profiling(nerf_trainer* tr, int enable);
int nerf_trainer_stage_ms(nerf_trainer* tr, float* ms_out /* [NERF_TRAIN_N_STAGES] */);
/* Algorithmic fp32 FLOP of the last step's GEMMs (forward, backward-data, backward-weight,
 * unpadded shapes), for roofline reporting. */
double nerf_trainer_gemm_flops(const nerf_trainer* tr);

#ifdef __cplusplus
}
#endif
#endif /* NERF_MI355X_H */
