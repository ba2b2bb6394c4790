// C ABI of libnerf_mi355x.so (declared in include/nerf_mi355x.h).
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

#include "nerf_device.h"
#include "nerf_internal.h"

namespace {

thread_local char g_err[512] = "";

}  // namespace

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int nerf::current_device_cus() {
  static int cache[64] = {};   // benign race: every writer stores the same value
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cache[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

#define HIP_TRY(expr)                                                                                 \
  do {                                                                                                \
    hipError_t e_ = (expr);                                                                           \
    if (e_ != hipSuccess) return set_error(NERF_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                           __FILE__, __LINE__);                                      \
  } while (0)

using namespace nerf;

struct NetDev {
  float* f32 = nullptr;
  void* bf16 = nullptr;
  void* fp8 = nullptr;      // e4m3 fragments + E8M0 row scales (nerf_layout.h)
  void* bf16x3 = nullptr;   // split-bf16 fragments: W_hi and W_lo units (nerf_layout.h)
  void* f16x3 = nullptr;    // split-fp16 fragments, the same layout
  bool f16x3_ok = false;    // the loaded weights fit fp16's range
  float* params = nullptr;
  bool loaded = false;
  int layout = NERF_LAYOUT_NERFMODEL;   // NERF_LAYOUT_ORIGINAL_NERF: f32 blob + params only
};

struct nerf_ctx {
  int device = 0;
  NetDev net[2];
  // scratch, grown on demand and reused across renders
  float* rays = nullptr;       // [2][n_rays][3] (o then d)
  size_t rays_cap = 0;         // rays
  float* mlp_out = nullptr;    // [P][4]
  size_t mlp_cap = 0;          // points
  float* zbuf = nullptr;       // coarse table [S] + per-ray fine z [R][S+N]
  size_t z_cap = 0;            // floats
  float* wbuf = nullptr;       // coarse weights [R][S] + u [N]
  size_t w_cap = 0;            // floats
  float* host_stage = nullptr; // pinned: z table + u
  // what the last upload put on the device (nerf_render skips an unchanged upload,
  // so back-to-back renders queue without a host synchronisation)
  std::vector<float> up_z, up_u;
  const float* up_zbuf = nullptr;
  const float* up_wbuf = nullptr;
  hipEvent_t stage_ev = nullptr; // recorded after the last upload from host_stage
  int* d_range = nullptr;        // device int: an NERF_F16X3 launch saw an activation outside fp16's range
  // The stream of the last render: a render on another stream first waits for the
  // previous render's end event (its uploads and its use of the shared scratch)
  hipStream_t last_stream = nullptr;
  // the fine-pass sample depths of the last hierarchical render (nerf_ctx_last_fine_z)
  const float* last_zfine = nullptr;
  long last_zfine_rays = 0;
  int last_zfine_per_ray = 0;
  bool profiling = false;
  int fused_composite = 3;     // NERF_OPT_FUSED_COMPOSITE bits: 1 render passes, 2 hierarchical coarse pass
  int coarse_precision = -1;   // NERF_OPT_COARSE_PRECISION: -1 = the render's precision
  // stage events of the last kEvFrames renders (a ring, so that per-frame stage
  // times can be read after a run of back-to-back renders without a host sync each)
  struct Frame {
    hipEvent_t ev[NERF_N_STAGES + 1] = {};
    bool ran[NERF_N_STAGES] = {};
    bool profiled = false;
  };
  static constexpr int kEvFrames = 64;
  Frame frames[kEvFrames];
  long n_frames = 0;              // renders issued on this context
};

namespace {

template <typename T>
int grow(T*& p, size_t& cap, size_t need, const char* what) {
  if (need <= cap) return NERF_OK;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  size_t n = need + need / 8;
  hipError_t e = hipMalloc((void**)&p, n * sizeof(T));
  if (e != hipSuccess) return set_error(NERF_E_HIP, "hipMalloc %s (%zu bytes): %s", what, n * sizeof(T), hipGetErrorString(e));
  cap = n;
  return NERF_OK;
}

int check_net(nerf_ctx* ctx, int net, int precision) {
  if (!ctx) return set_error(NERF_E_INVALID, "null context");
  if (net != NERF_NET_COARSE && net != NERF_NET_FINE) return set_error(NERF_E_INVALID, "bad net %d", net);
  if (precision != NERF_FP32 && precision != NERF_BF16 && precision != NERF_FP8 && precision != NERF_BF16X3 &&
      precision != NERF_F16X3)
    return set_error(NERF_E_INVALID, "bad precision %d", precision);
  if (!ctx->net[net].loaded) return set_error(NERF_E_NO_WEIGHTS, "%s network not loaded", net ? "fine" : "coarse");
  if (ctx->net[net].layout == NERF_LAYOUT_ORIGINAL_NERF && precision != NERF_FP32 && precision != NERF_F16X3)
    return set_error(NERF_E_INVALID, "%s network has the original-NeRF layout: NERF_FP32 and NERF_F16X3 only",
                     net ? "fine" : "coarse");
  if (precision == NERF_F16X3 && !ctx->net[net].f16x3_ok)
    return set_error(NERF_E_INVALID, "%s network has weights outside fp16's range: NERF_F16X3 unavailable",
                     net ? "fine" : "coarse");
  return NERF_OK;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
    else prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

hipError_t run_mlp(nerf_ctx* ctx, int net, int precision, const SampleSrc& src, long n, float* out, bool expl,
                   hipStream_t s, float* seg = nullptr, float* wloc = nullptr) {
  const NetDev& nd = ctx->net[net];
  if (precision == NERF_BF16) return launch_mlp_bf16(nd.bf16, nd.params, src, n, out, expl, s, seg, wloc);
  if (precision == NERF_FP8) return launch_mlp_fp8(nd.fp8, nd.params, src, n, out, expl, s, seg, wloc);
  if (precision == NERF_BF16X3) return launch_mlp_bf16x3(nd.bf16x3, nd.params, src, n, out, expl, s, seg);
  if (precision == NERF_F16X3)
    return launch_mlp_f16x3(nd.f16x3, nd.params, src, n, out, expl, s, seg, ctx->d_range, nd.layout);
  return launch_mlp_f32(nd.f32, nd.params, src, n, out, expl, s, nd.layout);
}

}  // namespace

extern "C" {

int nerf_abi_version(void) { return NERF_ABI_VERSION; }
const char* nerf_last_error(void) { return g_err; }

int nerf_device_name(int device, char* buf, int buf_len) {
  if (!buf || buf_len <= 0) return set_error(NERF_E_INVALID, "bad buffer");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  snprintf(buf, size_t(buf_len), "%s (%s, %d CUs)", prop.name, prop.gcnArchName, prop.multiProcessorCount);
  return NERF_OK;
}

int nerf_ctx_create(int device, nerf_ctx** out) {
  if (!out) return set_error(NERF_E_INVALID, "null out pointer");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
    return set_error(NERF_E_NO_DEVICE, "no HIP device %d (count %d)", device, n);
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return set_error(NERF_E_NO_DEVICE, "device %d is %s; this library is built for gfx950 (MI355X)", device,
                     prop.gcnArchName);
  DeviceGuard g(device);
  nerf_ctx* ctx = new nerf_ctx();
  ctx->device = device;
  for (auto& f : ctx->frames)
    for (auto& e : f.ev) HIP_TRY(hipEventCreate(&e));
  HIP_TRY(hipEventCreateWithFlags(&ctx->stage_ev, hipEventDisableTiming));
  HIP_TRY(hipHostMalloc((void**)&ctx->host_stage, sizeof(float) * 2048, hipHostMallocDefault));
  HIP_TRY(hipMalloc((void**)&ctx->d_range, sizeof(int)));
  HIP_TRY(hipMemset(ctx->d_range, 0, sizeof(int)));
  *out = ctx;
  return NERF_OK;
}

void nerf_ctx_destroy(nerf_ctx* ctx) {
  if (!ctx) return;
  DeviceGuard g(ctx->device);
  (void)hipDeviceSynchronize();
  for (auto& nd : ctx->net) {
    if (nd.f32) (void)hipFree(nd.f32);
    if (nd.bf16) (void)hipFree(nd.bf16);
    if (nd.fp8) (void)hipFree(nd.fp8);
    if (nd.bf16x3) (void)hipFree(nd.bf16x3);
    if (nd.f16x3) (void)hipFree(nd.f16x3);
    if (nd.params) (void)hipFree(nd.params);
  }
  for (float* p : {ctx->rays, ctx->mlp_out, ctx->zbuf, ctx->wbuf})
    if (p) (void)hipFree(p);
  if (ctx->host_stage) (void)hipHostFree(ctx->host_stage);
  for (auto& f : ctx->frames)
    for (auto& e : f.ev)
      if (e) (void)hipEventDestroy(e);
  if (ctx->stage_ev) (void)hipEventDestroy(ctx->stage_ev);
  if (ctx->d_range) (void)hipFree(ctx->d_range);
  delete ctx;
}

int nerf_ctx_load_weights(nerf_ctx* ctx, int net, const float* const* params, int n_params) {
  if (!ctx) return set_error(NERF_E_INVALID, "null context");
  if (net != NERF_NET_COARSE && net != NERF_NET_FINE) return set_error(NERF_E_INVALID, "bad net %d", net);
  size_t nf32, nbf16, nprm;
  nerf_packed_sizes(&nf32, &nbf16, &nprm);
  std::vector<float> f32(nf32 / 4), prm(nprm / 4);
  std::vector<uint16_t> bf(nbf16 / 2);
  int rc = nerf_pack_weights(params, n_params, f32.data(), bf.data(), prm.data());
  if (rc != NERF_OK) return rc;
  const size_t nfp8 = nerf_fp8_blob_bytes();
  std::vector<uint8_t> f8(nfp8);
  if ((rc = nerf_pack_weights_fp8(params, n_params, f8.data())) != NERF_OK) return rc;
  const size_t nx3 = nerf_bf16x3_blob_bytes();
  std::vector<uint16_t> x3(nx3 / 2);
  if ((rc = nerf_pack_weights_bf16x3(params, n_params, x3.data())) != NERF_OK) return rc;
  // fp16 halves: only when every weight fits fp16's range (else NERF_F16X3 stays unavailable,
  // and check_net says so when it is asked for); the probe's refusal is not this call's error
  std::vector<uint16_t> h3(nx3 / 2);
  char saved_err[sizeof(g_err)];
  std::memcpy(saved_err, g_err, sizeof(g_err));
  const bool have_f16x3 = nerf_pack_weights_f16x3(params, n_params, h3.data()) == NERF_OK;
  if (!have_f16x3) std::memcpy(g_err, saved_err, sizeof(g_err));
  DeviceGuard g(ctx->device);
  NetDev& nd = ctx->net[net];
  if (!nd.f32) HIP_TRY(hipMalloc((void**)&nd.f32, nf32));
  if (!nd.bf16) HIP_TRY(hipMalloc(&nd.bf16, nbf16));
  if (!nd.params) HIP_TRY(hipMalloc((void**)&nd.params, nprm));
  if (!nd.fp8) HIP_TRY(hipMalloc(&nd.fp8, nfp8));
  if (!nd.bf16x3) HIP_TRY(hipMalloc(&nd.bf16x3, nx3));
  HIP_TRY(hipMemcpy(nd.fp8, f8.data(), nfp8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(nd.bf16x3, x3.data(), nx3, hipMemcpyHostToDevice));
  if (have_f16x3) {
    if (!nd.f16x3) HIP_TRY(hipMalloc(&nd.f16x3, nx3));
    HIP_TRY(hipMemcpy(nd.f16x3, h3.data(), nx3, hipMemcpyHostToDevice));
  }
  nd.f16x3_ok = have_f16x3;
  HIP_TRY(hipMemcpy(nd.f32, f32.data(), nf32, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(nd.bf16, bf.data(), nbf16, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(nd.params, prm.data(), nprm, hipMemcpyHostToDevice));
  nd.loaded = true;
  nd.layout = NERF_LAYOUT_NERFMODEL;
  return NERF_OK;
}

int nerf_ctx_load_weights_layout(nerf_ctx* ctx, int net, int layout, const float* const* params, int n_params) {
  if (layout == NERF_LAYOUT_NERFMODEL) return nerf_ctx_load_weights(ctx, net, params, n_params);
  if (!ctx) return set_error(NERF_E_INVALID, "null context");
  if (net != NERF_NET_COARSE && net != NERF_NET_FINE) return set_error(NERF_E_INVALID, "bad net %d", net);
  if (layout != NERF_LAYOUT_ORIGINAL_NERF) return set_error(NERF_E_INVALID, "unknown layout %d", layout);
  size_t nf32, nbf16, nprm;
  nerf_packed_sizes(&nf32, &nbf16, &nprm);
  std::vector<float> f32(nf32 / 4), prm(nprm / 4);
  int rc = nerf_pack_weights_layout(params, n_params, layout, f32.data(), prm.data(), nullptr);
  if (rc != NERF_OK) return rc;
  // the split-fp16 blob when every weight fits fp16's range (else NERF_F16X3 stays unavailable)
  const size_t nx3 = nerf_bf16x3_blob_bytes();
  std::vector<uint16_t> h3(nx3 / 2);
  char saved_err[sizeof(g_err)];
  std::memcpy(saved_err, g_err, sizeof(g_err));
  const bool have_f16x3 = nerf_pack_weights_layout(params, n_params, layout, nullptr, nullptr, h3.data()) == NERF_OK;
  if (!have_f16x3) std::memcpy(g_err, saved_err, sizeof(g_err));
  DeviceGuard g(ctx->device);
  NetDev& nd = ctx->net[net];
  if (!nd.f32) HIP_TRY(hipMalloc((void**)&nd.f32, nf32));
  if (!nd.params) HIP_TRY(hipMalloc((void**)&nd.params, nprm));
  HIP_TRY(hipMemcpy(nd.f32, f32.data(), nf32, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(nd.params, prm.data(), nprm, hipMemcpyHostToDevice));
  if (have_f16x3) {
    if (!nd.f16x3) HIP_TRY(hipMalloc(&nd.f16x3, nx3));
    HIP_TRY(hipMemcpy(nd.f16x3, h3.data(), nx3, hipMemcpyHostToDevice));
  }
  nd.f16x3_ok = have_f16x3;
  nd.loaded = true;
  nd.layout = layout;
  return NERF_OK;
}

int nerf_generate_rays(nerf_ctx* ctx, const float* c2w, int width, int height, int row0, int row1, float focal,
                       float* rays_o, float* rays_d, void* stream) {
  if (!ctx || !c2w || !rays_o || !rays_d) return set_error(NERF_E_INVALID, "nerf_generate_rays: null argument");
  if (width <= 0 || height <= 0 || row0 < 0 || row1 > height || row0 > row1)
    return set_error(NERF_E_INVALID, "nerf_generate_rays: bad image/rows %dx%d [%d,%d)", width, height, row0, row1);
  DeviceGuard g(ctx->device);
  HIP_TRY(launch_generate_rays(c2w, width, height, row0, row1, focal, rays_o, rays_d, (hipStream_t)stream));
  return NERF_OK;
}

int nerf_mlp_forward(nerf_ctx* ctx, int net, int precision, const float* rays_o, const float* rays_d, const float* z,
                     int z_ray_stride, int n_rays, int n_samples, float* out, void* stream) {
  int rc = check_net(ctx, net, precision);
  if (rc != NERF_OK) return rc;
  if (n_rays < 0 || n_samples <= 0 || z_ray_stride < 0) return set_error(NERF_E_INVALID, "nerf_mlp_forward: bad sizes");
  if (n_rays == 0) return NERF_OK;
  if (!rays_o || !rays_d || !z || !out) return set_error(NERF_E_INVALID, "nerf_mlp_forward: null pointer");
  DeviceGuard g(ctx->device);
  SampleSrc src{rays_o, rays_d, z, z_ray_stride, n_samples, nullptr, nullptr};
  HIP_TRY(run_mlp(ctx, net, precision, src, long(n_rays) * n_samples, out, false, (hipStream_t)stream));
  return NERF_OK;
}

int nerf_query(nerf_ctx* ctx, int net, int precision, const float* positions, const float* directions, int n,
               float* out, void* stream) {
  int rc = check_net(ctx, net, precision);
  if (rc != NERF_OK) return rc;
  if (n < 0) return set_error(NERF_E_INVALID, "nerf_query: n < 0");
  if (n == 0) return NERF_OK;
  if (!positions || !directions || !out) return set_error(NERF_E_INVALID, "nerf_query: null pointer");
  DeviceGuard g(ctx->device);
  SampleSrc src{nullptr, nullptr, nullptr, 0, 1, positions, directions};
  HIP_TRY(run_mlp(ctx, net, precision, src, n, out, true, (hipStream_t)stream));
  return NERF_OK;
}

int nerf_composite(const float* sigma, int sigma_stride, const float* rgb, int rgb_stride, const float* z,
                   int z_ray_stride, const float* rays_d, int n_rays, int n_samples, float* rgb_out, float* depth_out,
                   float* acc_out, float* weights_out, void* stream) {
  if (n_rays < 0 || n_samples <= 0) return set_error(NERF_E_INVALID, "nerf_composite: bad sizes");
  if (n_rays == 0) return NERF_OK;
  if (!sigma || !rgb || !z || !rays_d || !rgb_out || !depth_out) return set_error(NERF_E_INVALID, "nerf_composite: null pointer");
  HIP_TRY(launch_composite(sigma, sigma_stride, rgb, rgb_stride, z, z_ray_stride, rays_d, n_rays, n_samples, rgb_out,
                           depth_out, acc_out, weights_out, (hipStream_t)stream));
  return NERF_OK;
}

int nerf_importance_sample(const float* z_coarse, int z_ray_stride, const float* weights, const float* u,
                           int u_ray_stride, int n_rays, int n_coarse, int n_importance, float* z_fine, void* stream) {
  if (n_rays < 0 || n_coarse < 2 || n_coarse > 256 || n_importance < 0)
    return set_error(NERF_E_INVALID, "nerf_importance_sample: bad sizes (n_coarse must be 2..256)");
  if (n_rays == 0) return NERF_OK;
  if (!z_coarse || !weights || !z_fine || (n_importance > 0 && !u))
    return set_error(NERF_E_INVALID, "nerf_importance_sample: null pointer");
  HIP_TRY(launch_importance(z_coarse, z_ray_stride, weights, u, u_ray_stride, n_rays, n_coarse, n_importance, z_fine,
                            (hipStream_t)stream));
  return NERF_OK;
}

int nerf_sample_points(nerf_ctx* ctx, const float* rays_o, const float* rays_d, int n_rays, const float* t_vals,
                       int n_samples, float near_, float far_, const float* t_rand, float* z_out, float* points_out,
                       void* stream) {
  if (!ctx) return set_error(NERF_E_INVALID, "null context");
  if (n_rays < 0 || n_samples <= 0 || n_samples > 1024) return set_error(NERF_E_INVALID, "nerf_sample_points: bad sizes");
  if (n_rays == 0) return NERF_OK;
  if (!t_vals || !z_out || (points_out && (!rays_o || !rays_d)))
    return set_error(NERF_E_INVALID, "nerf_sample_points: null pointer");
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  int rc = grow(ctx->zbuf, ctx->z_cap, 1024, "z");
  if (rc != NERF_OK) return rc;
  HIP_TRY(hipStreamSynchronize(s));   // host_stage may still feed a previous copy
  HIP_TRY(hipEventSynchronize(ctx->stage_ev));
  ctx->up_zbuf = nullptr;             // the table slot is overwritten below
  nerf_uniform_z(t_vals, n_samples, near_, far_, ctx->host_stage);
  HIP_TRY(hipMemcpyAsync(ctx->zbuf, ctx->host_stage, sizeof(float) * n_samples, hipMemcpyHostToDevice, s));
  HIP_TRY(launch_sample(ctx->zbuf, t_rand, n_rays, n_samples, rays_o, rays_d, z_out, points_out, s));
  return NERF_OK;
}

int nerf_ctx_set_profiling(nerf_ctx* ctx, int enable) {
  if (!ctx) return set_error(NERF_E_INVALID, "null context");
  ctx->profiling = enable != 0;
  return NERF_OK;
}

int nerf_ctx_set_option(nerf_ctx* ctx, int option, int value) {
  if (!ctx) return set_error(NERF_E_INVALID, "null context");
  if (option == NERF_OPT_FUSED_COMPOSITE) {
    if (value < 0 || value > 3) return set_error(NERF_E_INVALID, "NERF_OPT_FUSED_COMPOSITE takes 0..3, got %d", value);
    ctx->fused_composite = value;
    return NERF_OK;
  }
  if (option == NERF_OPT_COARSE_PRECISION) {
    if (value != -1 && value != NERF_FP32 && value != NERF_BF16 && value != NERF_FP8 && value != NERF_BF16X3 &&
        value != NERF_F16X3)
      return set_error(NERF_E_INVALID, "NERF_OPT_COARSE_PRECISION takes -1 or a precision, got %d", value);
    ctx->coarse_precision = value;
    return NERF_OK;
  }
  return set_error(NERF_E_INVALID, "unknown option %d", option);
}

int nerf_ctx_stage_ms_history(nerf_ctx* ctx, int n, float* ms_out) {
  if (!ctx || !ms_out) return set_error(NERF_E_INVALID, "null argument");
  if (n <= 0 || n > nerf_ctx::kEvFrames || n > ctx->n_frames)
    return set_error(NERF_E_INVALID, "stage history of %d frames: %ld rendered, ring of %d", n, ctx->n_frames,
                     nerf_ctx::kEvFrames);
  DeviceGuard g(ctx->device);
  for (int k = 0; k < n; ++k) {
    const nerf_ctx::Frame& f = ctx->frames[(ctx->n_frames - n + k) % nerf_ctx::kEvFrames];
    HIP_TRY(hipEventSynchronize(f.ev[NERF_N_STAGES]));
    for (int i = 0; i < NERF_N_STAGES; ++i) {
      float* o = ms_out + k * NERF_N_STAGES + i;
      *o = 0.0f;
      if (f.profiled && f.ran[i]) HIP_TRY(hipEventElapsedTime(o, f.ev[i], f.ev[i + 1]));
    }
  }
  return NERF_OK;
}

int nerf_ctx_stage_ms(nerf_ctx* ctx, float* ms_out) {
  if (!ctx || !ms_out) return set_error(NERF_E_INVALID, "null argument");
  if (ctx->n_frames == 0) {
    for (int i = 0; i < NERF_N_STAGES; ++i) ms_out[i] = 0.0f;
    return NERF_OK;
  }
  return nerf_ctx_stage_ms_history(ctx, 1, ms_out);
}

int nerf_render(nerf_ctx* ctx, const float* c2w, int width, int height, int row0, int row1, float focal, float near_,
                float far_, const float* t_vals, int n_samples, int n_importance, const float* u, int precision,
                float* rgb_out, float* depth_out, void* stream) {
  return nerf_render_sampled(ctx, c2w, width, height, row0, row1, focal, near_, far_, t_vals, n_samples, n_importance,
                             u, nullptr, nullptr, precision, rgb_out, depth_out, stream);
}

}  // extern "C"

namespace {

// The whole render path (nerf_render, nerf_render_sampled, nerf_render_band):
// outputs at rgb_out + os.rgb * ray and depth_out + os.depth * ray.
int render_impl(nerf_ctx* ctx, const float* c2w, int width, int height, int row0, int row1, float focal,
                float near_, float far_, const float* t_vals, int n_samples, int n_importance, const float* u,
                const float* t_rand, const float* u_rays, int precision, float* rgb_out, float* depth_out,
                OutStrides os, void* stream) {
  const int net_main = NERF_NET_FINE;
  const int coarse_prec = ctx->coarse_precision >= 0 ? ctx->coarse_precision : precision;
  int rc = check_net(ctx, net_main, precision);
  if (rc != NERF_OK) return rc;
  if (n_importance > 0 && (rc = check_net(ctx, NERF_NET_COARSE, coarse_prec)) != NERF_OK) return rc;
  if (!c2w || !t_vals) return set_error(NERF_E_INVALID, "nerf_render: null argument");
  if (width <= 0 || height <= 0 || row0 < 0 || row1 > height || row0 > row1)
    return set_error(NERF_E_INVALID, "nerf_render: bad image/rows %dx%d [%d,%d)", width, height, row0, row1);
  if (row1 > row0 && (!rgb_out || !depth_out)) return set_error(NERF_E_INVALID, "nerf_render: null output");
  if (n_samples <= 0 || n_samples > 1024 || n_importance < 0 || n_importance > 1024 ||
      (n_importance > 0 && (n_samples < 2 || n_samples > 256)))
    return set_error(NERF_E_INVALID, "nerf_render: bad sample counts %d+%d", n_samples, n_importance);
  // any render that gets this far may overwrite the z buffer: the last fine z stays readable
  // only if this render's importance stage completes (set again there)
  ctx->last_zfine = nullptr;
  const long n_rays = long(row1 - row0) * width;
  if (n_rays == 0) return NERF_OK;
  const int n_fine = n_samples + n_importance;
  if (n_rays * n_fine > 0x7FFFFFFFL * 128L) return set_error(NERF_E_INVALID, "nerf_render: too many samples");
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (ctx->n_frames > 0 && s != ctx->last_stream) {
    // another stream than the last render's: order this render after that one
    // (the uploads it skips below and the scratch buffers are shared)
    HIP_TRY(hipStreamWaitEvent(s, ctx->frames[(ctx->n_frames - 1) % nerf_ctx::kEvFrames].ev[NERF_N_STAGES], 0));
  }

  // z table (base_renderer.py:274-275) and the importance draw
  std::vector<float> hz(n_samples), hu(n_importance);
  nerf_uniform_z(t_vals, n_samples, near_, far_, hz.data());
  for (int k = 0; k < n_importance; ++k)
    hu[k] = u ? u[k] : (n_importance > 1 ? float(k) / float(n_importance - 1) : 0.0f);

  if ((rc = grow(ctx->rays, ctx->rays_cap, size_t(n_rays) * 6, "rays")) != NERF_OK) return rc;
  if ((rc = grow(ctx->mlp_out, ctx->mlp_cap, size_t(n_rays) * n_fine * 4, "mlp_out")) != NERF_OK) return rc;
  // z buffer: [table 1024][stratified first-pass z, R x S][fine z, R x (S+N)]
  const size_t strat_floats = t_rand ? size_t(n_rays) * n_samples : 0;
  const size_t zfloats = 1024 + strat_floats + (n_importance > 0 ? size_t(n_rays) * n_fine : 0);
  const size_t z_cap0 = ctx->z_cap, w_cap0 = ctx->w_cap;
  if ((rc = grow(ctx->zbuf, ctx->z_cap, zfloats, "z")) != NERF_OK) return rc;
  const size_t wfloats = 1024 + (n_importance > 0 ? size_t(n_rays) * n_samples : 0);
  if ((rc = grow(ctx->wbuf, ctx->w_cap, wfloats, "weights")) != NERF_OK) return rc;
  if (ctx->z_cap != z_cap0) {   // reallocated: the uploaded tables (and the last fine z) are gone
    ctx->up_zbuf = nullptr;
    ctx->last_zfine = nullptr;
  }
  if (ctx->w_cap != w_cap0) ctx->up_wbuf = nullptr;

  float* d_ztab = ctx->zbuf;
  float* d_zstrat = ctx->zbuf + 1024;
  float* d_zfine = ctx->zbuf + 1024 + strat_floats;
  float* d_u = ctx->wbuf;
  float* d_w = ctx->wbuf + 1024;
  float* rays_o = ctx->rays;
  float* rays_d = ctx->rays + n_rays * 3;
  // upload through pinned staging only what changed since the last render
  const bool need_z = !(ctx->up_zbuf == ctx->zbuf && ctx->up_z == hz);
  const bool need_u = n_importance > 0 && !(ctx->up_wbuf == ctx->wbuf && ctx->up_u == hu);
  if (need_z || need_u) {
    HIP_TRY(hipEventSynchronize(ctx->stage_ev));   // host_stage no longer feeds an earlier copy
    if (need_z) {
      std::memcpy(ctx->host_stage, hz.data(), sizeof(float) * n_samples);
      HIP_TRY(hipMemcpyAsync(d_ztab, ctx->host_stage, sizeof(float) * n_samples, hipMemcpyHostToDevice, s));
      ctx->up_z = hz;
      ctx->up_zbuf = ctx->zbuf;
    }
    if (need_u) {
      std::memcpy(ctx->host_stage + 1024, hu.data(), sizeof(float) * n_importance);
      HIP_TRY(hipMemcpyAsync(d_u, ctx->host_stage + 1024, sizeof(float) * n_importance, hipMemcpyHostToDevice, s));
      ctx->up_u = hu;
      ctx->up_wbuf = ctx->wbuf;
    }
    HIP_TRY(hipEventRecord(ctx->stage_ev, s));
  }

  nerf_ctx::Frame& fr = ctx->frames[ctx->n_frames % nerf_ctx::kEvFrames];
  for (bool& b : fr.ran) b = false;
  fr.profiled = ctx->profiling;
  auto mark = [&](int i) -> int {
    if (ctx->profiling) HIP_TRY(hipEventRecord(fr.ev[i], s));
    return NERF_OK;
  };
  if ((rc = mark(0)) != NERF_OK) return rc;
  HIP_TRY(launch_generate_rays(c2w, width, height, row0, row1, focal, rays_o, rays_d, s));
  // first-pass samples: the shared table, or stratified per ray (rendering.py:42-47)
  const float* z_first = d_ztab;
  int z_first_stride = 0;
  if (t_rand) {
    HIP_TRY(launch_sample(d_ztab, t_rand, int(n_rays), n_samples, nullptr, nullptr, d_zstrat, nullptr, s));
    z_first = d_zstrat;
    z_first_stride = n_samples;
  }
  fr.ran[0] = true;
  if ((rc = mark(1)) != NERF_OK) return rc;
  const float* z_main = z_first;
  int z_stride = z_first_stride;
  if (n_importance > 0) {
    // bf16 / fp8 coarse pass with whole segments: the weights come out of the MLP
    // epilogue (in-segment weight per sample + the segment records) and the
    // sampler scales them by the earlier segments' transmittance; otherwise the
    // (sigma, rgb) buffer and the sequential composite kernel (the coarse image
    // itself is not an output of render_image)
    const bool fuse_coarse = (ctx->fused_composite & 2) && (coarse_prec == NERF_BF16 || coarse_prec == NERF_FP8) &&
                             n_samples % 32 == 0 &&
                             n_importance <= 1024;
    SampleSrc src{rays_o, rays_d, z_first, z_first_stride, n_samples, nullptr, nullptr};
    HIP_TRY(run_mlp(ctx, NERF_NET_COARSE, coarse_prec, src, n_rays * n_samples, ctx->mlp_out, false, s,
                    fuse_coarse ? ctx->mlp_out : nullptr, fuse_coarse ? d_w : nullptr));
    fr.ran[1] = true;
    if ((rc = mark(2)) != NERF_OK) return rc;
    if (!fuse_coarse)
      HIP_TRY(launch_composite(ctx->mlp_out, 4, ctx->mlp_out + 1, 4, z_first, z_first_stride, rays_d, int(n_rays),
                               n_samples, rgb_out, depth_out, nullptr, d_w, s, os));
    HIP_TRY(launch_importance(z_first, z_first_stride, d_w, u_rays ? u_rays : d_u, u_rays ? n_importance : 0,
                              int(n_rays), n_samples, n_importance, d_zfine, s,
                              fuse_coarse ? ctx->mlp_out : nullptr));
    fr.ran[2] = true;
    z_main = d_zfine;
    z_stride = n_fine;
    ctx->last_zfine = d_zfine;
    ctx->last_zfine_rays = n_rays;
    ctx->last_zfine_per_ray = n_fine;
  } else {
    // no importance stage: this render may overwrite where the last fine z lived
    // (the stratified first-pass z shares the z buffer), so it is no longer readable
    ctx->last_zfine = nullptr;
    if ((rc = mark(2)) != NERF_OK) return rc;
  }
  if ((rc = mark(3)) != NERF_OK) return rc;
  // bf16 / fp8 / the split paths with whole 32-sample segments per ray: compositing
  // fused into the MLP epilogue (one record per segment), then chained per ray; the
  // fp32 parity path keeps the sequential composite kernel
  const bool fused = (ctx->fused_composite & 1) &&
                     (precision == NERF_BF16 || precision == NERF_FP8 || precision == NERF_BF16X3 ||
                      precision == NERF_F16X3) &&
                     n_fine > 1 && n_fine % 32 == 0;
  {
    SampleSrc src{rays_o, rays_d, z_main, z_stride, n_fine, nullptr, nullptr};
    HIP_TRY(run_mlp(ctx, net_main, precision, src, n_rays * n_fine, ctx->mlp_out, false, s,
                    fused ? ctx->mlp_out : nullptr));
    fr.ran[3] = true;
  }
  if ((rc = mark(4)) != NERF_OK) return rc;
  if (fused)
    HIP_TRY(launch_composite_segments(ctx->mlp_out, int(n_rays), n_fine / 32, rgb_out, depth_out, s, os));
  else
    HIP_TRY(launch_composite(ctx->mlp_out, 4, ctx->mlp_out + 1, 4, z_main, z_stride, rays_d, int(n_rays), n_fine,
                             rgb_out, depth_out, nullptr, nullptr, s, os));
  fr.ran[4] = true;
  HIP_TRY(hipEventRecord(fr.ev[NERF_N_STAGES], s));
  ++ctx->n_frames;
  ctx->last_stream = s;
  return NERF_OK;
}

}  // namespace

extern "C" {

int nerf_render_sampled(nerf_ctx* ctx, const float* c2w, int width, int height, int row0, int row1, float focal,
                        float near_, float far_, const float* t_vals, int n_samples, int n_importance, const float* u,
                        const float* t_rand, const float* u_rays, int precision, float* rgb_out, float* depth_out,
                        void* stream) {
  return render_impl(ctx, c2w, width, height, row0, row1, focal, near_, far_, t_vals, n_samples, n_importance, u,
                     t_rand, u_rays, precision, rgb_out, depth_out, OutStrides{}, stream);
}

int nerf_render_band(nerf_ctx* ctx, const float* c2w, int width, int height, int row0, int row1, float focal,
                     float near_, float far_, const float* t_vals, int n_samples, int n_importance, const float* u,
                     int precision, float* rgbd_out, void* stream) {
  if (row1 > row0 && !rgbd_out) return set_error(NERF_E_INVALID, "nerf_render_band: null output");
  return render_impl(ctx, c2w, width, height, row0, row1, focal, near_, far_, t_vals, n_samples, n_importance, u,
                     nullptr, nullptr, precision, rgbd_out, rgbd_out ? rgbd_out + 3 : nullptr, OutStrides{4, 4},
                     stream);
}

int nerf_ctx_range_status(nerf_ctx* ctx, void* stream) {
  if (!ctx) return set_error(NERF_E_INVALID, "nerf_ctx_range_status: null context");
  DeviceGuard g(ctx->device);
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  int flag = 0;
  HIP_TRY(hipMemcpy(&flag, ctx->d_range, sizeof(int), hipMemcpyDeviceToHost));
  if (flag == 0) return NERF_OK;
  HIP_TRY(hipMemset(ctx->d_range, 0, sizeof(int)));
  return set_error(NERF_E_RANGE, "NERF_F16X3: an activation reached fp16's range (|x| >= 65520) since the last "
                                 "check; the outputs of those launches are not valid (use NERF_FP32 or NERF_BF16X3)");
}

int nerf_ctx_last_fine_z(nerf_ctx* ctx, long n_rays, int per_ray, float* z_out, void* stream) {
  if (!ctx || !z_out) return set_error(NERF_E_INVALID, "nerf_ctx_last_fine_z: null argument");
  if (!ctx->last_zfine) return set_error(NERF_E_INVALID, "nerf_ctx_last_fine_z: no hierarchical render yet");
  if (n_rays != ctx->last_zfine_rays || per_ray != ctx->last_zfine_per_ray)
    return set_error(NERF_E_INVALID, "nerf_ctx_last_fine_z: the last hierarchical render had %ld rays x %d samples",
                     ctx->last_zfine_rays, ctx->last_zfine_per_ray);
  DeviceGuard g(ctx->device);
  hipStream_t s = (hipStream_t)stream;
  if (s != ctx->last_stream)   // order the copy after the render that wrote the samples
    HIP_TRY(hipStreamWaitEvent(s, ctx->frames[(ctx->n_frames - 1) % nerf_ctx::kEvFrames].ev[NERF_N_STAGES], 0));
  HIP_TRY(hipMemcpyAsync(z_out, ctx->last_zfine, sizeof(float) * size_t(n_rays) * per_ray, hipMemcpyDeviceToDevice, s));
  return NERF_OK;
}

int nerf_positional_encoding(int precision, const float* x, long n, int n_freqs, float* out, void* stream) {
  if (precision != NERF_FP32 && precision != NERF_BF16 && precision != NERF_FP8 && precision != NERF_BF16X3 &&
      precision != NERF_F16X3)
    return set_error(NERF_E_INVALID, "bad precision %d", precision);
  if (n < 0 || (n_freqs != kPosL && n_freqs != kDirL))
    return set_error(NERF_E_INVALID, "nerf_positional_encoding: n %ld, n_freqs %d (the model's are 10 and 4)", n,
                     n_freqs);
  if (n == 0) return NERF_OK;
  if (!x || !out) return set_error(NERF_E_INVALID, "nerf_positional_encoding: null pointer");
  HIP_TRY(launch_encode(x, n, n_freqs, precision == NERF_BF16 || precision == NERF_FP8, out, (hipStream_t)stream));
  return NERF_OK;
}

}  // extern "C"
