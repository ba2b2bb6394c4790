/*
 * Plain-C host driving libnerf_mi355x.so through include/nerf_mi355x.h only:
 * no Python, no torch.  Renders one frame of the reference benchmark
 * (render_image, base_renderer/pytorch_renderers semantics) from a checkpoint
 * given as 22 raw little-endian fp32 tensors in state-dict order (the layout
 * NERF_N_PARAMS documents), and writes RGB and depth as raw fp32.
 *
 *   render_c <params.bin> <width> <height> <spp> <precision 0|1|2|3|4> <out.bin> [t.bin]
 *
 * t.bin (optional): the spp fp32 values of torch.linspace(0, 1, spp), for bit
 * parity with the Python host; otherwise the table is computed here.
 *
 * Device buffers come from the HIP runtime (hipMalloc); everything else is the
 * C ABI.  Build: see examples/Makefile.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>

#include "nerf_mi355x.h"

static const int kOut[11] = {256, 256, 256, 256, 256, 256, 256, 256, 1, 128, 3};
static const int kIn[11] = {63, 256, 256, 256, 319, 256, 256, 256, 256, 283, 128};

static int die(const char* what, int rc) {
  fprintf(stderr, "%s failed (%d): %s\n", what, rc, nerf_last_error());
  return 1;
}

int main(int argc, char** argv) {
  if (argc != 7 && argc != 8) {
    fprintf(stderr, "usage: %s params.bin width height spp precision out.bin [t.bin]\n", argv[0]);
    return 2;
  }
  const int width = atoi(argv[2]), height = atoi(argv[3]), spp = atoi(argv[4]), precision = atoi(argv[5]);
  FILE* f = fopen(argv[1], "rb");
  if (!f) return die("fopen params", -1);
  float* tensors[NERF_N_PARAMS];
  for (int i = 0; i < NERF_N_PARAMS; ++i) {
    const size_t n = (i & 1) ? (size_t)kOut[i / 2] : (size_t)kOut[i / 2] * kIn[i / 2];
    tensors[i] = (float*)malloc(n * sizeof(float));
    if (fread(tensors[i], sizeof(float), n, f) != n) return die("read params", -1);
  }
  fclose(f);

  nerf_ctx* ctx = NULL;
  int rc;
  if ((rc = nerf_ctx_create(0, &ctx)) != NERF_OK) return die("nerf_ctx_create", rc);
  char name[256];
  if (nerf_device_name(0, name, sizeof name) == NERF_OK) fprintf(stderr, "device: %s\n", name);
  for (int net = 0; net < 2; ++net)   /* same weights for the coarse and fine slots */
    if ((rc = nerf_ctx_load_weights(ctx, net, (const float* const*)tensors, NERF_N_PARAMS)) != NERF_OK)
      return die("nerf_ctx_load_weights", rc);

  /* torch.linspace(0, 1, spp) in fp32: start + i*step for i < n/2, end - (n-1-i)*step
   * above (ATen's symmetric fill), step = (end-start)/(n-1) */
  float* t = (float*)malloc(sizeof(float) * (size_t)spp);
  const float step = spp > 1 ? 1.0f / (float)(spp - 1) : 0.0f;
  for (int i = 0; i < spp; ++i) t[i] = i < spp / 2 ? (float)i * step : 1.0f - (float)(spp - 1 - i) * step;
  if (argc == 8) {
    FILE* tf = fopen(argv[7], "rb");
    if (!tf || fread(t, sizeof(float), (size_t)spp, tf) != (size_t)spp) return die("read t table", -1);
    fclose(tf);
  }

  const float pose[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 4, 0, 0, 0, 1};   /* suite view 0 */
  const size_t n_rays = (size_t)width * height;
  float *rgb_d, *depth_d;
  if (hipMalloc((void**)&rgb_d, n_rays * 3 * sizeof(float)) != hipSuccess ||
      hipMalloc((void**)&depth_d, n_rays * sizeof(float)) != hipSuccess)
    return die("hipMalloc", -2);
  if ((rc = nerf_render(ctx, pose, width, height, 0, height, 800.0f, 2.0f, 6.0f, t, spp, 0, NULL, precision, rgb_d,
                        depth_d, NULL)) != NERF_OK)
    return die("nerf_render", rc);
  float* out = (float*)malloc(n_rays * 4 * sizeof(float));
  if (hipMemcpy(out, rgb_d, n_rays * 3 * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(out + n_rays * 3, depth_d, n_rays * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
    return die("hipMemcpy", -2);
  FILE* o = fopen(argv[6], "wb");
  if (!o || fwrite(out, sizeof(float), n_rays * 4, o) != n_rays * 4) return die("write output", -1);
  fclose(o);
  fprintf(stderr, "rendered %dx%d x %d spp (precision %d)\n", width, height, spp, precision);
  (void)hipFree(rgb_d);
  (void)hipFree(depth_d);
  nerf_ctx_destroy(ctx);
  return 0;
}
