// Hardware probe (diagnostic, not part of the library): the numerics of the
// fp8 path's two instructions on gfx950, on random data, for comparison with
// exact host arithmetic (tools/probes/fp8_numerics_probe.py):
//   * v_cvt_scalef32_pk_fp8_f32 / v_cvt_pk_fp8_f32: rounding of x / scale to e4m3;
//   * v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3, E8M0 scales) and
//     v_mfma_f32_32x32x16_bf16: D = C + scaled A.B, as the accumulation chain sees it.
//   hipcc -shared -fPIC --offload-arch=gfx950 -O2 fp8_numerics_probe.hip -o libfp8num.so
#include <hip/hip_runtime.h>

typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__global__ void cvt_kernel(const float* x, const float* s, unsigned* out_scaled, unsigned* out_plain, int n_pairs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_pairs) return;
  i16x2 z = {0, 0};
  const i16x2 a = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(z, x[2 * i], x[2 * i + 1], s[i], false);
  const int b = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
  out_scaled[i] = __builtin_bit_cast(unsigned, a) & 0xFFFFu;
  out_plain[i] = unsigned(b) & 0xFFFFu;
}

// one wave per trial: a, b [trial][64 lanes][32 B]; sa, sb [trial][64]; c, d [trial][64][16]
__global__ void mfma8_kernel(const i32x8* a, const i32x8* b, const int* sa, const int* sb, const f32x16* c,
                             f32x16* d) {
  const int t = blockIdx.x, l = threadIdx.x;
  d[t * 64 + l] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[t * 64 + l], b[t * 64 + l], c[t * 64 + l], 0, 0,
                                                                  0, sa[t * 64 + l], 0, sb[t * 64 + l]);
}
// a, b [trial][64][8 bf16]
__global__ void mfma16_kernel(const bf16x8* a, const bf16x8* b, const f32x16* c, f32x16* d) {
  const int t = blockIdx.x, l = threadIdx.x;
  d[t * 64 + l] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[t * 64 + l], b[t * 64 + l], c[t * 64 + l], 0, 0, 0);
}

template <typename T>
static int up(T** d, const void* h, size_t n) {
  if (hipMalloc((void**)d, n) != hipSuccess) return -1;
  return h && hipMemcpy(*d, h, n, hipMemcpyHostToDevice) != hipSuccess ? -1 : 0;
}

extern "C" int probe_cvt(const float* x, const float* s, unsigned* out_scaled, unsigned* out_plain, int n_pairs) {
  float *dx, *ds;
  unsigned *d1, *d2;
  if (up(&dx, x, 8L * n_pairs) || up(&ds, s, 4L * n_pairs) || up(&d1, nullptr, 4L * n_pairs) ||
      up(&d2, nullptr, 4L * n_pairs))
    return -1;
  hipLaunchKernelGGL(cvt_kernel, dim3((n_pairs + 255) / 256), dim3(256), 0, 0, dx, ds, d1, d2, n_pairs);
  if (hipMemcpy(out_scaled, d1, 4L * n_pairs, hipMemcpyDeviceToHost) != hipSuccess) return -2;
  if (hipMemcpy(out_plain, d2, 4L * n_pairs, hipMemcpyDeviceToHost) != hipSuccess) return -2;
  (void)hipFree(dx); (void)hipFree(ds); (void)hipFree(d1); (void)hipFree(d2);
  return 0;
}

extern "C" int probe_mfma8(const void* a, const void* b, const int* sa, const int* sb, const float* c, float* d,
                           int trials) {
  i32x8 *da, *db;
  int *dsa, *dsb;
  f32x16 *dc, *dd;
  const size_t n = size_t(trials) * 64;
  if (up(&da, a, n * 32) || up(&db, b, n * 32) || up(&dsa, sa, n * 4) || up(&dsb, sb, n * 4) || up(&dc, c, n * 64) ||
      up(&dd, nullptr, n * 64))
    return -1;
  hipLaunchKernelGGL(mfma8_kernel, dim3(trials), dim3(64), 0, 0, da, db, dsa, dsb, dc, dd);
  if (hipMemcpy(d, dd, n * 64, hipMemcpyDeviceToHost) != hipSuccess) return -2;
  (void)hipFree(da); (void)hipFree(db); (void)hipFree(dsa); (void)hipFree(dsb); (void)hipFree(dc); (void)hipFree(dd);
  return 0;
}

extern "C" int probe_mfma16(const void* a, const void* b, const float* c, float* d, int trials) {
  bf16x8 *da, *db;
  f32x16 *dc, *dd;
  const size_t n = size_t(trials) * 64;
  if (up(&da, a, n * 16) || up(&db, b, n * 16) || up(&dc, c, n * 64) || up(&dd, nullptr, n * 64)) return -1;
  hipLaunchKernelGGL(mfma16_kernel, dim3(trials), dim3(64), 0, 0, da, db, dc, dd);
  if (hipMemcpy(d, dd, n * 64, hipMemcpyDeviceToHost) != hipSuccess) return -2;
  (void)hipFree(da); (void)hipFree(db); (void)hipFree(dc); (void)hipFree(dd);
  return 0;
}
