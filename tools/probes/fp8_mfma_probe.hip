// Hardware probe (diagnostic, not part of the library): one wave runs
// v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3) on caller-given per-lane
// fragments and scales, so tests can pin its operand lane maps and the
// meaning of the E8M0 scale operands with exact integer data.
#include <hip/hip_runtime.h>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(const i32x8* a, const i32x8* b, const int* sa, const int* sb, f32x16* d) {
  const int l = threadIdx.x;
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0, sb[l]);
  d[l] = acc;
}

extern "C" int fp8_probe(const void* a, const void* b, const int* sa, const int* sb, float* d) {
  void *da, *db, *dsa, *dsb, *dd;
  if (hipMalloc(&da, 64 * 32) || hipMalloc(&db, 64 * 32) || hipMalloc(&dsa, 256) || hipMalloc(&dsb, 256) ||
      hipMalloc(&dd, 64 * 64))
    return -1;
  (void)hipMemcpy(da, a, 64 * 32, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b, 64 * 32, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, (const i32x8*)da, (const i32x8*)db, (const int*)dsa,
                     (const int*)dsb, (f32x16*)dd);
  const hipError_t e = hipMemcpy(d, dd, 64 * 64, hipMemcpyDeviceToHost);
  (void)hipFree(da); (void)hipFree(db); (void)hipFree(dsa); (void)hipFree(dsb); (void)hipFree(dd);
  return e == hipSuccess ? 0 : -2;
}

typedef short i16x2 __attribute__((ext_vector_type(2)));
// v_cvt_scalef32_pk_fp8_f32 and v_cvt_pk_fp8_f32 on pairs (x[2i], x[2i+1]) with scale s[i]
__global__ void cvt(const float* x, const float* s, unsigned* out, int n) {
  const int i = threadIdx.x;
  if (i >= n) return;
  i16x2 z = {0, 0};
  const i16x2 a = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(z, x[2 * i], x[2 * i + 1], s[i], false);
  const int b = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
  out[2 * i] = __builtin_bit_cast(unsigned, a) & 0xFFFFu;
  out[2 * i + 1] = unsigned(b) & 0xFFFFu;
}

extern "C" int fp8_cvt_probe(const float* x, const float* s, unsigned* out, int n) {
  float *dx, *ds;
  unsigned* dout;
  if (n > 64 || hipMalloc(&dx, 8 * n) || hipMalloc(&ds, 4 * n) || hipMalloc(&dout, 8 * n)) return -1;
  (void)hipMemcpy(dx, x, 8 * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(ds, s, 4 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(cvt, dim3(1), dim3(64), 0, 0, dx, ds, dout, n);
  const hipError_t e = hipMemcpy(out, dout, 8 * n, hipMemcpyDeviceToHost);
  (void)hipFree(dx); (void)hipFree(ds); (void)hipFree(dout);
  return e == hipSuccess ? 0 : -2;
}
