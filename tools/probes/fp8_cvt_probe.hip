// Overflow behaviour of v_cvt_scalef32_pk_fp8_f32 (OCP e4m3) on gfx950: does a
// value above 448 * scale saturate to 0x7E / 0xFE, or become the NaN 0x7F / 0xFF?
// (Input to the fp8 static-activation-scale design)
//   hipcc -shared -fPIC --offload-arch=gfx950 -O2 fp8_cvt_probe.hip -o libfp8cvtprobe.so
#include <hip/hip_runtime.h>

typedef short i16x2 __attribute__((ext_vector_type(2)));

__global__ void cvt_kernel(const float* in, float scale, unsigned* out, int n_pairs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_pairs) return;
  i16x2 w = {0, 0};
  w = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(w, in[2 * i], in[2 * i + 1], scale, false);
  out[i] = unsigned(__builtin_bit_cast(unsigned, w)) & 0xFFFFu;
}

extern "C" int fp8_cvt_probe(const float* host_in, int n_pairs, float scale, unsigned* host_out) {
  float* din = nullptr;
  unsigned* dout = nullptr;
  if (hipMalloc(&din, n_pairs * 8) != hipSuccess) return -1;
  if (hipMalloc(&dout, n_pairs * 4) != hipSuccess) return -2;
  if (hipMemcpy(din, host_in, n_pairs * 8, hipMemcpyHostToDevice) != hipSuccess) return -3;
  hipLaunchKernelGGL(cvt_kernel, dim3((n_pairs + 63) / 64), dim3(64), 0, 0, din, scale, dout, n_pairs);
  if (hipDeviceSynchronize() != hipSuccess) return -4;
  if (hipMemcpy(host_out, dout, n_pairs * 4, hipMemcpyDeviceToHost) != hipSuccess) return -5;
  (void)hipFree(din);
  (void)hipFree(dout);
  return 0;
}
