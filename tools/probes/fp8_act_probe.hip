// A candidate fp8 activation conversion (round 3 lab; bit-exact but slower inside the
// kernel, not kept: DESIGN.md section 7) on gfx950: v_pk_mul_f32 by 2^-8 with the
// clamp bit (ReLU + saturation at 256 on a pair), then v_cvt_scalef32_pk_fp8_f32 at
// scale 2^-8.  Checked against e4m3(min(max(x, 0), 256)) by tools/probes/fp8_act_probe.py.
//   hipcc -shared -fPIC --offload-arch=gfx950 -O2 fp8_act_probe.hip -o libfp8actprobe.so
#include <hip/hip_runtime.h>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

__global__ void act_kernel(const float* in, unsigned* out, int n_quads) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_quads) return;
  f32x2 lo, hi;
  asm("v_pk_mul_f32 %0, %1, %2 clamp" : "=v"(lo) : "v"(f32x2{in[4 * i], in[4 * i + 1]}), "s"(0x3B8000003B800000ull));
  asm("v_pk_mul_f32 %0, %1, %2 clamp" : "=v"(hi) : "v"(f32x2{in[4 * i + 2], in[4 * i + 3]}), "s"(0x3B8000003B800000ull));
  s16x2 w = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(s16x2{0, 0}, lo[0], lo[1], 0x1p-8f, false);
  w = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(w, hi[0], hi[1], 0x1p-8f, true);
  out[i] = __builtin_bit_cast(unsigned, w);
}

extern "C" int fp8_act_probe(const float* host_in, int n_quads, unsigned* host_out) {
  float* din = nullptr;
  unsigned* dout = nullptr;
  if (hipMalloc(&din, size_t(n_quads) * 16) != hipSuccess) return -1;
  if (hipMalloc(&dout, size_t(n_quads) * 4) != hipSuccess) return -2;
  if (hipMemcpy(din, host_in, size_t(n_quads) * 16, hipMemcpyHostToDevice) != hipSuccess) return -3;
  hipLaunchKernelGGL(act_kernel, dim3((n_quads + 255) / 256), dim3(256), 0, 0, din, dout, n_quads);
  if (hipDeviceSynchronize() != hipSuccess) return -4;
  if (hipMemcpy(host_out, dout, size_t(n_quads) * 4, hipMemcpyDeviceToHost) != hipSuccess) return -5;
  (void)hipFree(din);
  (void)hipFree(dout);
  return 0;
}
