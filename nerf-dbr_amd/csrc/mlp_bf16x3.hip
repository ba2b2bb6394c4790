// NERF_BF16X3: the split-bf16 instantiations of mlp_x3.h (the render pass, explicit
// points and the training forward).  Built with -amdgpu-mfma-vgpr-form like the f16 unit
// (-2.2 %, bit-identical); round 3's wrong sigmas under that flag came from the asm
// fragment reads' waits, which the compiler now counts (nerf_asm.h, Makefile).
#include "mlp_x3.h"

namespace nerf {

hipError_t launch_mlp_bf16x3(const void* blob, const float* params, const SampleSrc& src, long n_points, float* out,
                             bool explicit_points, hipStream_t stream, float* seg) {
  return launch_x3<OpBf16>(blob, params, src, n_points, out, explicit_points, stream, seg, nullptr);
}

hipError_t launch_mlp_bf16x3_train(const void* blob, const float* params, const SampleSrc& src, long n_points,
                                   const X3TrainOut& o, hipStream_t stream) {
  if (n_points <= 0) return hipSuccess;
  if (n_points >= (1L << 27)) return hipErrorInvalidValue;   // the ReLU-bit words' 32-bit byte offsets
  const long tiles = (n_points + kSamplesPerBlock - 1) / kSamplesPerBlock;
  const long blocks = tiles < current_device_cus() ? tiles : current_device_cus();   // one workgroup per CU
  hipLaunchKernelGGL((mlp_x3_kernel<false, true, OpBf16>), dim3(unsigned(blocks)), dim3(kThreads), 0, stream,
                     (const char*)blob, params, src, n_points, (f32x4*)nullptr, (f32x4*)nullptr, o, nullptr);
  return hipGetLastError();
}

}  // namespace nerf
