// NERF_F16X3: the split-fp16 instantiations of mlp_x3.h (the parity-grade fast path),
// built with the MFMA accumulators in VGPRs (-amdgpu-mfma-vgpr-form, Makefile).
#include "mlp_x3.h"

namespace nerf {

hipError_t launch_mlp_f16x3(const void* blob, const float* params, const SampleSrc& src, long n_points, float* out,
                            bool explicit_points, hipStream_t stream, float* seg, int* range_flag, int layout) {
  return launch_x3<OpF16>(blob, params, src, n_points, out, explicit_points, stream, seg, range_flag, layout);
}

}  // namespace nerf
