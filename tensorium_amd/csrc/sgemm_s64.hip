// sgemm_s64.hip — SGEMM launchers for tile shapes 64x256, 32x256.
// Kernel template: sgemm_kernel.hpp (split across files so hipcc builds them in parallel).
#include "sgemm_kernel.hpp"

namespace tns {

hipError_t launch_shape_64x256(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_full<sgemm_detail::S64x256>(a, ta, tb, av, bv, s);
}

hipError_t launch_shape_32x256(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_full<sgemm_detail::S32x256>(a, ta, tb, av, bv, s);
}


hipError_t launch_conv_32x256(const GemmArgs& a, bool av, hipStream_t s) {
  return sgemm_detail::launch_conv<sgemm_detail::S32x256>(a, av, s);
}

}  // namespace tns
