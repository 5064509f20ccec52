// sgemm_s128.hip — SGEMM launchers for tile shapes 128x128, 128x64, 64x128.
// Kernel template: sgemm_kernel.hpp (split across files so hipcc builds them in parallel).
#include "sgemm_kernel.hpp"

namespace tns {

hipError_t launch_shape_128x128(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_full<sgemm_detail::S128x128>(a, ta, tb, av, bv, s);
}

hipError_t launch_shape_128x64(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_full<sgemm_detail::S128x64>(a, ta, tb, av, bv, s);
}

hipError_t launch_shape_64x128(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_full<sgemm_detail::S64x128>(a, ta, tb, av, bv, s);
}


hipError_t launch_conv_128x64(const GemmArgs& a, bool av, hipStream_t s) {
  return sgemm_detail::launch_conv<sgemm_detail::S128x64>(a, av, s);
}

hipError_t launch_conv_64x128(const GemmArgs& a, bool av, hipStream_t s) {
  return sgemm_detail::launch_conv<sgemm_detail::S64x128>(a, av, s);
}

}  // namespace tns
