// sgemm_big.hip — SGEMM launchers for tile shapes 256x256, 256x256k16, 256x128, 128x256, 256x128k16.
// Kernel template: sgemm_kernel.hpp (split across files so hipcc builds them in parallel).
#include "sgemm_kernel.hpp"

namespace tns {

hipError_t launch_shape_256x256(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_nn4<sgemm_detail::S256x256>(a, ta, tb, av, bv, s);
}

hipError_t launch_shape_256x256k16(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_nn4<sgemm_detail::S256x256k16>(a, ta, tb, av, bv, s);
}

hipError_t launch_shape_256x128(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_nn4<sgemm_detail::S256x128>(a, ta, tb, av, bv, s);
}

hipError_t launch_shape_128x256(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_nn4<sgemm_detail::S128x256>(a, ta, tb, av, bv, s);
}


hipError_t launch_shape_256x128k16(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_nn4<sgemm_detail::S256x128k16>(a, ta, tb, av, bv, s);
}

}  // namespace tns

