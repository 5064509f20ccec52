// sgemm_s256.hip — SGEMM launcher for the 256x256 (8-wave) tile shape, the
// production shape for large GEMMs.  Kernel template: sgemm_kernel.hpp.
#include "sgemm_kernel.hpp"

namespace tns {

hipError_t launch_shape_256x256w8(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_trans4<sgemm_detail::S256x256w8>(a, ta, tb, av, bv, s);
}


}  // namespace tns
