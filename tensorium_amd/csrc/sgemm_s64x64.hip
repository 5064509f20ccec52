// sgemm_s64x64.hip — SGEMM launchers for the 64x64 tile (4 waves of 32x32):
// the most blocks per problem, for GEMMs too small to fill 256 CUs with the
// larger tiles (no split-K: it would change the k order, DESIGN.md Numerics).
// Kernel template: sgemm_kernel.hpp.
#include "sgemm_kernel.hpp"

namespace tns {

hipError_t launch_shape_64x64(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  return sgemm_detail::launch_full<sgemm_detail::S64x64>(a, ta, tb, av, bv, s);
}

hipError_t launch_conv_64x64(const GemmArgs& a, bool av, hipStream_t s) {
  return sgemm_detail::launch_conv<sgemm_detail::S64x64>(a, av, s);
}

}  // namespace tns
