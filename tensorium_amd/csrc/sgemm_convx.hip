// sgemm_convx.hip — SGEMM / implicit-conv launchers for the 8-wave and
// depth-1 tile shapes (conv tile sweep candidates).
// Kernel template: sgemm_kernel.hpp.
#include "sgemm_kernel.hpp"

namespace tns {

#define TNS_CX(ID)                                                                          \
  hipError_t launch_shape_##ID(const GemmArgs& a, bool ta, bool tb, bool av, bool bv,     \
                               hipStream_t s) {                                           \
    return sgemm_detail::launch_nn4<sgemm_detail::S##ID>(a, ta, tb, av, bv, s);           \
  }                                                                                       \
  hipError_t launch_conv_##ID(const GemmArgs& a, bool av, hipStream_t s) {                \
    return sgemm_detail::launch_conv<sgemm_detail::S##ID>(a, av, s);                      \
  }
TNS_CX(128x64w8)
TNS_CX(64x128w8)
TNS_CX(128x128w8)
TNS_CX(64x64d1)
TNS_CX(64x64w8m16)
#undef TNS_CX

}  // namespace tns
