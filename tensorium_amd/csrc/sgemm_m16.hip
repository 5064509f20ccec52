// sgemm_m16.hip — SGEMM / implicit-conv launchers for the 16x16x4 MFMA tile
// shapes (finer output granularity for GEMMs with few output tiles; the
// 4096^3 8-wave shape for the large-GEMM comparison).
// Kernel template: sgemm_kernel.hpp.
#include "sgemm_kernel.hpp"

namespace tns {

#define TNS_M16(ID, KIND)                                                                   \
  hipError_t launch_shape_##ID(const GemmArgs& a, bool ta, bool tb, bool av, bool bv,     \
                               hipStream_t s) {                                           \
    return sgemm_detail::KIND<sgemm_detail::S##ID>(a, ta, tb, av, bv, s);                 \
  }
TNS_M16(64x64m16, launch_full)
TNS_M16(32x32m16, launch_full)
TNS_M16(64x32m16, launch_nn4)
TNS_M16(32x64m16, launch_nn4)
TNS_M16(128x128m16, launch_nn4)
TNS_M16(256x256w8m16, launch_trans4)
#undef TNS_M16

#define TNS_M16C(ID)                                                             \
  hipError_t launch_conv_##ID(const GemmArgs& a, bool av, hipStream_t s) {       \
    return sgemm_detail::launch_conv<sgemm_detail::S##ID>(a, av, s);             \
  }
TNS_M16C(64x64m16)
TNS_M16C(32x32m16)
TNS_M16C(64x32m16)
TNS_M16C(32x64m16)
#undef TNS_M16C

}  // namespace tns
