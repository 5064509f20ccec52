// tns_act.hpp — device-side activation formulas (TActivationType ordinals,
// ntypes.pas:66-71), shared by the elementwise kernels and the SGEMM epilogue.
// Restates nactivation.pas scalar formulas (272-501) and the AVX2
// leaky_array constant (0.1f, nactivation.pas:234-267).  Compiled with
// -ffp-contract=off so no multiply/add pair is fused behind our back.
#pragma once
#include <hip/hip_runtime.h>

namespace tns {

__device__ __forceinline__ float act_apply(float x, int act) {
  switch (act) {
    case 0:  // acLOGISTIC: 1/(1+exp(-x))
      return 1.0f / (1.0f + expf(-x));
    case 1:  // acRELU: x*(x>0)
      return x * (float)(x > 0.0f);
    case 6:  // acTANH
      return tanhf(x);
    case 8:
    case 9:  // acREVLEAKY / acLEAKY: if 0 > x then 0.1f*x
      return (0.0f > x) ? 0.1f * x : x;
    case 13:  // acHARDTAN
      return x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
    default:  // acLINEAR (4) and anything the host rejected earlier
      return x;
  }
}

__device__ __forceinline__ float grad_apply(float y, int act) {
  switch (act) {
    case 0:
      return (1.0f - y) * y;  // logistic_gradient
    case 1:
      return (float)(y > 0.0f);
    case 6:
      return 1.0f - y * y;
    case 8:
    case 9:
      return y > 0.0f ? 1.0f : 0.1f;  // leaky_gradient
    case 13:
      return (y > -1.0f && y < 1.0f) ? 1.0f : 0.0f;
    default:
      return 1.0f;
  }
}

}  // namespace tns
