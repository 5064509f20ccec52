// tns_act.hpp — device-side activation formulas (TActivationType ordinals,
// ntypes.pas:66-71), shared by the elementwise kernels and the SGEMM epilogue.
// Restates nactivation.pas scalar formulas (272-501) and the AVX2
// leaky_array constant (0.1f, nactivation.pas:234-267).  exp is evaluated in
// double and rounded where the Pascal stores it (FPC's exp returns a real):
// the same values as the oracle's libm up to exp's last-ulp differences.  Compiled with
// -ffp-contract=off so no multiply/add pair is fused behind our back.
#pragma once
#include <hip/hip_runtime.h>

#include "tns_internal.hpp"

namespace tns {

// logistic / tanh evaluate exp in double: kept out of the GEMM epilogue
// (the conv drivers apply them in a separate elementwise pass — the same
// values, since the activation is applied to the stored single anyway)
// every supported activation except logistic / tanh (GEMM epilogues)
__device__ __forceinline__ float act_apply_cheap(float x, int act) {
  switch (act) {
    case 1:  // acRELU: x*(x>0)
      return x * (float)(x > 0.0f);
    case 8:
    case 9:  // acREVLEAKY / acLEAKY: if 0 > x then 0.1f*x
      return (0.0f > x) ? 0.1f * x : x;
    case 13:  // acHARDTAN
      return x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
    default:  // acLINEAR (4) and anything the host rejected earlier
      return x;
  }
}

__device__ __forceinline__ float act_apply(float x, int act) {
  if (act == 0)  // acLOGISTIC: 1/(1+exp(-x)) — exp's real result, one rounding
    return (float)(1.0 / (1.0 + exp(-(double)x)));
  if (act == 6) {  // acTANH: px := exp(x); nx := exp(-x) (singles); (px-nx)/(px+nx)
    const float px = (float)exp((double)x), nx = (float)exp(-(double)x);
    return (px - nx) / (px + nx);
  }
  return act_apply_cheap(x, act);
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
