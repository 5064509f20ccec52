// elementwise.hip — wave64 elementwise kernels for gfx950 (HBM-bound).
//
//   forward_bias    vsAddB / TNNCuda.forwardBias (ntensors.pas:4066-4093,
//                   nncuda.pas:582): dst[(b*F+f)*bs + j] += bias[f*incb]
//   activate        activate_array (nactivation.pas:508-621)
//   bias_activate   the two above in one pass (conv forward, unfused GEMM path)
//   derive          gradient_array (nactivation.pas:624-717)
//   backward_bias   addSums (ntensors.pas:7729-7781) — one workgroup per
//                   output, fixed-order tree reduction (deterministic; not
//                   the reference's sequential order)
//   axpy/scale/fill/copy/clamp  TNNCuda BLAS-1 helpers
// Contiguous kernels move 16 B per lane (float4) when alignment allows.
#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {

bool act_supported(int act) {
  switch (act) {
    case 0: case 1: case 4: case 6: case 8: case 9: case 13:
      return true;
    default:
      return false;
  }
}

namespace {

constexpr int TPB = 256;

inline unsigned grid_for(int64_t work) {
  int64_t g = (work + TPB - 1) / TPB;
  // grid-stride loops cover the rest; 256 CUs x 16 blocks keeps HBM busy
  if (g > 256 * 64) g = 256 * 64;
  if (g < 1) g = 1;
  return (unsigned)g;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// dst is [batch][F][bs]; VEC elements per thread along bs (bs % VEC == 0).
template <int VEC, bool ACT>
__global__ __launch_bounds__(TPB) void bias_act_kernel(float* __restrict__ dst, int64_t F,
                                                       int64_t bs, const float* __restrict__ bias,
                                                       int64_t incb, int64_t total_vec, int act) {
  const int64_t bsv = bs / VEC;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < total_vec;
       i += (int64_t)gridDim.x * TPB) {
    const int64_t blk = i / bsv;  // (b*F + f)
    const int64_t f = blk % F;
    const float bb = bias[f * incb];
    if constexpr (VEC == 4) {
      float4 v = reinterpret_cast<float4*>(dst)[i];
      v.x = v.x + bb; v.y = v.y + bb; v.z = v.z + bb; v.w = v.w + bb;
      if (ACT) {
        v.x = act_apply(v.x, act); v.y = act_apply(v.y, act);
        v.z = act_apply(v.z, act); v.w = act_apply(v.w, act);
      }
      reinterpret_cast<float4*>(dst)[i] = v;
    } else {
      float v = dst[i] + bb;
      if (ACT) v = act_apply(v, act);
      dst[i] = v;
    }
  }
}

template <int VEC>
__global__ __launch_bounds__(TPB) void act_kernel(float* __restrict__ x, int64_t nvec, int act) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * TPB) {
    if constexpr (VEC == 4) {
      float4 v = reinterpret_cast<float4*>(x)[i];
      v.x = act_apply(v.x, act); v.y = act_apply(v.y, act);
      v.z = act_apply(v.z, act); v.w = act_apply(v.w, act);
      reinterpret_cast<float4*>(x)[i] = v;
    } else {
      x[i] = act_apply(x[i], act);
    }
  }
}

__global__ __launch_bounds__(TPB) void derive_kernel(const float* __restrict__ x, int64_t n,
                                                     int act, float* __restrict__ delta) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * TPB)
    delta[i] = delta[i] * grad_apply(x[i], act);
}

// one workgroup per output element; tree reduction in a fixed order.
__global__ __launch_bounds__(TPB) void backward_bias_kernel(float* __restrict__ dst, int64_t nDst,
                                                            const float* __restrict__ src,
                                                            int64_t bs, int64_t batch,
                                                            int64_t incb) {
  const int64_t i = blockIdx.x;
  float s = 0.0f;
  const int64_t per = batch * bs;
  for (int64_t t = threadIdx.x; t < per; t += TPB) {
    const int64_t b = t / bs, j = t - b * bs;
    s += src[(b * nDst + i) * bs + j];
  }
  // wave reduce (64 lanes) then across the 4 waves
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  __shared__ float part[TPB / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = (part[0] + part[1]) + (part[2] + part[3]);
    dst[i * incb] = dst[i * incb] + tot;
  }
}

__global__ __launch_bounds__(TPB) void axpy_kernel(int64_t n, float a, const float* __restrict__ x,
                                                   int64_t incx, float* __restrict__ y,
                                                   int64_t incy) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * TPB)
    y[i * incy] = fmaf(a, x[i * incx], y[i * incy]);  // saxpy: one FMA
}

__global__ __launch_bounds__(TPB) void scale_kernel(int64_t n, float a, float* __restrict__ x,
                                                    int64_t stride) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * TPB)
    x[i * stride] = a * x[i * stride];
}

__global__ __launch_bounds__(TPB) void fill_kernel(int64_t n, float* __restrict__ x, float v,
                                                   int64_t stride) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * TPB)
    x[i * stride] = v;
}

__global__ __launch_bounds__(TPB) void copy_kernel(int64_t n, const float* __restrict__ src,
                                                   int64_t inca, float* __restrict__ dst,
                                                   int64_t incb) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * TPB)
    dst[i * incb] = src[i * inca];
}

__global__ __launch_bounds__(TPB) void clamp_kernel(int64_t n, float alpha,
                                                    const float* __restrict__ src,
                                                    float* __restrict__ dst, int64_t stride) {
  // vsClamp(-alpha, alpha) as used by delta.Clamp (ntensors.pas:10077)
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * TPB) {
    float v = src[i * stride];
    v = v < -alpha ? -alpha : (v > alpha ? alpha : v);
    dst[i * stride] = v;
  }
}

}  // namespace

hipError_t launch_bias_activate(float* dst, int64_t F, int64_t bs, const float* bias,
                                int64_t batch, int act, hipStream_t s) {
  const int64_t total = batch * F * bs;
  if (total <= 0) return hipSuccess;
  const bool act_on = act != TNS_acLINEAR;
  if (bs % 4 == 0 && aligned16(dst)) {
    const int64_t tv = total / 4;
    if (act_on)
      hipLaunchKernelGGL((bias_act_kernel<4, true>), dim3(grid_for(tv)), dim3(TPB), 0, s, dst, F,
                         bs, bias, (int64_t)1, tv, act);
    else
      hipLaunchKernelGGL((bias_act_kernel<4, false>), dim3(grid_for(tv)), dim3(TPB), 0, s, dst,
                         F, bs, bias, (int64_t)1, tv, act);
  } else {
    if (act_on)
      hipLaunchKernelGGL((bias_act_kernel<1, true>), dim3(grid_for(total)), dim3(TPB), 0, s, dst,
                         F, bs, bias, (int64_t)1, total, act);
    else
      hipLaunchKernelGGL((bias_act_kernel<1, false>), dim3(grid_for(total)), dim3(TPB), 0, s,
                         dst, F, bs, bias, (int64_t)1, total, act);
  }
  return hipGetLastError();
}

hipError_t launch_forward_bias(float* dst, int64_t F, int64_t bs, const float* bias,
                               int64_t incb, int64_t batch, hipStream_t s) {
  const int64_t total = batch * F * bs;
  if (total <= 0) return hipSuccess;
  if (bs % 4 == 0 && aligned16(dst)) {
    const int64_t tv = total / 4;
    hipLaunchKernelGGL((bias_act_kernel<4, false>), dim3(grid_for(tv)), dim3(TPB), 0, s, dst, F,
                       bs, bias, incb, tv, 4);
  } else {
    hipLaunchKernelGGL((bias_act_kernel<1, false>), dim3(grid_for(total)), dim3(TPB), 0, s, dst,
                       F, bs, bias, incb, total, 4);
  }
  return hipGetLastError();
}

hipError_t launch_activate(float* x, int64_t n, int act, hipStream_t s) {
  if (n <= 0 || act == TNS_acLINEAR) return hipSuccess;
  if (n % 4 == 0 && aligned16(x)) {
    hipLaunchKernelGGL(act_kernel<4>, dim3(grid_for(n / 4)), dim3(TPB), 0, s, x, n / 4, act);
  } else {
    hipLaunchKernelGGL(act_kernel<1>, dim3(grid_for(n)), dim3(TPB), 0, s, x, n, act);
  }
  return hipGetLastError();
}

hipError_t launch_derive(const float* x, int64_t n, int act, float* delta, hipStream_t s) {
  if (n <= 0 || act == TNS_acLINEAR) return hipSuccess;
  hipLaunchKernelGGL(derive_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, x, n, act, delta);
  return hipGetLastError();
}

hipError_t launch_backward_bias(float* dst, int64_t nDst, const float* src, int64_t bs,
                                int64_t batch, int64_t incb, hipStream_t s) {
  if (nDst <= 0) return hipSuccess;
  hipLaunchKernelGGL(backward_bias_kernel, dim3((unsigned)nDst), dim3(TPB), 0, s, dst, nDst, src,
                     bs, batch, incb);
  return hipGetLastError();
}

hipError_t launch_axpy(int64_t n, float a, const float* x, int64_t incx, float* y, int64_t incy,
                       hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(axpy_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, n, a, x, incx, y, incy);
  return hipGetLastError();
}

hipError_t launch_scale(int64_t n, float a, float* x, int64_t stride, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, n, a, x, stride);
  return hipGetLastError();
}

hipError_t launch_fill(int64_t n, float* x, float v, int64_t stride, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, n, x, v, stride);
  return hipGetLastError();
}

hipError_t launch_copy(int64_t n, const float* src, int64_t inca, float* dst, int64_t incb,
                       hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(copy_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, n, src, inca, dst, incb);
  return hipGetLastError();
}

hipError_t launch_clamp(int64_t n, float alpha, const float* src, float* dst, int64_t stride,
                        hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(clamp_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, n, alpha, src, dst,
                     stride);
  return hipGetLastError();
}

}  // namespace tns
