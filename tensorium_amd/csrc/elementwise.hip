// elementwise.hip — wave64 elementwise kernels for gfx950 (HBM-bound).
//
//   forward_bias    vsAddB / TNNCuda.forwardBias (ntensors.pas:4066-4093,
//                   nncuda.pas:582): dst[(b*F+f)*bs + j] += bias[f*incb]
//   activate        activate_array (nactivation.pas:508-621)
//   bias_activate   the two above in one pass (conv forward, unfused GEMM path)
//   derive          gradient_array (nactivation.pas:624-717)
//   backward_bias   addSums (ntensors.pas:7729-7781) in the reference's
//                   order (vssum_avx2 per block, blocks in sequence)
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
// float4 form (n % 4 == 0, 16-byte aligned): same product per element
__global__ __launch_bounds__(TPB) void derive4_kernel(const float4* __restrict__ x, int64_t n4,
                                                      int act, float4* __restrict__ delta) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * TPB) {
    const float4 o = x[i];
    float4 d = delta[i];
    d.x = d.x * grad_apply(o.x, act);
    d.y = d.y * grad_apply(o.y, act);
    d.z = d.z * grad_apply(o.z, act);
    d.w = d.w * grad_apply(o.w, act);
    delta[i] = d;
  }
}

// addSums (ntensors.pas:7729-7781) in the reference's order: for output i,
// _sum := _sum + sumv(bs, block_j) over groups j ascending, then
// dst[i] := dst[i] + _sum; sumv = vssum_avx2 (3592-3620) on contiguous
// blocks: 8 lanes of sequential adds over the full 8-blocks, lane pairs
// (l, l+4) then ((s0+s1)+(s2+s3)), then the tail added in order.  One
// workgroup per output; 8 consecutive lanes own one block (lane l = the
// vssum lane), block totals meet in LDS and one thread adds them in j order.
constexpr int BB_SLOTS = TPB / 8;
constexpr int BB_CHUNK = 1024;
__global__ __launch_bounds__(TPB) void backward_bias_kernel(float* __restrict__ dst, int64_t nDst,
                                                            const float* __restrict__ src,
                                                            int64_t bs, int64_t groups,
                                                            int64_t incb) {
  __shared__ float tot[BB_CHUNK];
  const int64_t i = blockIdx.x;
  const int l = threadIdx.x & 7, q = threadIdx.x >> 3;
  const int64_t nb = bs >> 3;
  float sum = 0.0f;
  for (int64_t j0 = 0; j0 < groups; j0 += BB_CHUNK) {
    const int64_t jn = groups - j0 < BB_CHUNK ? groups - j0 : BB_CHUNK;
    for (int64_t jj = q; jj < ((jn + BB_SLOTS - 1) / BB_SLOTS) * BB_SLOTS; jj += BB_SLOTS) {
      const bool on = jj < jn;  // whole 8-lane groups are on or off
      const float* blk = src + ((j0 + (on ? jj : 0)) * nDst + i) * bs;
      float acc = 0.0f;
      if (on) {
        const float* p = blk + l;
        int64_t t = 0;
        for (; t + 8 <= nb; t += 8) {  // loads issued ahead of the dependent adds
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = p[8 * (t + u)];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc = acc + v[u];
        }
        for (; t < nb; ++t) acc = acc + p[8 * t];
      }
      const float s = acc + __shfl_down(acc, 4, 8);  // s_l = lane_l + lane_{l+4}
      const float h = s + __shfl_down(s, 1, 8);      // s0+s1 (l=0), s2+s3 (l=2)
      float r = h + __shfl_down(h, 2, 8);            // (s0+s1)+(s2+s3)
      if (on && l == 0) {
        for (int64_t u = nb * 8; u < bs; ++u) r = r + blk[u];
        tot[jj] = r;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int64_t jj = 0; jj < jn; ++jj) sum = sum + tot[jj];
    __syncthreads();
  }
  if (threadIdx.x == 0) dst[i * incb] = dst[i * incb] + sum;
}

// Same order for long blocks (conv layers at high resolution): 8 blocks at a
// time, staged through LDS in tiles of BB_T elements per block by all 256
// threads (coalesced, double-buffered), while wave 0's 64 lanes (8 per block,
// the vssum lanes) run the sequential chains out of LDS.  The chains are
// inherently serial; with one workgroup per output the tile loads' latency
// bounds the widest layers (32 x 173056 x 8: 0.35 ms, 0.5 TB/s).
constexpr int BB_T = 1024;
constexpr int BB_LD = BB_T + 8;  // row stride: the 8 blocks' lanes hit distinct banks
constexpr int BB_E = 8 * BB_T / TPB;
__global__ __launch_bounds__(TPB) void backward_bias_tiled_kernel(float* __restrict__ dst,
                                                                  int64_t nDst,
                                                                  const float* __restrict__ src,
                                                                  int64_t bs, int64_t groups,
                                                                  int64_t incb) {
  __shared__ float buf[2][8 * BB_LD];
  __shared__ float tot[8];
  const int64_t i = blockIdx.x;
  const int tid = threadIdx.x, jj = (tid & 63) >> 3, l = tid & 7;
  const bool chain = tid < 64;
  const int64_t nb8 = (bs >> 3) << 3;  // elements in full 8-blocks
  const int ntile = (int)((nb8 + BB_T - 1) / BB_T);
  float sum = 0.0f;
  for (int64_t j0 = 0; j0 < groups; j0 += 8) {
    const int jn = groups - j0 < 8 ? (int)(groups - j0) : 8;
    float r[BB_E];
    auto load = [&](int t) {
#pragma unroll
      for (int u = 0; u < BB_E; ++u) {
        const int e = tid + TPB * u, b = e / BB_T, x = e % BB_T;
        const int64_t k = (int64_t)t * BB_T + x;
        r[u] = (b < jn && k < nb8) ? src[((j0 + b) * nDst + i) * bs + k] : 0.0f;
      }
    };
    auto store = [&](float* d) {
#pragma unroll
      for (int u = 0; u < BB_E; ++u) {
        const int e = tid + TPB * u;
        d[(e / BB_T) * BB_LD + e % BB_T] = r[u];
      }
    };
    float acc = 0.0f;
    if (ntile > 0) {
      load(0);
      store(buf[0]);
      __syncthreads();
    }
    for (int t = 0; t < ntile; ++t) {
      if (t + 1 < ntile) load(t + 1);
      if (chain && jj < jn) {
        const float* row = buf[t & 1] + jj * BB_LD + l;
        const int64_t rem = nb8 - (int64_t)t * BB_T;
        const int cnt = (int)((rem < BB_T ? rem : BB_T) >> 3);
        int u = 0;
        for (; u + 16 <= cnt; u += 16) {
          float v[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] = row[8 * (u + q)];
#pragma unroll
          for (int q = 0; q < 16; ++q) acc = acc + v[q];
        }
        for (; u < cnt; ++u) acc = acc + row[8 * u];
      }
      if (t + 1 < ntile) store(buf[(t + 1) & 1]);
      __syncthreads();
    }
    {
      const float s = acc + __shfl_down(acc, 4, 8);
      const float h = s + __shfl_down(s, 1, 8);
      float q = h + __shfl_down(h, 2, 8);
      if (chain && l == 0 && jj < jn) {
        const float* blk = src + ((j0 + jj) * nDst + i) * bs;
        for (int64_t u = nb8; u < bs; ++u) q = q + blk[u];
        tot[jj] = q;
      }
    }
    __syncthreads();
    if (tid == 0)
      for (int b = 0; b < jn; ++b) sum = sum + tot[b];
    __syncthreads();
  }
  if (tid == 0) dst[i * incb] = dst[i * incb] + sum;
}

// TConnectedLayer.update / TConvolutionalLayer.update (nconnectedlayer.pas:
// 324-359, nConvolutionLayer.pas:673-705) in one pass: per weight
//   u = fma(ndb, w, dw)       weight_updates.axpy(-decay*batch, weights)
//   w = fma(lrb, u, w)        weights.axpy(lr/batch, weight_updates)
//   dw = momentum * u         weight_updates.Multiply(momentum)
// and per output the biases / scales axpy + momentum scale.  16 B of HBM per
// weight instead of the 32 B of the three separate passes.
template <int V>
__global__ __launch_bounds__(TPB) void sgd_update_kernel(int64_t nw, float* __restrict__ w,
                                                         float* __restrict__ dw, int64_t n,
                                                         float* __restrict__ b,
                                                         float* __restrict__ db,
                                                         float* __restrict__ sc,
                                                         float* __restrict__ dsc, float lrb,
                                                         float ndb, float mom) {
  const int64_t stride = (int64_t)gridDim.x * TPB;
  const int64_t t0 = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if constexpr (V == 4) {
    float4* w4 = reinterpret_cast<float4*>(w);
    float4* d4 = reinterpret_cast<float4*>(dw);
    for (int64_t i = t0; i < nw / 4; i += stride) {
      const float4 x = w4[i], g = d4[i];
      float4 u, y;
      u.x = fmaf(ndb, x.x, g.x); u.y = fmaf(ndb, x.y, g.y);
      u.z = fmaf(ndb, x.z, g.z); u.w = fmaf(ndb, x.w, g.w);
      y.x = fmaf(lrb, u.x, x.x); y.y = fmaf(lrb, u.y, x.y);
      y.z = fmaf(lrb, u.z, x.z); y.w = fmaf(lrb, u.w, x.w);
      w4[i] = y;
      d4[i] = make_float4(mom * u.x, mom * u.y, mom * u.z, mom * u.w);
    }
  }
  for (int64_t i = (V == 4 ? nw / 4 * 4 : 0) + t0; i < nw; i += stride) {
    const float x = w[i];
    const float u = fmaf(ndb, x, dw[i]);
    w[i] = fmaf(lrb, u, x);
    dw[i] = mom * u;
  }
  for (int64_t i = t0; i < n; i += stride) {
    b[i] = fmaf(lrb, db[i], b[i]);
    db[i] = mom * db[i];
    if (sc) {
      sc[i] = fmaf(lrb, dsc[i], sc[i]);
      dsc[i] = mom * dsc[i];
    }
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


// TNNCuda.addvv / subvv / mulvv / fmavv (nncuda.pas:120-123; kernels
// addv/subv/mulv/fmav): strided, one rounding per arithmetic operation
// (fmavv = src1*src2 rounded, then + src3 rounded — the CPU sfmavss form;
// the library is built without contraction)
template <int OP>
__global__ __launch_bounds__(TPB) void vv_kernel(int64_t n, const float* __restrict__ a,
                                                 int64_t inca, const float* __restrict__ b,
                                                 int64_t incb, const float* __restrict__ c,
                                                 int64_t incc, float* __restrict__ d,
                                                 int64_t incd) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * TPB) {
    const float x = a[i * inca], y = b[i * incb];
    float r;
    if (OP == 0) r = x + y;
    else if (OP == 1) r = x - y;
    else if (OP == 2) r = x * y;
    else r = x * y + c[i * incc];
    d[i * incd] = r;
  }
}

// TNNCuda.fmavss (nncuda.pas:137, kernel fmavss) / sfmavss (ntensors.pas:
// 3355-3368): dst = src*scalar + bias, mul then add
__global__ __launch_bounds__(TPB) void fmavss_kernel(int64_t n, const float* __restrict__ src,
                                                     float scalar, float bias,
                                                     float* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * TPB)
    dst[i] = src[i] * scalar + bias;
}

// TNNCuda.inverseSqrt (nncuda.pas:1563, kernel inverse_sqrt):
// dst = 1 / sqrt(max(src, eps)) (alpha is unused by the reference)
__global__ __launch_bounds__(TPB) void inverse_sqrt_kernel(int64_t n, const float* __restrict__ src,
                                                           float* __restrict__ dst,
                                                           int64_t stride) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * TPB) {
    const float v = src[i * stride];
    dst[i * stride] = 1.0f / sqrtf(v > 0.000001f ? v : 0.000001f);
  }
}

}  // namespace

hipError_t launch_vv(int op, int64_t n, const float* a, int64_t inca, const float* b, int64_t incb,
                     const float* c, int64_t incc, float* d, int64_t incd, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const unsigned g = grid_for(n);
  switch (op) {
    case 0: hipLaunchKernelGGL(vv_kernel<0>, dim3(g), dim3(TPB), 0, s, n, a, inca, b, incb, c, incc, d, incd); break;
    case 1: hipLaunchKernelGGL(vv_kernel<1>, dim3(g), dim3(TPB), 0, s, n, a, inca, b, incb, c, incc, d, incd); break;
    case 2: hipLaunchKernelGGL(vv_kernel<2>, dim3(g), dim3(TPB), 0, s, n, a, inca, b, incb, c, incc, d, incd); break;
    default: hipLaunchKernelGGL(vv_kernel<3>, dim3(g), dim3(TPB), 0, s, n, a, inca, b, incb, c, incc, d, incd); break;
  }
  return hipGetLastError();
}

hipError_t launch_fmavss(int64_t n, const float* src, float scalar, float bias, float* dst,
                         hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fmavss_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, n, src, scalar, bias, dst);
  return hipGetLastError();
}

hipError_t launch_inverse_sqrt(int64_t n, const float* src, float* dst, int64_t stride,
                               hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(inverse_sqrt_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, n, src, dst, stride);
  return hipGetLastError();
}

namespace {
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
  if (n % 4 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(delta)) & 15) == 0) {
    hipLaunchKernelGGL(derive4_kernel, dim3(grid_for(n / 4)), dim3(TPB), 0, s,
                       reinterpret_cast<const float4*>(x), n / 4, act,
                       reinterpret_cast<float4*>(delta));
    return hipGetLastError();
  }
  hipLaunchKernelGGL(derive_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, x, n, act, delta);
  return hipGetLastError();
}

hipError_t launch_backward_bias(float* dst, int64_t nDst, const float* src, int64_t bs,
                                int64_t batch, int64_t incb, hipStream_t s) {
  if (nDst <= 0) return hipSuccess;
  if (bs >= 2048)
    hipLaunchKernelGGL(backward_bias_tiled_kernel, dim3((unsigned)nDst), dim3(TPB), 0, s, dst,
                       nDst, src, bs, batch, incb);
  else
    hipLaunchKernelGGL(backward_bias_kernel, dim3((unsigned)nDst), dim3(TPB), 0, s, dst, nDst,
                       src, bs, batch, incb);
  return hipGetLastError();
}

hipError_t launch_sgd_update(int64_t nw, float* w, float* dw, int64_t n, float* b, float* db,
                             float* sc, float* dsc, float lrb, float ndb, float mom,
                             hipStream_t s) {
  if (nw <= 0 && n <= 0) return hipSuccess;
  const bool v4 = ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(dw)) & 15) == 0;
  const unsigned g = grid_for((v4 ? nw / 4 : nw) > n ? (v4 ? nw / 4 : nw) : n);
  if (v4)
    hipLaunchKernelGGL(sgd_update_kernel<4>, dim3(g), dim3(TPB), 0, s, nw, w, dw, n, b, db, sc,
                       dsc, lrb, ndb, mom);
  else
    hipLaunchKernelGGL(sgd_update_kernel<1>, dim3(g), dim3(TPB), 0, s, nw, w, dw, n, b, db, sc,
                       dsc, lrb, ndb, mom);
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

namespace {
__global__ __launch_bounds__(TPB) void add_in_order_kernel(float* __restrict__ C,
                                                           const float* __restrict__ part,
                                                           int64_t n, int64_t batch) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * TPB) {
    float acc = C[i];
    for (int64_t b = 0; b < batch; ++b) acc = acc + part[b * n + i];
    C[i] = acc;
  }
}

// float4 form (n % 4 == 0, 16-byte aligned): the same per-element order
// C + part[0] + part[1] + ...; up to 8 partials are loaded before the adds
// so their HBM reads are in flight together
__global__ __launch_bounds__(TPB) void add_in_order4_kernel(float4* __restrict__ C,
                                                            const float4* __restrict__ part,
                                                            int64_t n4, int64_t batch) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * TPB) {
    float4 acc = C[i];
    for (int64_t b0 = 0; b0 < batch; b0 += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (b0 + u < batch) v[u] = part[(b0 + u) * n4 + i];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (b0 + u < batch) {
          acc.x = acc.x + v[u].x;
          acc.y = acc.y + v[u].y;
          acc.z = acc.z + v[u].z;
          acc.w = acc.w + v[u].w;
        }
    }
    C[i] = acc;
  }
}
}  // namespace

hipError_t launch_add_in_order(float* C, const float* part, int64_t n, int64_t batch,
                               hipStream_t s) {
  if (n <= 0 || batch <= 0) return hipSuccess;
  if (n % 4 == 0 && aligned16(C) && aligned16(part)) {
    const int64_t n4 = n / 4;
    hipLaunchKernelGGL(add_in_order4_kernel, dim3(grid_for(n4)), dim3(TPB), 0, s,
                       reinterpret_cast<float4*>(C), reinterpret_cast<const float4*>(part), n4,
                       batch);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(add_in_order_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, C, part, n, batch);
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
