// conv_direct.hip — direct convolution for layers with a short k (C*kH*kW
// <= 32) and few filters: the first layer of a darknet net on a 3-channel
// image (YOLOv3 layer 0: 3 x 416^2, 3x3, 32 filters, K = 27).
//
// Same arithmetic as sim2Col + the reference GEMM + forwardBias + activate
// (TConvolutionalLayer.forward: nConvolutionLayer.pas:457-569; Conv2D
// ntensors.pas:8252-8349; sim2Col's column order 11415-11532; cblas_sgemm →
// s_nn over saxpy_avx2, 2061-2157 / 2231-2286): every output is the ascending
// k = (c, kr, kc) fmaf chain from +0 of w[f][k] * col[k][pixel], col being the
// image value in the window or 0 outside it (the zero the im2col matrix
// holds), then + bias[f] and the activation, each rounded once.  Bit-identical
// to the implicit-GEMM kernels (MFMA chains are the same fmaf sequence).
//
// Why not the GEMM: at K = 27 an output does 27 FMAs and the layer is bound by
// writing its 177 MB output (batch 8); the MFMA tiles spend their time in
// staging and the k-tile barrier (15 TF, 0.16 ms).  Here one thread owns NP
// pixels of one image and all F filters (F*NP accumulators), the weights are
// staged in LDS transposed (a tap's weights one broadcast ds_read_b128
// per 4 filters), the image taps are
// coalesced vector loads (consecutive pixels across lanes), and each filter's
// row is written by contiguous 256-byte wave stores: one HBM pass.
#include <type_traits>

#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
namespace {

constexpr int NT = 256;  // threads per block
#ifndef TNS_CD_NP
#define TNS_CD_NP 2
#endif
constexpr int NP = TNS_CD_NP;  // pixels per thread (NT apart)

struct DirectArgs {
  const float* in;    // [batch][C][H][W]
  const float* w;     // [F][K], K = C*KS*KS (sim2Col order: c, kr, kc)
  const float* bias;  // [F] or null (raw convolution)
  float* out;         // [batch][F][oh][ow]
  int H, W, oh, ow, stride, pad, dil, act, filters;
  int blocks_per_img;
};

template <int F, int C, int KS>
__global__ __launch_bounds__(NT) void conv_direct_kernel(DirectArgs p) {
  constexpr int K = C * KS * KS;
  const int img = blockIdx.x / p.blocks_per_img;
  const int blk = blockIdx.x - img * p.blocks_per_img;
  const int ohw = p.oh * p.ow;
  const float* __restrict__ in = p.in + (int64_t)img * C * p.H * p.W;
  const float* __restrict__ w = p.w;
  // the weights, filter rows padded to KP floats (16-byte aligned rows read
  // by wave-uniform ds_read_b128: broadcasts)
  constexpr int KP = (K + 3) & ~3;
  __shared__ __attribute__((aligned(16))) float ws[F * KP];
  for (int i = threadIdx.x; i < F * K; i += NT) {
    const int f = i / K;
    ws[f * KP + (i - f * K)] = w[i];
  }
  __syncthreads();
  int y0[NP], x0[NP];
  bool live[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int px = blk * NT * NP + j * NT + threadIdx.x;
    live[j] = px < ohw;
    const int pp = live[j] ? px : 0;
    const int y = pp / p.ow;
    y0[j] = y * p.stride - p.pad;
    x0[j] = (pp - y * p.ow) * p.stride - p.pad;
  }
  // every tap's image values first (K*NP loads in flight per thread) ...
  float v[K][NP];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int kr = 0; kr < KS; ++kr)
#pragma unroll
      for (int kc = 0; kc < KS; ++kc)
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          const int iy = y0[j] + kr * p.dil, ix = x0[j] + kc * p.dil;
          const bool ok = (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
          // (an out-of-window tap loads element 0 and selects 0: no masked
          // loads, whose exec masks would crowd the scalar registers)
          const float x = in[ok ? (c * p.H + iy) * p.W + ix : 0];
          v[(c * KS + kr) * KS + kc][j] = ok ? x : 0.0f;
        }
  // ... then filter by filter: the K weights of filter f are one LDS row,
  // its NP chains run over k, and its output row is stored at once — only NP
  // accumulators live
  float* __restrict__ out = p.out + (int64_t)img * F * ohw;
  auto filters = [&](auto ACT) {
    constexpr int act = decltype(ACT)::value;
#pragma unroll 2
    for (int f = 0; f < F; ++f) {
      float wf[KP];
#pragma unroll
      for (int k = 0; k < KP; k += 4) {
        const float4 q = *reinterpret_cast<const float4*>(&ws[f * KP + k]);
        wf[k] = q.x; wf[k + 1] = q.y; wf[k + 2] = q.z; wf[k + 3] = q.w;
      }
      float acc[NP];
#pragma unroll
      for (int j = 0; j < NP; ++j) acc[j] = 0.0f;
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int j = 0; j < NP; ++j) acc[j] = __builtin_fmaf(wf[k], v[k][j], acc[j]);
      const float b = act >= 0 ? p.bias[f] : 0.0f;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        if (!live[j]) continue;
        float r = acc[j];
        if constexpr (act >= 0) r = act_apply(r + b, act);  // forwardBias, then activate
        out[(int64_t)f * ohw + blk * NT * NP + j * NT + threadIdx.x] = r;
      }
    }
  };
  // (the activation switch hoisted: one instance per form)
  if (!p.bias) filters(std::integral_constant<int, -1>{});  // raw convolution
  else if (p.act == 0) filters(std::integral_constant<int, 0>{});
  else if (p.act == 1) filters(std::integral_constant<int, 1>{});
  else if (p.act == 6) filters(std::integral_constant<int, 6>{});
  else if (p.act == 8 || p.act == 9) filters(std::integral_constant<int, 9>{});
  else if (p.act == 13) filters(std::integral_constant<int, 13>{});
  else filters(std::integral_constant<int, 4>{});
}

}  // namespace

bool conv_direct_applies(int64_t C, int64_t ks, int64_t filters) {
  return C == 3 && ks == 3 && (filters == 16 || filters == 32);
}

hipError_t launch_conv_direct(const float* in, const float* w, const float* bias, float* out,
                              int64_t batch, int64_t C, int64_t H, int64_t W, int64_t filters,
                              int64_t ks, int64_t stride, int64_t pad, int64_t dil, int64_t oh,
                              int64_t ow, int act, hipStream_t s) {
  if (!conv_direct_applies(C, ks, filters) || batch <= 0 || oh <= 0 || ow <= 0)
    return hipErrorInvalidValue;
  // 32-bit pixel and image indexing within one image
  if (C * H * W > 0x7fffffffLL || filters * oh * ow > 0x7fffffffLL) return hipErrorInvalidValue;
  DirectArgs a{};
  a.in = in; a.w = w; a.bias = bias; a.out = out;
  a.H = (int)H; a.W = (int)W; a.oh = (int)oh; a.ow = (int)ow;
  a.stride = (int)stride; a.pad = (int)pad; a.dil = (int)dil; a.act = act;
  a.filters = (int)filters;
  a.blocks_per_img = (int)((oh * ow + NT * NP - 1) / (NT * NP));
  const int64_t grid = batch * a.blocks_per_img;
  if (grid > 0x7fffffffLL) return hipErrorInvalidValue;
  // (the weights are read as w[f*K + k] for every f < F: F == filters)
  if (filters == 16)
    hipLaunchKernelGGL((conv_direct_kernel<16, 3, 3>), dim3((unsigned)grid), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((conv_direct_kernel<32, 3, 3>), dim3((unsigned)grid), dim3(NT), 0, s, a);
  return hipGetLastError();
}

}  // namespace tns
