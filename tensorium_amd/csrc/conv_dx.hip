// conv_dx.hip — the conv backward's state.delta for stride-1 layers, with the
// col matrix never written: TConvolutionalLayer.backward's
//   col_b := W^T . delta_b   (gemm TN, beta 0: nConvolutionLayer.pas:646-655)
//   state.delta_b += col2im(col_b)  (scol2im, ntensors.pas:11650-11763; 656-660)
// as one kernel.  scol2im adds, per image pixel (c, y, x), the col entries of
// its window taps in ascending (kr, kc) order to the pixel's existing value,
// skipping taps whose output position falls outside the oh x ow plane; each
// col entry (c*k^2 + kr*k + kc, orow, ocol) is an ascending-f fmaf chain from
// +0 over the filters.  Here a block owns a 64-channel x 64-pixel tile of one
// image's state.delta: for tap t = (kr, kc) it runs that chain on the f32
// MFMA (v_mfma_f32_32x32x2_f32: a k-ordered fmaf chain, bit for bit) with B
// gathered from delta at (y + P - kr*d, x + P - kc*d) (zero past the plane:
// fma(w, 0, acc) = acc for the +0-started chain's non-negative-zero values),
// then adds the finished chain to the pixel's running value — only for the
// taps scol2im does not skip — before the next tap's chain starts.  Same
// roundings, same order: bit-identical to TN GEMM + col2im, without the
// C*k^2*oh*ow col matrix round trip through HBM and the col2im pass.
//
// The weights are read as Wt[t][f][c] (a transposed copy made once per call,
// tns_api.cpp) so a tap's A tile rows are contiguous; k-tiles of 32 filters,
// two LDS stages, one barrier per k-tile; the chains of all taps run back to
// back through one pipeline (chunk q = t * ceil(F/32) + f-chunk).
#include <algorithm>

#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BM = 64, BN = 64, BK = 32, NT = 256;
constexpr int LD = 96;  // LDS row length: rows k and k+1 (lane halves) 32 banks apart
constexpr int STAGE = 2 * BK * LD;

struct DxArgs {
  const float* wt;     // [K2][F][C]
  const float* delta;  // [batch][F][oh][ow]
  float* im;           // [batch][C][H][W], accumulated into
  int C, F, H, W, oh, ow, ks, pad, dil;
  int tiles_c;
};

__global__ __launch_bounds__(NT) void conv_dx_col2im_kernel(DxArgs p) {
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lc = lane & 31, h = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;
  const int tc = blockIdx.x % p.tiles_c, tp = blockIdx.x / p.tiles_c;
  const int c0 = tc * BM, px0 = tp * BN;
  const int64_t img = blockIdx.y;
  const int HW = p.H * p.W, OHW = p.oh * p.ow;
  const float* __restrict__ dl = p.delta + img * (int64_t)p.F * OHW;
  float* __restrict__ im = p.im + img * (int64_t)p.C * HW;
  const int nkf = (p.F + BK - 1) / BK, K2 = p.ks * p.ks, nq = K2 * nkf;

  // ---- staging: A = Wt[t][f0 + f][c0 + 4*c4 .. +3] (two float4 per thread),
  // B = delta at this thread's pixel for filters f0 + fb + 4u (8 per thread)
  const int a_f = tid >> 4, a_c = 4 * (tid & 15);  // rows a_f and a_f + 16
  const bool a_ok = c0 + a_c < p.C;                // C % 4 == 0: a float4 is all in or out
  const int b_px = tid & 63, b_f = tid >> 6;       // filters b_f + 4u
  const int px = px0 + b_px;
  const int y = px < HW ? px / p.W : 0, x = px < HW ? px - (px / p.W) * p.W : 0;
  float4 ra[2];
  float rb[8];
  auto load = [&](int q) {
    const int t = q / nkf, f0 = (q - t * nkf) * BK;
    const int kr = t / p.ks, kc = t - kr * p.ks;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int f = f0 + a_f + 16 * u;
      ra[u] = (a_ok && f < p.F)
                  ? *reinterpret_cast<const float4*>(p.wt + ((int64_t)t * p.F + f) * p.C + c0 + a_c)
                  : float4{0.f, 0.f, 0.f, 0.f};
    }
    const int orow = y + p.pad - kr * p.dil, ocol = x + p.pad - kc * p.dil;
    const bool in = px < HW && (unsigned)orow < (unsigned)p.oh && (unsigned)ocol < (unsigned)p.ow;
    const int off = in ? orow * p.ow + ocol : 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int f = f0 + b_f + 4 * u;
      const float v = dl[(int64_t)(f < p.F ? f : 0) * OHW + off];
      rb[u] = (in && f < p.F) ? v : 0.0f;
    }
  };
  auto store = [&](float* st) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
      *reinterpret_cast<float4*>(st + (a_f + 16 * u) * LD + a_c) = ra[u];
#pragma unroll
    for (int u = 0; u < 8; ++u) st[BK * LD + (b_f + 4 * u) * LD + b_px] = rb[u];
  };

  // ---- the running state.delta values of this lane's outputs -------------
  // accumulator register e: channel c0 + 32*wm + (e&3) + 8*(e>>2) + 4h, pixel
  // px0 + 32*wn + lc
  const int opx = px0 + 32 * wn + lc;
  const int oy = opx < HW ? opx / p.W : 0, ox = opx < HW ? opx - (opx / p.W) * p.W : 0;
  float run[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int c = c0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
    run[e] = (c < p.C && opx < HW) ? im[(int64_t)c * HW + opx] : 0.0f;
  }
  floatx16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.0f;

  load(0);
  store(smem);
  __syncthreads();
  for (int q = 0; q < nq; ++q) {
    if (q + 1 < nq) load(q + 1);
    const float* st = smem + (q & 1) * STAGE;
    const float* ap = st + h * LD + 32 * wm + lc;
    const float* bp = st + BK * LD + h * LD + 32 * wn + lc;
#pragma unroll
    for (int s = 0; s < BK / 2; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[2 * s * LD], bp[2 * s * LD], acc, 0, 0, 0);
    if (q + 1 < nq) store(smem + ((q + 1) & 1) * STAGE);
    __syncthreads();
    const int t = q / nkf;
    if (q - t * nkf == nkf - 1) {  // tap t's chains are complete: scol2im's add
      const int kr = t / p.ks, kc = t - kr * p.ks;
      const int orow = oy + p.pad - kr * p.dil, ocol = ox + p.pad - kc * p.dil;
      const bool in = (unsigned)orow < (unsigned)p.oh && (unsigned)ocol < (unsigned)p.ow;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        run[e] = in ? run[e] + acc[e] : run[e];
        acc[e] = 0.0f;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int c = c0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
    if (c < p.C && opx < HW) im[(int64_t)c * HW + opx] = run[e];
  }
}

// Wt[s][f][c] = W[f][c*K2 + tap(s)], tap(s) = nibble s of `order` (K2 <= 16),
// or s itself for order = ~0 (any K2)
__global__ __launch_bounds__(256) void transpose_taps_kernel(const float* w, float* wt, int F,
                                                              int C, int K2,
                                                              unsigned long long order) {
  const int64_t n = (int64_t)F * C * K2;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t sl = i / ((int64_t)F * C);
    const int64_t r = i - sl * F * C;
    const int64_t f = r / C, c = r - f * C;
    const int64_t t = order == ~0ULL ? sl : (int64_t)((order >> (4 * sl)) & 15);
    wt[i] = w[f * C * K2 + c * K2 + t];
  }
}

}  // namespace

// Measured on the YOLOv3 layers at batch 8 (scripts/conv_bwd_layers.py
// --dx-fused 0/1, whole backward calls): ahead of TN GEMM + col2im on the 1x1
// layers with >= 104^2 pixels (208^2 0.279 -> 0.224 ms, 104^2 0.138 ->
// 0.128); behind on every 3x3 layer once the TN GEMM took 64x64 16x16-MFMA
// tiles (208^2 0.88 vs 0.99, 104^2 0.48 vs 0.53; before that it led there
// too) and on small planes (a block runs all k^2 * F chain steps of its tile
// in sequence, and small planes give too few tiles to fill the chip).
bool conv_dx_fused_applies(int64_t C, int64_t H, int64_t W, int64_t ks, int64_t stride, int64_t F,
                           int64_t oh, int64_t ow) {
  return ks == 1 && stride == 1 && C % 4 == 0 && H * W >= 8192 && C * H * W <= 0x7fffffffLL &&
         F * oh * ow <= 0x7fffffffLL && (int64_t)F * C <= 0x7fffffffLL;
}
bool conv_dx_fused_fits(int64_t C, int64_t H, int64_t W, int64_t stride, int64_t F, int64_t oh,
                        int64_t ow) {
  return stride == 1 && C % 4 == 0 && C * H * W <= 0x7fffffffLL && F * oh * ow <= 0x7fffffffLL &&
         (int64_t)F * C <= 0x7fffffffLL;
}

// wt[s][f][c] = W[f][c*K2 + tap(s)]: the weights tap-major (taps in the
// order given, nibble s = tap of slot s; ~0 = natural order), k-major per tap
hipError_t launch_transpose_taps(const float* w, float* wt, int64_t F, int64_t C, int64_t K2,
                                 hipStream_t s, unsigned long long order) {
  const int64_t n = F * C * K2;
  if (n <= 0) return hipSuccess;
  if (n > 0x7fffffffLL || (order != ~0ULL && K2 > 16)) return hipErrorInvalidValue;
  const int64_t tb = std::min<int64_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(transpose_taps_kernel, dim3((unsigned)tb), dim3(256), 0, s, w, wt, (int)F,
                     (int)C, (int)K2, order);
  return hipGetLastError();
}

hipError_t launch_conv_dx_col2im(const float* w, float* wt, const float* delta, float* im,
                                 int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F,
                                 int64_t ks, int64_t pad, int64_t dil, int64_t oh, int64_t ow,
                                 hipStream_t s) {
  if (batch <= 0 || C <= 0 || F <= 0) return hipSuccess;
  const int64_t K2 = ks * ks;
  if (hipError_t e = launch_transpose_taps(w, wt, F, C, K2, s); e != hipSuccess) return e;
  DxArgs a{};
  a.wt = wt; a.delta = delta; a.im = im;
  a.C = (int)C; a.F = (int)F; a.H = (int)H; a.W = (int)W; a.oh = (int)oh; a.ow = (int)ow;
  a.ks = (int)ks; a.pad = (int)pad; a.dil = (int)dil;
  a.tiles_c = (int)((C + BM - 1) / BM);
  const int64_t tiles = a.tiles_c * ((H * W + BN - 1) / BN);
  if (tiles > 0x7fffffffLL) return hipErrorInvalidValue;
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
    const int64_t nb = std::min<int64_t>(65535, batch - b0);
    DxArgs sub = a;
    sub.delta = delta + b0 * F * oh * ow;
    sub.im = im + b0 * C * H * W;
    hipLaunchKernelGGL(conv_dx_col2im_kernel, dim3((unsigned)tiles, (unsigned)nb), dim3(NT), 0, s,
                       sub);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace tns
