// conv_pp.hip — implicit-GEMM convolution on the ping-pong schedule
// (TConvolutionalLayer.forward → Conv2D + forwardBias + activate after
// fuseBatchNorm: nConvolutionLayer.pas:457-569, ntensors.pas:8252-8349; the
// im2col column order of sim2Col, 11415-11532).
//
// Same arithmetic as conv_tile.hip / the ConvBIO path of sgemm_kernel.hpp:
// each output an ascending-k fma chain over k = (c, kr, kc) from +0 through
// the v_mfma_f32_16x16x4_f32 lane-quarter order (lane quarter q = the q-th k
// of a step), then bias add and activation, each rounded once — so
// bit-identical to sim2Col + the reference GEMM.  What changes is the
// schedule (the one sgemm_nn_pp.hip runs for the plain GEMM):
//
//   * 8 waves in two groups of 4, one wave of each per SIMD; group g owns
//     block rows [g*BM/2, (g+1)*BM/2), its 4 waves split them WMG x WNG;
//   * each 32-deep k-tile in two phases separated by a barrier: in phase A
//     group 0 runs its MFMAs of tile t while group 1 writes k 0..15 of tile
//     t+1 into the other LDS stage; in phase B group 1 computes tile t while
//     group 0 writes k 16..31 of tile t+1 — every SIMD's matrix pipe has a
//     wave with MFMAs to issue while its partner stages;
//   * a staging job (the B gathers from the unpadded images with the window
//     bounds checked, out-of-window taps read as 0 through the buffer
//     resource's range check; the A float4 loads; the LDS writes) runs in
//     the group's memory phase;
//   * B is gathered for a fixed k per lane (the lanes of a quarter take 16
//     consecutive output pixels of one k: coalesced), (c, kr, kc) advanced
//     incrementally by 32 per tile; A (weights, k-contiguous) transposed into
//     a k-major image with permuted columns (a lane's TM strip values
//     adjacent) and the k-quad swizzle of the half-split staging.
#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
// Measured and not picked (profiles/): compiled only into the
// diagnostics build (TNS_DIAG=1 python -m tensorium_amd.build); the default
// library reports no forms of this family.
#ifdef TNS_DIAG_KERNELS

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32, NT = 512;

template <int BM_, int BN_, int WMG_, int WNG_>
struct PGeo {
  static constexpr int BM = BM_, BN = BN_, WMG = WMG_, WNG = WNG_;
  static constexpr int GM = BM / 2;                 // group rows
  static constexpr int WTM = GM / WMG, WTN = BN / WNG;
  static constexpr int TM = WTM / 16, J = WTN / 16;  // wave tile in 16x16 blocks
  static constexpr int JB = BN / 16;                 // B column strips (gather)
  static constexpr int LDA = BM + (TM == 2 ? 32 : 16);
  static constexpr int LDB = BN % 32 == 16 ? BN : BN + 16;
  static constexpr int A_TILE = BK * LDA, STAGE = BK * (LDA + LDB);
  static constexpr int AU = BM / 64;  // float4 A units per thread per half
  static_assert(WMG * WNG == 4, "4 waves per group");
  static_assert(TM == 1 || TM == 2, "strips read as one b32 / b64");
  static_assert(BN % (16 * WNG) == 0 && GM % (16 * WMG) == 0 && AU >= 1, "geometry");
};

template <class G, int KS>
__global__ __launch_bounds__(NT, 1) void conv_pp_kernel(GemmArgs p, int dil) {
  constexpr int BM = G::BM, BN = G::BN, WTM = G::WTM, WTN = G::WTN, TM = G::TM, J = G::J;
  constexpr int JB = G::JB, LDA = G::LDA, LDB = G::LDB, A_TILE = G::A_TILE, STAGE = G::STAGE;
  constexpr int AU = G::AU, WNG = G::WNG;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wid >> 2, wq = wid & 3, tg = tid & 255;
  const int wr = wq / WNG, wc = wq % WNG;
  const int r16 = lane & 15, q = lane >> 4;
  const int tiles_m = (int)(p.M / BM);
  int tm, tn;
  {  // XCD-contiguous order, column tiles outer, tile rows inner
    const int nb = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, qq = nb >> 3, rr = nb & 7;
    const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    tm = wg % tiles_m;
    tn = wg / tiles_m;
  }
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;
  const int N = (int)p.N, K = (int)p.K;
  const int H = p.conv_H, W = p.conv_W, HW = H * W;

  // ---- gather state: the JB column strips of the block, fixed -----------
  unsigned vbase[JB];
  int ir0[JB], ic0[JB];
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    int n = n0 + 16 * j + r16;
    n = n < N ? n : N - 1;  // past N: any valid pixel, never stored
    const int img = n / p.conv_ohw, pix = n - img * p.conv_ohw;
    const int orow = pix / p.conv_ow, ocol = pix - orow * p.conv_ow;
    ir0[j] = orow * p.conv_sY - p.conv_pH;
    ic0[j] = ocol * p.conv_sX - p.conv_pW;
    vbase[j] = 4u * (unsigned)(img * (int)p.strideB + ir0[j] * W + ic0[j]);
  }
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.B), 0, p.conv_bytes, 0x00020000);

  // this thread's k inside every tile: group 1 stages k 0..15, group 0 k
  // 16..31; wave wq of the group its quad, lane quarter q the k in it
  const int kt = 16 * (1 - g) + 4 * wq + q;
  int cc, kr, kc;
  {
    cc = kt / (KS * KS);
    const int rem = kt - cc * KS * KS;
    kr = rem / KS;
    kc = rem - kr * KS;
  }
  auto advance = [&]() {  // k += BK
    if constexpr (KS == 1) {
      cc += BK;
    } else {
      constexpr int DC = BK / (KS * KS), DR = BK % (KS * KS);  // 3, 5 for KS = 3
      int rem = kr * KS + kc + DR;
      int c = cc + DC;
      if (rem >= KS * KS) { rem -= KS * KS; ++c; }
      cc = c;
      kr = rem >= 2 * KS ? 2 : (rem >= KS ? 1 : 0);
      kc = rem - kr * KS;
    }
  };
  float rb[JB];
  auto gather_b = [&]() {
    const int y = kr * dil, z = kc * dil;
    const unsigned x = 4u * (unsigned)(cc * HW + y * W + z);
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const bool ok = ((unsigned)(ir0[j] + y) < (unsigned)H) & ((unsigned)(ic0[j] + z) < (unsigned)W);
      const unsigned off = ok ? vbase[j] + x : 0x80000000u;
      rb[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0));
    }
  };

  // ---- A (weights [M][K]): unit u = k-quad kq of the half, permuted col mm
  const float* a_src[AU];
  int a_dst[AU];
#pragma unroll
  for (int u = 0; u < AU; ++u) {
    const int idx = tg + 256 * u;
    const int kq = idx & 3, mm = idx >> 2;
    const int m = (mm & ~(WTM - 1)) | ((mm % TM) << 4) | ((mm & (WTM - 1)) / TM);
    a_src[u] = p.A + (m0 + m) * p.lda + 16 * (1 - g) + 4 * kq;
    a_dst[u] = (16 * (1 - g) + 4 * kq) * LDA + (mm ^ (kq << 3));
  }
  float4 ra[AU];
  auto issue = [&](int tile) {  // global side of this group's half of `tile`
#pragma unroll
    for (int u = 0; u < AU; ++u)
      ra[u] = *reinterpret_cast<const float4*>(a_src[u] + (int64_t)tile * BK);
    gather_b();
  };
  auto finish = [&](float* st) {  // LDS side (the memory phase)
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      st[a_dst[u]] = ra[u].x;
      st[a_dst[u] + LDA] = ra[u].y;
      st[a_dst[u] + 2 * LDA] = ra[u].z;
      st[a_dst[u] + 3 * LDA] = ra[u].w;
    }
    float* bs = st + A_TILE + kt * LDB + r16;
#pragma unroll
    for (int j = 0; j < JB; ++j) bs[16 * j] = rb[j];
  };

  // ---- MFMA: step s consumes k = 4s + q ----------------------------------
  floatx4 acc[TM][J];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int a_frag = g * G::GM + wr * WTM + TM * r16;
  const int b_frag = wc * WTN + r16;
  auto frag = [&](const float* st, int s, float (&a)[TM], float (&b)[J]) {
    const int k = 4 * s + q;
    const float* ap = st + k * LDA + (a_frag ^ ((s & 3) << 3));
    if constexpr (TM == 2) {
      const float2 v = *reinterpret_cast<const float2*>(ap);
      a[0] = v.x; a[1] = v.y;
    } else {
      a[0] = ap[0];
    }
    const float* bp = st + A_TILE + k * LDB + b_frag;
#pragma unroll
    for (int j = 0; j < J; ++j) b[j] = bp[16 * j];
  };
  auto mma = [&](const float (&a)[TM], const float (&b)[J]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < J; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
  };
  float a0[TM], b0[J];
  auto compute = [&](const float* cur) {
    float a1[TM], b1[J];
#pragma unroll
    for (int s = 0; s < BK / 4; s += 2) {
      frag(cur, s + 1, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a0, b0);
      if (s + 2 < BK / 4) frag(cur, s + 2, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b1);
    }
  };

  const int nt = K / BK;
  if (nt > 0) {
    issue(0);
    finish(smem);
    __syncthreads();
    if (g == 0) frag(smem, 0, a0, b0);
  }
  for (int t = 0; t < nt; ++t) {
    const float* cur = smem + (t & 1) * STAGE;
    float* nxt = smem + ((t + 1) & 1) * STAGE;
    const bool more = t + 1 < nt;
    // phase A: group 0 computes tile t, group 1 writes k 0..15 of tile t+1
    if (g == 0) {
      compute(cur);
    } else {
      if (more) {
        advance();
        issue(t + 1);
        finish(nxt);
      }
      frag(cur, 0, a0, b0);
    }
    __syncthreads();
    // phase B: group 1 computes tile t, group 0 writes k 16..31 of tile t+1
    if (g == 1) {
      compute(cur);
    } else if (more) {
      advance();
      issue(t + 1);
      finish(nxt);
      frag(nxt, 0, a0, b0);  // k 0..3 of tile t+1: written in phase A
    }
    if (more) __syncthreads();
  }

  // ---- epilogue: forwardBias + activate, conv output [img][filter][pixel] --
  const bool fuse = p.epi == EPI_BIAS_ACT;
  const int act = p.act;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int n = n0 + wc * WTN + 16 * j + r16;
    if (n >= N) continue;
    const int img = n / p.conv_ohw, pix = n - img * p.conv_ohw;
    const int64_t cofs = (int64_t)img * p.strideC + pix;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t row = m0 + g * G::GM + wr * WTM + 16 * i + 4 * q + e;
        float v = acc[i][j][e];
        if (fuse) v = act_apply_cheap(v + p.bias[row], act);
        p.C[row * p.ldc + cofs] = v;
      }
  }
}

template <class G>
hipError_t launch_g(const GemmArgs& a, int ks, int dil, hipStream_t s) {
  if (a.M % G::BM || a.K % BK || a.K <= 0 || a.lda % 4 ||
      (reinterpret_cast<uintptr_t>(a.A) & 15))
    return hipErrorInvalidValue;
  const int64_t tiles = (a.M / G::BM) * ((a.N + G::BN - 1) / G::BN);
  if (tiles > 0x7fffffff || a.N > 0x7fffffff || a.K > 0x7fffffff) return hipErrorInvalidValue;
  if (ks == 3)
    hipLaunchKernelGGL((conv_pp_kernel<G, 3>), dim3((unsigned)tiles), dim3(NT), 0, s, a, dil);
  else if (ks == 1)
    hipLaunchKernelGGL((conv_pp_kernel<G, 1>), dim3((unsigned)tiles), dim3(NT), 0, s, a, dil);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

struct TileInfo {
  int bm, bn;
  hipError_t (*fn)(const GemmArgs&, int, int, hipStream_t);
  const char* name;
};
#define TNS_CP(BMv, BNv, WMGv, WNGv) \
  {BMv, BNv, launch_g<PGeo<BMv, BNv, WMGv, WNGv>>, "conv_pp<" #BMv "x" #BNv ",g" #WMGv "x" #WNGv ">"}
const TileInfo kTiles[] = {
    TNS_CP(128, 176, 4, 1),  // 0: the plane-sized tile (52^2: 2 x 123 blocks)
    TNS_CP(64, 192, 2, 2),   // 1: 512-filter layers (26^2: 8 x 29 blocks)
    TNS_CP(64, 96, 2, 2),    // 2: 1024-filter layers (13^2: 16 x 15 blocks)
    TNS_CP(128, 96, 4, 1),   // 3
};
#undef TNS_CP
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

}  // namespace

int conv_pp_count() { return kNumTiles; }
const char* conv_pp_name(int v) { return v >= 0 && v < kNumTiles ? kTiles[v].name : ""; }

// not picked by default until measured (TNS_OPT_CONV_VARIANT = 200 + v)
int conv_pp_pick(const GemmArgs& a, int ks) {
  (void)a; (void)ks;
  return -1;
}

hipError_t launch_conv_pp(int v, const GemmArgs& a, int ks, int dil, hipStream_t s) {
  if (v < 0 || v >= kNumTiles) return hipErrorInvalidValue;
  return kTiles[v].fn(a, ks, dil, s);
}

#else
int conv_pp_count() { return 0; }
const char* conv_pp_name(int) { return ""; }
int conv_pp_pick(const GemmArgs&, int) { return -1; }
hipError_t launch_conv_pp(int, const GemmArgs&, int, int, hipStream_t) { return hipErrorInvalidValue; }
#endif  // TNS_DIAG_KERNELS

}  // namespace tns
