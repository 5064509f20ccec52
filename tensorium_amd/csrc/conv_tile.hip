// conv_tile.hip — implicit-GEMM convolution with output tiles sized to the
// YOLOv3 planes (TConvolutionalLayer.forward → Conv2D + forwardBias +
// activate after fuseBatchNorm: nConvolutionLayer.pas:457-569, ntensors.pas:
// 8252-8349; the im2col column order of sim2Col, 11415-11532).
//
// Same arithmetic as the ConvBIO path of sgemm_kernel.hpp (each output an
// ascending-k fma chain over k = (c, kr, kc) from +0 through the
// v_mfma_f32_16x16x4_f32 lane-quarter order, then bias add and activation,
// each rounded once), so bit-identical to sim2Col + the reference GEMM.  What
// differs is the geometry:
//
//   * N = batch*oH*oW = 1352*4^j on the 13*2^j YOLOv3 planes; a tile width of
//     176 (11 MFMA columns) puts 96-100 % of 256 CUs to work on one round of
//     blocks at every 3x3 layer (52^2: 2 x 123 blocks of 128 x 176; 26^2:
//     8 x 31 of 64 x 176; 13^2: 32 x 8 of 32 x 176), where the 64-multiple
//     tiles left a third of a round idle or shrank the tiles;
//   * every wave owns all BN columns (J = BN/16 accumulators per 16-row
//     strip, TM strips), so its B fragments are shared by TM*J MFMAs;
//   * B is gathered straight from the unpadded images (no zero-padded copy):
//     the lanes of a 16-lane quarter take 16 consecutive output pixels of one
//     k (coalesced), the k of each lane's slots stepping by 32 per tile with
//     (c, kr, kc) advanced incrementally (no k-table), the window bounds
//     checked per element and out-of-window taps read as 0 through the buffer
//     resource's range check;
//   * A (weights, k-contiguous) is transposed into a k-major image whose
//     columns are permuted so a lane's TM strip values are adjacent (one
//     ds_read_b64 for TM = 2) and XOR-swizzled by k/4 (conflict-free
//     transposing stores), as sgemm_nn_big.hip;
//   * the next tile's A loads and B gathers are issued at the top of a tile,
//     written to the other LDS stage mid-tile, one barrier per tile; the last
//     tile is peeled (no conditional staging in the loop body).
#include <type_traits>

#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;

template <int BM_, int BN_, int WM_, int SS_, bool PIN_ = true>
struct CGeo {
  static constexpr int BM = BM_, BN = BN_, WM = WM_;
  // PIN: step s+1's fragment reads issued before step s's MFMAs, held there
  // by scheduling fences (hipcc otherwise re-read the A strip and waited on
  // LDS every two MFMAs): 52^2 layers 0.131 -> 0.126 ms; the 4-wave 64 x 96
  // tile is 6-8 % slower with it
  static constexpr bool PIN = PIN_;
  static constexpr int SS = SS_;  // tile t+1 stored to LDS after MFMA step SS (0..7)
  static constexpr int NT = 64 * WM;
  static constexpr int WTM = BM / WM, TM = WTM / 16, J = BN / 16;
  // LDS row lengths: A rows k and k+1 are read by lane quarters 0 and 1 of one
  // half-wave (b32: 32 banks, b64: 64), B rows likewise (b32)
  static constexpr int LDA = BM + (TM == 2 ? 32 : 16);
  static constexpr int LDB = BN % 32 == 16 ? BN : BN + 16;
  static constexpr int A_TILE = BK * LDA, STAGE = BK * (LDA + LDB);
  static constexpr int AU = BM * BK / 4 / NT;  // float4 A units per thread
  static constexpr int KI = BK / 4 / WM;        // B k-slots per thread
  static_assert(TM == 1 || TM == 2, "strips read as one b32 / b64");
  static_assert(BN % 16 == 0 && AU >= 1 && BM * BK / 4 % NT == 0 && KI >= 1, "geometry");
};

// KS: kernel size (1 or 3), window offsets kr*d, kc*d
template <class G, int KS>
__global__ __launch_bounds__(G::NT) void conv_tile_kernel(GemmArgs p, int dil) {
  constexpr int BM = G::BM, BN = G::BN, NT = G::NT, WTM = G::WTM, TM = G::TM, J = G::J;
  constexpr int LDA = G::LDA, LDB = G::LDB, A_TILE = G::A_TILE, STAGE = G::STAGE;
  constexpr int AU = G::AU, KI = G::KI;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wm = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int tiles_m = (int)(p.M / BM);
  // XCD-contiguous order, column tiles outer (blocks of one XCD share the
  // images' rows in its L2); tile rows inner
  int tm, tn;
  {
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

  // ---- per-column state (the thread's J columns, fixed for the launch) ----
  unsigned vbase[J];  // byte offset of the window origin (may wrap: checked)
  int ir0[J], ic0[J];
  int64_t cofs[J];    // output element of (row 0, column)
#pragma unroll
  for (int j = 0; j < J; ++j) {
    int n = n0 + 16 * j + r16;
    n = n < N ? n : N - 1;  // past N: any valid pixel, never stored
    const int img = n / p.conv_ohw, pix = n - img * p.conv_ohw;
    const int orow = pix / p.conv_ow, ocol = pix - orow * p.conv_ow;
    ir0[j] = orow * p.conv_sY - p.conv_pH;
    ic0[j] = ocol * p.conv_sX - p.conv_pW;
    vbase[j] = 4u * (unsigned)(img * (int)p.strideB + ir0[j] * W + ic0[j]);
    cofs[j] = (int64_t)img * p.strideC + pix;
  }
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.B), 0, p.conv_bytes, 0x00020000);

  // ---- B k-slots: k = k0 + 4*(wm*KI + i) + q, advanced by BK per tile -----
  int kc_[KI], kr_[KI], cc_[KI];
#pragma unroll
  for (int i = 0; i < KI; ++i) {
    const int k = 4 * (wm * KI + i) + q;
    cc_[i] = k / (KS * KS);
    const int rem = k - cc_[i] * KS * KS;
    kr_[i] = rem / KS;
    kc_[i] = rem - kr_[i] * KS;
  }
  auto advance = [&]() {  // k += BK
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      if constexpr (KS == 1) {
        cc_[i] += BK;
      } else {
        constexpr int DC = BK / (KS * KS), DR = BK % (KS * KS);  // 3, 5 for KS = 3
        int rem = kr_[i] * KS + kc_[i] + DR;
        int c = cc_[i] + DC;
        if (rem >= KS * KS) { rem -= KS * KS; ++c; }
        cc_[i] = c;
        kr_[i] = rem >= 2 * KS ? 2 : (rem >= KS ? 1 : 0);
        kc_[i] = rem - kr_[i] * KS;
      }
    }
  };
  float rb[KI][J];
  auto gather_b = [&](int k0) {
    (void)k0;  // (K % BK == 0: every slot is inside K)
#pragma unroll
    for (int i = 0; i < KI; ++i) {
      const int y = kr_[i] * dil, z = kc_[i] * dil;
      const unsigned x = 4u * (unsigned)(cc_[i] * HW + y * W + z);
#pragma unroll
      for (int j = 0; j < J; ++j) {
#if defined(TNS_CT_NOGATHER)  // diagnostic builds only: timing without the gather
        rb[i][j] = (float)(x + j);
        continue;
#endif
#if defined(TNS_CT_NOCHECK)  // diagnostic: no window check (wrong values at the borders)
        const bool ok = true;
#else
        const bool ok = ((unsigned)(ir0[j] + y) < (unsigned)H) &
                        ((unsigned)(ic0[j] + z) < (unsigned)W);
#endif
        const unsigned off = ok ? vbase[j] + x : 0x80000000u;
        rb[i][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0));
      }
    }
  };
  auto store_b = [&](float* bs) {
#pragma unroll
    for (int i = 0; i < KI; ++i)
#pragma unroll
      for (int j = 0; j < J; ++j) bs[(4 * (wm * KI + i) + q) * LDB + 16 * j + r16] = rb[i][j];
  };

  // ---- A staging (weights [M][K]): unit u = k-quad kq of permuted column mm
  const float* a_src[AU];
  int a_dst[AU];
#pragma unroll
  for (int u = 0; u < AU; ++u) {
    const int idx = tid + NT * u;
    const int kq = idx & 7, mm = idx >> 3;
    const int m = (mm & ~(WTM - 1)) | ((mm % TM) << 4) | ((mm & (WTM - 1)) / TM);
    a_src[u] = p.A + (m0 + m) * p.lda + 4 * kq;
    a_dst[u] = (4 * kq) * LDA + (mm ^ (kq << 2));
  }
  float4 ra[AU];
  auto load_a = [&](int k0) {
#pragma unroll
    for (int u = 0; u < AU; ++u) {
#if defined(TNS_CT_NOA)  // diagnostic: no A loads
      ra[u] = make_float4(k0, u, 0, 1);
      continue;
#endif
      ra[u] = *reinterpret_cast<const float4*>(a_src[u] + k0);
    }
  };
  auto store_a = [&](float* as) {
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      as[a_dst[u]] = ra[u].x;
      as[a_dst[u] + LDA] = ra[u].y;
      as[a_dst[u] + 2 * LDA] = ra[u].z;
      as[a_dst[u] + 3 * LDA] = ra[u].w;
    }
  };

  // ---- MFMA: step s consumes k = 4s + q (lane quarter q) ------------------
  floatx4 acc[TM][J];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int a_frag = wm * WTM + TM * r16;
  auto frag = [&](const float* st, int s, float (&a)[TM], float (&b)[J]) {
    const int k = 4 * s + q;
    const float* ap = st + k * LDA + (a_frag ^ (s << 2));  // (k >> 2) & 7 == s
    if constexpr (TM == 2) {
      const float2 v = *reinterpret_cast<const float2*>(ap);
      a[0] = v.x; a[1] = v.y;
    } else {
      a[0] = ap[0];
    }
    const float* bp = st + A_TILE + k * LDB + r16;
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

  const int nt = K / BK;
  if (nt > 0) {
    load_a(0);
    gather_b(0);
    store_a(smem);
    store_b(smem + A_TILE);
    __syncthreads();
  }
  auto tile = [&](int t, auto MORE) {
    constexpr bool more = decltype(MORE)::value;
    const float* cur = smem + (t & 1) * STAGE;
    float* nxt = smem + ((t + 1) & 1) * STAGE;
    if constexpr (more) {
      advance();
      load_a((t + 1) * BK);
      gather_b((t + 1) * BK);
      __builtin_amdgcn_sched_barrier(0);  // keep the loads at the top of the tile
    }
    float a0[TM], b0[J], a1[TM], b1[J];
    frag(cur, 0, a0, b0);
#pragma unroll
    for (int s = 0; s < BK / 4; s += 2) {
      frag(cur, s + 1, a1, b1);
      if constexpr (G::PIN) __builtin_amdgcn_sched_barrier(0);
      mma(a0, b0);
      if (s + 2 < BK / 4) frag(cur, s + 2, a0, b0);
      if constexpr (G::PIN) __builtin_amdgcn_sched_barrier(0);
      if constexpr (more)
        if (s == G::SS) {  // tile t+1 into the other stage, after MFMA step SS
          __builtin_amdgcn_sched_barrier(0);
#if !defined(TNS_CT_NOSTORE)  // diagnostic builds only: timing without the LDS fill
          store_a(nxt);
          store_b(nxt + A_TILE);
#endif
        }
      mma(a1, b1);
    }
#if !defined(TNS_CT_NOBAR)  // diagnostic: no per-tile barrier (wrong results)
    if constexpr (more) __syncthreads();
#endif
  };
  for (int t = 0; t + 1 < nt; ++t) tile(t, std::true_type{});
  if (nt > 0) tile(nt - 1, std::false_type{});

  // ---- epilogue: forwardBias + activate, conv output [img][filter][pixel] --
  const bool fuse = p.epi == EPI_BIAS_ACT;
  const int act = p.act;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t row = m0 + wm * WTM + 16 * i + 4 * q + e;
      const float bias = fuse ? p.bias[row] : 0.0f;
      float* crow = p.C + row * p.ldc;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        if (n0 + 16 * j + r16 >= N) continue;
        float v = acc[i][j][e];
        if (fuse) v = act_apply_cheap(v + bias, act);
        crow[cofs[j]] = v;
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
    hipLaunchKernelGGL((conv_tile_kernel<G, 3>), dim3((unsigned)tiles), dim3(G::NT), 0, s, a, dil);
  else if (ks == 1)
    hipLaunchKernelGGL((conv_tile_kernel<G, 1>), dim3((unsigned)tiles), dim3(G::NT), 0, s, a, dil);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

struct TileInfo {
  int bm, bn;
  hipError_t (*fn)(const GemmArgs&, int, int, hipStream_t);
  const char* name;
};
#define TNS_CT(BMv, BNv, WMv, SSv, PINv)                                               \
  {BMv, BNv, launch_g<CGeo<BMv, BNv, WMv, SSv, PINv>>,                                 \
   "conv_tile<" #BMv "x" #BNv ",w" #WMv ",s" #SSv ">"}
const TileInfo kTiles[] = {
    TNS_CT(128, 176, 8, 4, true),   // 0: 52^2 / 104^2 3x3 layers (M = 256 / 128)
    TNS_CT(64, 96, 4, 6, false),    // 1: 208^2 3x3 layers (M = 64)
    TNS_CT(128, 96, 8, 4, true),    // 2
    TNS_CT(128, 176, 4, 4, true),   // 3: one wave per SIMD (measured slower: kept for the record)
};
#undef TNS_CT
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);
// the conv_tile4.hip forms picked by default
#ifndef TNS_CT4_NO_PF
// the 2-group 26^2 and the 13^2 forms as their loads-two-tiles-ahead twins
// (PF); the others keep one register set (PF: 128 x 176 spills, 64 x 96 and
// 64 x 32 lose blocks per CU)
constexpr int kT4Big = 3;
constexpr int kT4Small = 8;
constexpr int kT4OneByOne = 13;
// 64 x 176 x 32, wave columns 6 + 5 fragments, PF: stride 1 with the stores
// interleaved into group 0 (SI), stride 2 with the loads (IL) — warm clock,
// batch 8 (scripts/conv_fwd_layers.py, profiles/r05_conv_fwd_sweep.json):
// 26^2 0.1348 -> 0.1268 ms (PF alone 0.1296), 52^2 -> 26^2 stride 2 0.1431
// -> 0.1320 (PF alone 0.1426)
constexpr int kT4Uneven = 27;
constexpr int kT4UnevenS2 = 26;
constexpr int kT4OneByOnePF = 25;
constexpr int kT4Narrow = 21;    // 128 x 48 x 64 (every PF form level or slower on 13^2)
#else
constexpr int kT4OneByOnePF = 13;
constexpr int kT4UnevenS2 = 18;
constexpr int kT4Big = 3;    // 128 x 176 x 64, stores after group 1 and reads interleaved
constexpr int kT4Small = 8;  // 64 x 96 x 32, reads interleaved
constexpr int kT4OneByOne = 13;  // 64 x 32 x 32, 4 waves (1x1 layers)
constexpr int kT4Uneven = 18;    // 64 x 176 x 32, wave columns 6 + 5 fragments
constexpr int kT4Narrow = 21;    // 128 x 48 x 64, stores and reads interleaved
#endif

}  // namespace

// variants kNumTiles + v: conv_tile4.hip's form v (k-permuted b128 fragments)
int conv_tile_count() { return kNumTiles + conv_tile4_count(); }
bool conv_tile_is_ap(int v) { return v >= kNumTiles && conv_tile4_is_ap(v - kNumTiles); }
const char* conv_tile_name(int v) {
  return v >= 0 && v < kNumTiles ? kTiles[v].name : conv_tile4_name(v - kNumTiles);
}

// Measured per YOLOv3 layer shape (scripts/conv_tile_sweep.py, profiles/
// r02_conv_tile_sweep.json): the 8-wave 128 x 176 tile beats the
// sgemm_kernel.hpp shapes on the 3x3 layers with 128 / 256 filters (52^2
// 0.142 -> 0.131 ms, 104^2 0.146 -> 0.142 ms), the 64 x 96 tile on the 64-filter
// 3x3 layers by ~2 %; everywhere else (1x1, the 13^2 / 26^2 layers with 512 /
// 1024 filters over K = 2304 / 4608) the older shapes stay ahead; stride-2
// 128/256-filter layers are a tie.  -1: not this kernel.
//
// Round 3: the conv_tile4.hip forms (k-permuted ds_read_b128 fragments) of the
// same tiles, measured at a held clock (scripts/conv_fwd_layers.py --warm-ms,
// profiles/r03_conv_tile4.json): 128 x 176 x 64 with interleaved stores and
// reads 10-11 % ahead on the 128 / 256-filter 3x3 layers of either stride
// (52^2 0.127 -> 0.115 ms, 104^2 0.138 -> 0.123), 64 x 96 x 32 13 % ahead on
// the 64-filter ones (208^2 0.166 -> 0.145); the 512 / 1024-filter layers
// keep the multi-block sgemm_kernel.hpp tiles.
int conv_tile_pick(const GemmArgs& a, int ks) {
  if (a.K % BK || a.lda % 4 || (reinterpret_cast<uintptr_t>(a.A) & 15)) return -1;
  // 1x1 layers with 64..256 filters over >= 5408 pixels: the 64 x 32 form
  // (104^2 0.029 -> 0.022 ms, 52^2 0.023 -> 0.021, 26^2 0.023 -> 0.020); the
  // 512-filter 13^2 ones keep the sgemm_kernel.hpp tiles
  if (ks == 1) {
    if (a.M % 64 || a.M > 256 || a.N < 5408) return -1;
    // (round 5: the 26^2 planes on the PF twin, 0.0205 -> 0.0194 ms;
    // level on 52^2 / 104^2)
    return kNumTiles + (a.N < 16384 ? kT4OneByOnePF : kT4OneByOne);
  }
  if (ks != 3) return -1;
  if ((a.M == 128 || a.M == 256) && a.K % conv_tile4_bk(kT4Big) == 0) return kNumTiles + kT4Big;
  if ((a.M == 128 || a.M == 256) && a.conv_sY == 1) return 0;  // (stride 2: a tie)
  if (a.M == 64) return kNumTiles + kT4Small;
  // 512 filters (the 26^2 layers and the 52^2 -> 26^2 stride-2 one): 64 x 176
  // with wave columns of 6 + 5 fragments, 8 x 31 blocks (warm clock 0.137 ->
  // 0.128 ms, stride 2 0.151 -> 0.134)
  if (a.M == 512) return kNumTiles + (a.conv_sY == 1 ? kT4Uneven : kT4UnevenS2);
  // 1024 filters (13^2 planes, N = 1352): 8 x 29 blocks of 128 x 48 (warm clock
  // 0.149 -> 0.139 ms, the 26^2 -> 13^2 stride-2 layer 0.157 -> 0.140)
  if (a.M == 1024 && a.K % conv_tile4_bk(kT4Narrow) == 0) return kNumTiles + kT4Narrow;
  return -1;
}

hipError_t launch_conv_tile(int v, const GemmArgs& a, int ks, int dil, hipStream_t s) {
  if (v >= kNumTiles) return launch_conv_tile4(v - kNumTiles, a, ks, dil, s);
  if (v < 0) return hipErrorInvalidValue;
  return kTiles[v].fn(a, ks, dil, s);
}

}  // namespace tns
