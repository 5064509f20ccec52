// sgemm_kernel.hpp — fp32 SGEMM on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the reference's GEMM backends for TTensor<Single>.gemm /
// gemmStridedBatched (cblas_sgemm, ntensors.pas:2231-2304; TNNCuda.gemm,
// nncuda.pas:624-725; cl_las TXgemm, cl_las.pas:483-640).
//
// Numerics (why NN/TN are bit-identical to the reference CPU path):
//   The reference computes every C element as an ascending-k FMA chain
//   starting from beta*C:  c = fma(alpha*A[i,k], B[k,j], c)   (saxpy_avx2
//   vfmadd231, s_nn/s_tn ntensors.pas:2007-2133).  gfx950's f32 MFMA is
//   bit-for-bit a k-ordered fmaf chain (D = fma(a_k1,b_k1, fma(a_k0,b_k0,C))).
//   Every kernel here feeds each accumulator k in ascending order (k-tiles
//   ascending, MFMA steps ascending, lane-half 0 = the lower k of a step),
//   pre-multiplies A by alpha once (the reference's A_PART) and starts the
//   accumulator at beta*C (the reference's mulvs pre-scale).  No split-K.
//   NT/TT use a different order in the reference (8-lane sdot / unfused
//   mul+add): the default dispatch sends them to sgemm_sdot.hip / sgemm_tt.hip
//   (bit-exact); through this kernel they agree within the componentwise
//   bound documented in DESIGN.md.
//
// Structure (one template, several tile shapes picked per problem):
//   block tile BM x BN, k-tile BK, WM x WN waves, each wave owning
//   (BM/WM) x (BN/WN) as a grid of 32x32 (or 16x16) MFMA accumulators.  Operands are
//   staged global -> registers (float4 where the layout allows) -> LDS in
//   k-major [k][m] / [k][n] images, double-buffered with one barrier per
//   k-tile; the next tile's global loads are issued before the current
//   tile's MFMAs and written to LDS after them.  The block index is remapped
//   so each of the 8 XCDs sweeps a contiguous, grouped region of C.
#pragma once
#include <type_traits>
#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
namespace sgemm_detail {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int GROUP_M = 8;

// LDS row length of a k-major operand image.  K-contiguous operands are
// transposed on the way in (scalar ds_writes); a row length ≡ 1 (mod 32)
// makes those writes conflict-free.  MN-contiguous operands are written with
// ds_write_b128 and keep the plain length.  With 16x16 MFMA fragments the two
// 16-lane halves of a ds_read_b32 group read consecutive k rows, so the rows
// are also shifted by 16 banks (≡ 16 or 17 mod 32).
template <bool KCONTIG, int BMN, int MF>
struct LdsLd {
  static constexpr int value = (KCONTIG ? BMN + 1 : BMN) + (MF == 16 ? 16 : 0);
};

// 16 zero bytes every out-of-range staging load reads instead of the operand.
__device__ __attribute__((aligned(16))) static float4 g_zero_page;
__device__ __forceinline__ const float* zero_page() {
  return reinterpret_cast<const float*>(&g_zero_page);
}

// Loads one BK x BMN operand tile (k, mn) into E registers per thread.
//   KCONTIG:  element (k, mn) at base[(mn0+mn)*ld + k0+k]   (A NoTrans / B Trans)
//   else   :  element (k, mn) at base[(k0+k)*ld + mn0+mn]   (A Trans / B NoTrans)
// Out-of-range elements read as 0.  Branch-free: an out-of-range load is
// redirected to the zero page.  VEC=4
// is only instantiated when the contiguous extent is a multiple of 4 (the
// host checks), so a float4 is either wholly inside or wholly outside.
template <bool KCONTIG, int VEC, int BK, int BMN, int NT, int MF>
struct TileIO {
  static constexpr int E = BK * BMN / NT;
  static_assert(E % VEC == 0, "tile not divisible");
  static constexpr int LD = LdsLd<KCONTIG, BMN, MF>::value;

  __device__ static __forceinline__ void load(float (&r)[E], const float* __restrict__ base,
                                              int64_t ld, int64_t mn0, int64_t k0, int64_t MN,
                                              int64_t K, int tid) {
#pragma unroll
    for (int it = 0; it < E / VEC; ++it) {
      const int idx = tid + NT * it;
      int64_t gk, gmn;
      if constexpr (KCONTIG) {
        gk = k0 + VEC * (idx % (BK / VEC));
        gmn = mn0 + idx / (BK / VEC);
      } else {
        gk = k0 + idx / (BMN / VEC);
        gmn = mn0 + VEC * (idx % (BMN / VEC));
      }
      const bool ok = (gmn < MN) & (gk < K);
      // out of range: read the zero page instead (no select on the loaded
      // value, so nothing forces an early wait on the load)
      const float* src = ok ? base + (KCONTIG ? gmn * ld + gk : gk * ld + gmn) : zero_page();
      if constexpr (VEC == 4) {
        const float4 v = *reinterpret_cast<const float4*>(src);
        r[4 * it + 0] = v.x;
        r[4 * it + 1] = v.y;
        r[4 * it + 2] = v.z;
        r[4 * it + 3] = v.w;
      } else {
        r[it] = *src;
      }
    }
  }

  __device__ static __forceinline__ void store(const float (&r)[E], float* __restrict__ xs,
                                               int tid) {
    if constexpr (VEC == 4) {
#pragma unroll
      for (int it = 0; it < E / 4; ++it) {
        const int idx = tid + NT * it;
        if constexpr (KCONTIG) {
          const int kq = idx % (BK / 4), mn = idx / (BK / 4);
#pragma unroll
          for (int c = 0; c < 4; ++c) xs[(4 * kq + c) * LD + mn] = r[4 * it + c];
        } else {
          const int mq = idx % (BMN / 4), k = idx / (BMN / 4);
          *reinterpret_cast<float4*>(xs + k * LD + 4 * mq) =
              make_float4(r[4 * it], r[4 * it + 1], r[4 * it + 2], r[4 * it + 3]);
        }
      }
    } else {
#pragma unroll
      for (int it = 0; it < E; ++it) {
        const int idx = tid + NT * it;
        if constexpr (KCONTIG) {
          xs[(idx % BK) * LD + idx / BK] = r[it];
        } else {
          xs[(idx / BMN) * LD + idx % BMN] = r[it];
        }
      }
    }
  }
};

// Implicit-GEMM B operand of a convolution: element (k, n) of the im2col
// matrix, k = (c, kr, kc), n = (image, orow, ocol), read straight from the
// images.  Each thread owns one column n for the whole launch (NT % BN == 0);
// the BN threads of a row group walk E consecutive k, so a wave's k-table
// entries are one contiguous run (vector dwordx4 loads, fetched one k-tile
// ahead).  Image loads are buffer loads whose out-of-range offsets return 0:
//   PADDED   the images were copied with their zero border materialised, and
//            the k >= K sentinel is out of range: one add per element;
//   checked  the window row/column are bounds-checked against H x W and a
//            failing element gets an out-of-range offset.
// Same values as sim2Col => bit-identical GEMM.
template <int BK, int BN, int NT, bool PADDED, int MF>
struct ConvBIO {
  static_assert(NT % BN == 0, "conv staging needs NT % BN == 0");
  static constexpr int E = BK * BN / NT;
  static constexpr int LD = LdsLd<false, BN, MF>::value;
  struct State {
    unsigned vbase;  // byte offset of this column's window origin
    int ir0, ic0;    // window origin (checked form)
    __amdgpu_buffer_rsrc_t rsrc;
  };
  __device__ static __forceinline__ State init(const GemmArgs& p, const float* im, int64_t n0,
                                               int tid) {
    int n = (int)(n0 + tid % BN);
    n = n < (int)p.N ? n : (int)p.N - 1;  // columns past N: any valid pixel (not stored)
    const int img = n / p.conv_ohw;
    const int pix = n - img * p.conv_ohw;
    const int orow = pix / p.conv_ow;
    const int ocol = pix - orow * p.conv_ow;
    State st;
    st.ir0 = orow * p.conv_sY - p.conv_pH;  // pH = pW = 0 for padded images
    st.ic0 = ocol * p.conv_sX - p.conv_pW;
    st.vbase = 4u * (unsigned)(img * (int)p.strideB + st.ir0 * p.conv_W + st.ic0);
    st.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(im), 0, p.conv_bytes,
                                                0x00020000);
    return st;
  }
  // entries k0 + kl*E + it, it < E (the table is padded past K with
  // sentinels).  Fetched with vector buffer loads (E/4 x dwordx4): scalar
  // loads would share lgkmcnt with the LDS traffic and force full drains.
  struct Tab {
    int x[E];
    int yz[E];  // checked form only: kr*dY | kc*dX << 16
  };
  static_assert(E % 4 == 0, "k-table fetched as dwordx4");
  __device__ static __forceinline__ void fetch(Tab& tab, const GemmArgs& p,
                                               __amdgpu_buffer_rsrc_t trs, int k0, int tid) {
    // wave-uniform when a wave's 64 lanes lie in one row group (BN >= 64)
    const int kl = tid / BN;
    const int off = 4 * (k0 + kl * E);
#pragma unroll
    for (int q = 0; q < E / 4; ++q) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(trs, off + 16 * q, 0, 0);
#pragma unroll
      for (int c = 0; c < 4; ++c) tab.x[4 * q + c] = (int)v[c];
      if constexpr (!PADDED) {
        const auto w = __builtin_amdgcn_raw_buffer_load_b128(trs, off + 16 * q, 4 * p.ktab_n, 0);
#pragma unroll
        for (int c = 0; c < 4; ++c) tab.yz[4 * q + c] = (int)w[c];
      }
    }
  }
  __device__ static __forceinline__ void load(float (&r)[E], const State& st, const Tab& tab,
                                              const GemmArgs& p) {
#pragma unroll
    for (int it = 0; it < E; ++it) {
      unsigned off = st.vbase + (unsigned)tab.x[it];
      if constexpr (!PADDED) {
        const int y = tab.yz[it] & 0xffff, z = (int)((unsigned)tab.yz[it] >> 16);
        const bool ok = ((unsigned)(st.ir0 + y) < (unsigned)p.conv_H) &
                        ((unsigned)(st.ic0 + z) < (unsigned)p.conv_W);
        off = ok ? off : 0x80000000u;
      }
      r[it] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(st.rsrc, off, 0, 0));
    }
  }
  __device__ static __forceinline__ void store(const float (&r)[E], float* __restrict__ xs,
                                               int tid) {
    const int kl = tid / BN, n = tid % BN;
#pragma unroll
    for (int it = 0; it < E; ++it) xs[(kl * E + it) * LD + n] = r[it];
  }
};

// XCD-aware, grouped mapping of a linear block id onto (tile_m, tile_n).
__device__ __forceinline__ void map_tile(int bid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int nb = tiles_m * tiles_n;
  // blocks b and b+8 are dispatched to the same XCD: give each XCD a
  // contiguous range of the logical order (bijective for any nb).
  const int xcd = bid & 7, q = nb >> 3, r = nb & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  // grouped raster: GROUP_M tile rows swept column by column.
  const int per_group = GROUP_M * tiles_n;
  const int group = wg / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_group = wg - group * per_group;
  tm = first_m + in_group % gsize;
  tn = in_group / gsize;
}

// DEPTH_: how many k-tiles ahead the global loads run (register stages).
// Small tiles spend few cycles per k-tile, so one tile of lead does not cover
// the global-load latency; they load two tiles ahead.
// MF: MFMA tile, 32 (v_mfma_f32_32x32x2_f32: 2 k per step, lane half h = k)
// or 16 (v_mfma_f32_16x16x4_f32: 4 k per step, lane quarter q = k).  Both are
// bit-exact ascending-k fmaf chains on gfx950 (profiles/r01_mfma_order_probe.txt).
// 16x16 tiles give four times as many independent accumulator chains per
// output area: finer work granularity for GEMMs with few output tiles.
template <int BM_, int BN_, int BK_, int WM_, int WN_, int MINW_, int DEPTH_ = 1, int MF_ = 32>
struct Shape {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_, MINW = MINW_;
  static constexpr int DEPTH = DEPTH_;
  static constexpr int MF = MF_;
  static_assert(MF == 32 || MF == 16, "MFMA tile 32x32x2 or 16x16x4");
  static_assert(DEPTH == 1 || DEPTH == 2, "prefetch depth 1 or 2");
  static constexpr int NT = 64 * WM * WN;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int TM = WTM / MF, TN = WTN / MF;
  static constexpr int KS = 64 / MF;        // k per MFMA step
  static constexpr int NE = MF * MF / 64;   // accumulator registers per lane
  static_assert(TM >= 1 && TN >= 1 && WTM % MF == 0 && WTN % MF == 0, "bad wave tile");
  static_assert(BK % (2 * KS) == 0, "k-tile = two halves of MFMA steps");
};

template <int MF>
struct Acc;
template <>
struct Acc<32> {
  typedef floatx16 type;
  __device__ static __forceinline__ type mma(float a, float b, type c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
};
template <>
struct Acc<16> {
  typedef floatx4 type;
  __device__ static __forceinline__ type mma(float a, float b, type c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};

// MFMA steps [S0, S1) of one k-tile: step s consumes k = KS*s + lane/MF
// (lane half for 32x32x2, lane quarter for 16x16x4) — ascending k per
// accumulator (the MFMA chains its k in lane-group order).
// (Issuing all of a half-tile's fragment reads ahead of its MFMAs measured
// slower on the YOLOv3 layers; the compiler's interleaving is kept.)
template <int MF, int TM, int TN, int LDA_S, int LDB_S, int S0, int S1>
__device__ __forceinline__ void mma_steps(typename Acc<MF>::type (&acc)[TM][TN], const float* ap,
                                          const float* bp) {
  constexpr int KS = 64 / MF;
  {
#pragma unroll
    for (int s = S0; s < S1; ++s) {
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = ap[KS * s * LDA_S + MF * i];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = bp[KS * s * LDB_S + MF * j];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = Acc<MF>::mma(a[i], b[j], acc[i][j]);
    }
  }
}

// CONV: 0 = plain GEMM, 1 = implicit conv on padded images, 2 = implicit conv
// with bounds checks
template <class S, bool TA, bool TB, int AV, int BV, int CONV = 0>
__global__ __launch_bounds__(S::NT, S::MINW) void sgemm_mfma_kernel(GemmArgs p) {
  constexpr int BM = S::BM, BN = S::BN, BK = S::BK, NT = S::NT;
  constexpr int TM = S::TM, TN = S::TN, WTM = S::WTM, WTN = S::WTN;
  constexpr int MF = S::MF, KS = S::KS, NE = S::NE;
  constexpr bool AKC = !TA;  // A is k-contiguous in memory
  constexpr bool BKC = TB;   // B is k-contiguous in memory
  using AIO = TileIO<AKC, AV, BK, BM, NT, S::MF>;
  using CIO = ConvBIO<BK, BN, NT, CONV == 1, S::MF>;
  using BIO = std::conditional_t<CONV != 0, CIO, TileIO<BKC, BV, BK, BN, NT, S::MF>>;
  constexpr int LDA_S = AIO::LD, LDB_S = BIO::LD;
  constexpr int A_TILE = BK * LDA_S;
  constexpr int B_TILE = BK * LDB_S;
  constexpr int STAGE = A_TILE + B_TILE;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  const int tid = threadIdx.x;
#ifdef TNS_GEMM_STAMPS
  // diagnostic build only: block start time and placement (scripts/gemm_timeline.py)
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
#endif
  const int lane = tid & 63;
  const int lc = lane % MF;  // accumulator column / operand row of this lane
  const int h = lane / MF;   // k within an MFMA step; 4h = first output row
  const int wid = tid >> 6;
  const int wm = wid / S::WN, wn = wid % S::WN;

  const int tiles_m = (int)((p.M + BM - 1) / BM);
  const int tiles_n = (int)((p.N + BN - 1) / BN);
  int tm_, tn_;
  map_tile(blockIdx.x, tiles_m, tiles_n, tm_, tn_);
  const int64_t m0 = (int64_t)tm_ * BM, n0 = (int64_t)tn_ * BN;
  const int64_t bz = blockIdx.y;

  // (conv: batch folded into N, launched with one z-slice)
  const float* __restrict__ A = p.A + bz * p.strideA;
  const float* __restrict__ B = CONV ? p.B : p.B + bz * p.strideB;
  float* __restrict__ C = CONV ? p.C : p.C + bz * p.strideC;
  const int64_t M = p.M, N = p.N, K = p.K;
  // element (row, col) of C; conv columns are (image, pixel)
  auto c_at = [&](int64_t row, int64_t col) -> int64_t {
    if constexpr (CONV) {
      const int img = (int)col / p.conv_ohw;
      return (int64_t)img * p.strideC + row * p.ldc + ((int)col - img * p.conv_ohw);
    } else {
      return row * p.ldc + col;
    }
  };

  // ---- accumulator init: 0, C, or beta*C (reference mulvs pre-scale) -----
  // accumulator register e of tile (i, j) holds C[row_base + i*MF + erow(e)]
  // [col_base + j*MF]; erow(e) = (e & 3) + 8*(e >> 2) (e < 4 for 16x16)
  typename Acc<MF>::type acc[TM][TN];
  const int64_t row_base = m0 + wm * WTM + 4 * h;
  const int64_t col_base = n0 + wn * WTN + lc;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[i][j][e] = 0.0f;
  if (!CONV && p.beta_mode != BETA_ZERO) {  // (conv output is write-only)
    const bool scale = p.beta_mode == BETA_SCALE;
    const float beta = p.beta;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const int64_t row = row_base + i * MF + (e & 3) + 8 * (e >> 2);
          const int64_t col = col_base + j * MF;
          const bool ok = row < M && col < N;
          float v = C[ok ? c_at(row, col) : 0];
          v = scale ? beta * v : v;
          acc[i][j][e] = ok ? v : 0.0f;
        }
  }

  const int nt = (int)((K + BK - 1) / BK);
  const bool scale_a = p.alpha != 1.0f;
  const float alpha = p.alpha;
  float ra[AIO::E], rb[BIO::E];
  const int a_off = h * LDA_S + wm * WTM + lc;
  const int b_off = h * LDB_S + wn * WTN + lc;
  [[maybe_unused]] typename CIO::State cst;
  // k-table entries of two consecutive tiles (ping-pong by tile parity):
  // the next tile's are fetched BEFORE this tile's gathers are issued, so
  // waiting for them never drains this tile's loads
  [[maybe_unused]] typename CIO::Tab tabs[2];
  [[maybe_unused]] __amdgpu_buffer_rsrc_t trs;
  if constexpr (CONV) {
    cst = CIO::init(p, B, n0, tid);
    trs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p.ktab), 0, 8 * p.ktab_n,
                                            0x00020000);
    CIO::fetch(tabs[0], p, trs, 0, tid);
  }
  auto load_b = [&](float (&r)[BIO::E], int64_t k0, auto TP) {  // TP: tile parity
    if constexpr (CONV) {
      constexpr int tp = decltype(TP)::value;
      CIO::fetch(tabs[tp ^ 1], p, trs, (int)k0 + BK, tid);  // next tile's entries
      CIO::load(r, cst, tabs[tp], p);
    } else {
      BIO::load(r, B, p.ldb, n0, k0, N, K, tid);
    }
  };

  // k-tile pipeline: tile t is multiplied out of LDS buffer t&1 while tile
  // t+1 is written into the other buffer (from registers loaded DEPTH tiles
  // earlier) and tile t+DEPTH is loaded into registers.  One barrier per tile.
  // Loads past the last tile read the zero page; stores past it land in a
  // buffer that is never read again.
  auto scale = [&](float (&r)[AIO::E]) {
    if (scale_a) {
#pragma unroll
      for (int i = 0; i < AIO::E; ++i) r[i] = alpha * r[i];  // A_PART = ALPHA*A[kk]
    }
  };
  auto step = [&](float (&lra)[AIO::E], float (&lrb)[BIO::E], float (&sra)[AIO::E],
                  float (&srb)[BIO::E], int t, auto PAR) {
    constexpr int par = decltype(PAR)::value;  // == t & 1
    const float* as = smem + par * STAGE;
    float* nxt = smem + (par ^ 1) * STAGE;
    // unconditional: past the last tile every lane reads the zero page (a
    // branch here would merge the wait counters and force an early wait)
    const int64_t kl = (int64_t)(t + S::DEPTH) * BK;
    AIO::load(lra, A, p.lda, m0, kl, M, K, tid);
    load_b(lrb, kl, std::integral_constant<int, (par + S::DEPTH) & 1>{});
    constexpr int SP = BK / (2 * KS);  // half of the k-tile's MFMA steps
    mma_steps<MF, TM, TN, LDA_S, LDB_S, 0, SP>(acc, as + a_off, as + A_TILE + b_off);
    scale(sra);
    AIO::store(sra, nxt, tid);
    BIO::store(srb, nxt + A_TILE, tid);
    mma_steps<MF, TM, TN, LDA_S, LDB_S, SP, 2 * SP>(acc, as + a_off, as + A_TILE + b_off);
    __syncthreads();
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;

  if (nt > 0) {
    AIO::load(ra, A, p.lda, m0, 0, M, K, tid);
    load_b(rb, 0, std::integral_constant<int, 0>{});
    scale(ra);
    AIO::store(ra, smem, tid);
    BIO::store(rb, smem + A_TILE, tid);
    if constexpr (S::DEPTH == 1) {
      __syncthreads();
      // registers are reloaded each tile and stored in the same tile.  Pairs
      // of tiles, then the odd last one outside the loop (an exit inside the
      // body would make the compiler copy the accumulators every iteration)
      int t = 0;
      for (; t + 1 < nt; t += 2) {
        step(ra, rb, ra, rb, t, P0{});
        step(ra, rb, ra, rb, t + 1, P1{});
      }
      if (t < nt) step(ra, rb, ra, rb, t, P0{});
    } else {
      float ra2[AIO::E], rb2[BIO::E];
      AIO::load(ra2, A, p.lda, m0, BK, M, K, tid);
      load_b(rb2, BK, std::integral_constant<int, 1>{});
      __syncthreads();
      // (ra2, rb2) hold tile t+1 at even t; (ra, rb) at odd t
      int t = 0;
      for (; t + 1 < nt; t += 2) {
        step(ra, rb, ra2, rb2, t, P0{});
        step(ra2, rb2, ra, rb, t + 1, P1{});
      }
      if (t < nt) step(ra, rb, ra2, rb2, t, P0{});
    }
  }

  // ---- epilogue ----------------------------------------------------------
#ifdef TNS_GEMM_STAMPS
  if (tid == 0 && p.stamps != nullptr && blockIdx.x < (1u << 16) && blockIdx.y == 0) {
    const unsigned long long t_end = __builtin_amdgcn_s_memtime();
    unsigned* st = p.stamps + 8 * blockIdx.x;
    st[0] = (unsigned)t_start;
    st[1] = (unsigned)(t_start >> 32);
    st[2] = (unsigned)t_end;
    st[3] = (unsigned)(t_end >> 32);
    st[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    st[5] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  }
#endif
  const bool fuse = p.epi == EPI_BIAS_ACT, add = p.epi == EPI_ADD;
  const int act = p.act;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int64_t row = row_base + i * MF + (e & 3) + 8 * (e >> 2);
      if (row >= M) continue;
      const float bias = fuse ? p.bias[row] : 0.0f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int64_t col = col_base + j * MF;
        if (col >= N) continue;
        float v = acc[i][j][e];
        // forwardBias then activate (logistic/tanh: a separate pass, host side)
        if (fuse) v = act_apply_cheap(v + bias, act);
        if (add) v = C[c_at(row, col)] + v;
        C[c_at(row, col)] = v;
      }
    }
}
template <class S, bool TA, bool TB, int AV, int BV, int CONV = 0>
hipError_t launch_variant(const GemmArgs& a, hipStream_t s) {
  const int64_t tiles = ((a.M + S::BM - 1) / S::BM) * ((a.N + S::BN - 1) / S::BN);
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  for (int64_t b0 = 0; b0 < a.batch; b0 += 65535) {
    GemmArgs sub = a;
    const int64_t nb = a.batch - b0 < 65535 ? a.batch - b0 : 65535;
    sub.A = a.A + b0 * a.strideA;
    sub.B = a.B + b0 * a.strideB;
    sub.C = a.C + b0 * a.strideC;
    sub.batch = nb;
    hipLaunchKernelGGL((sgemm_mfma_kernel<S, TA, TB, AV, BV, CONV>), dim3((unsigned)tiles, (unsigned)nb),
                       dim3(S::NT), 0, s, sub);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// all transposes x all vector widths
template <class S>
hipError_t launch_full(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
#define TNS_VEC(TA, TB)                                               \
  do {                                                                \
    if (av && bv) return launch_variant<S, TA, TB, 4, 4>(a, s);       \
    if (av) return launch_variant<S, TA, TB, 4, 1>(a, s);             \
    if (bv) return launch_variant<S, TA, TB, 1, 4>(a, s);             \
    return launch_variant<S, TA, TB, 1, 1>(a, s);                     \
  } while (0)
  if (!ta && !tb) TNS_VEC(false, false);
  if (!ta && tb) TNS_VEC(false, true);
  if (ta && !tb) TNS_VEC(true, false);
  TNS_VEC(true, true);
#undef TNS_VEC
}

// all transposes, float4 operands only (large-GEMM production shape)
template <class S>
hipError_t launch_trans4(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  if (!av || !bv) return hipErrorInvalidValue;
  if (!ta && !tb) return launch_variant<S, false, false, 4, 4>(a, s);
  if (!ta && tb) return launch_variant<S, false, true, 4, 4>(a, s);
  if (ta && !tb) return launch_variant<S, true, false, 4, 4>(a, s);
  return launch_variant<S, true, true, 4, 4>(a, s);
}

// implicit-GEMM convolution: NN, A (weights) float4 or scalar, B from the
// images (a.conv: 1 padded, 2 checked)
template <class S>
hipError_t launch_conv(const GemmArgs& a, bool av, hipStream_t s) {
  if (a.conv == 1) {
    if (av) return launch_variant<S, false, false, 4, 1, 1>(a, s);
    return launch_variant<S, false, false, 1, 1, 1>(a, s);
  }
  if (av) return launch_variant<S, false, false, 4, 1, 2>(a, s);
  return launch_variant<S, false, false, 1, 1, 2>(a, s);
}

// experimental tile shapes: NN with float4 operands only
template <class S>
hipError_t launch_nn4(const GemmArgs& a, bool ta, bool tb, bool av, bool bv, hipStream_t s) {
  if (ta || tb || !av || !bv) return hipErrorInvalidValue;
  return launch_variant<S, false, false, 4, 4>(a, s);
}

//                 BM   BN  BK WM WN MINW
using S128x128 = Shape<128, 128, 32, 2, 2, 2>;
using S128x64 = Shape<128, 64, 32, 2, 2, 2, 2>;
using S64x64 = Shape<64, 64, 32, 2, 2, 2, 2>;
using S64x128 = Shape<64, 128, 32, 2, 2, 2, 2>;
using S64x256 = Shape<64, 256, 32, 1, 4, 2>;
using S32x256 = Shape<32, 256, 32, 1, 4, 2>;
using S256x256 = Shape<256, 256, 32, 2, 2, 1>;
using S256x256k16 = Shape<256, 256, 16, 2, 2, 1>;
using S256x128 = Shape<256, 128, 32, 2, 2, 1>;
using S128x256 = Shape<128, 256, 32, 2, 2, 1>;
using S256x256w8 = Shape<256, 256, 32, 2, 4, 2>;
using S256x128k16 = Shape<256, 128, 16, 2, 2, 2>;
// 16x16x4 MFMA tiles                     BM   BN  BK WM WN MINW DEPTH MF
using S64x64m16 = Shape<64, 64, 32, 2, 2, 2, 2, 16>;
using S32x32m16 = Shape<32, 32, 32, 2, 2, 2, 2, 16>;
using S64x32m16 = Shape<64, 32, 32, 2, 2, 2, 2, 16>;
using S32x64m16 = Shape<32, 64, 32, 2, 2, 2, 2, 16>;
using S128x128m16 = Shape<128, 128, 32, 2, 2, 2, 1, 16>;
using S256x256w8m16 = Shape<256, 256, 32, 2, 4, 2, 1, 16>;
// conv tile experiments: 8-wave blocks, prefetch depth 1
using S128x64w8 = Shape<128, 64, 32, 4, 2, 2, 2>;
using S64x128w8 = Shape<64, 128, 32, 2, 4, 2, 2>;
using S128x128w8 = Shape<128, 128, 32, 4, 2, 2, 1>;
using S64x64d1 = Shape<64, 64, 32, 2, 2, 2, 1>;
using S64x64w8m16 = Shape<64, 64, 32, 2, 4, 2, 2, 16>;


}  // namespace sgemm_detail

// one launcher per shape, defined in the sgemm_*.hip translation units
typedef hipError_t (*ShapeLauncher)(const GemmArgs&, bool, bool, bool, bool, hipStream_t);
#define TNS_SHAPES(X)                                    \
  X(128x128, "128x128x32_w2x2", 128, 128, launch_full)   \
  X(128x64, "128x64x32_w2x2", 128, 64, launch_full)      \
  X(64x128, "64x128x32_w2x2", 64, 128, launch_full)      \
  X(64x256, "64x256x32_w1x4", 64, 256, launch_full)      \
  X(32x256, "32x256x32_w1x4", 32, 256, launch_full)      \
  X(256x256w8, "256x256x32_w2x4", 256, 256, launch_trans4) \
  X(64x64, "64x64x32_w2x2", 64, 64, launch_full)          \
  X(256x256, "256x256x32_w2x2", 256, 256, launch_nn4)    \
  X(256x256k16, "256x256x16_w2x2", 256, 256, launch_nn4) \
  X(256x128, "256x128x32_w2x2", 256, 128, launch_nn4)    \
  X(128x256, "128x256x32_w2x2", 128, 256, launch_nn4)    \
  X(256x128k16, "256x128x16_w2x2", 256, 128, launch_nn4) \
  X(64x64m16, "64x64x32_w2x2_m16", 64, 64, launch_full)  \
  X(32x32m16, "32x32x32_w2x2_m16", 32, 32, launch_full)  \
  X(64x32m16, "64x32x32_w2x2_m16", 64, 32, launch_nn4)   \
  X(32x64m16, "32x64x32_w2x2_m16", 32, 64, launch_nn4)   \
  X(128x128m16, "128x128x32_w2x2_m16", 128, 128, launch_nn4) \
  X(256x256w8m16, "256x256x32_w2x4_m16", 256, 256, launch_trans4) \
  X(128x64w8, "128x64x32_w4x2", 128, 64, launch_nn4)     \
  X(64x128w8, "64x128x32_w2x4", 64, 128, launch_nn4)     \
  X(128x128w8, "128x128x32_w4x2", 128, 128, launch_nn4)  \
  X(64x64d1, "64x64x32_w2x2_d1", 64, 64, launch_nn4)     \
  X(64x64w8m16, "64x64x32_w2x4_m16", 64, 64, launch_nn4)

#define TNS_DECL(ID, NAME, BMv, BNv, KIND) \
  hipError_t launch_shape_##ID(const GemmArgs&, bool, bool, bool, bool, hipStream_t);
TNS_SHAPES(TNS_DECL)
#undef TNS_DECL

// implicit-GEMM conv launchers (the shapes the YOLOv3 sweep keeps)
hipError_t launch_conv_128x64(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_64x128(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_32x256(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_64x64(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_64x64m16(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_32x32m16(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_64x32m16(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_32x64m16(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_128x64w8(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_64x128w8(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_128x128w8(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_64x64d1(const GemmArgs&, bool, hipStream_t);
hipError_t launch_conv_64x64w8m16(const GemmArgs&, bool, hipStream_t);

}  // namespace tns
