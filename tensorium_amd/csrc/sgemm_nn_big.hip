// sgemm_nn_big.hip — large aligned gemm(NoTrans, NoTrans) on fp32 MFMA.
//
// The production kernel for the headline product (BASELINE config 2, M = N =
// K = 4096) and any NN GEMM whose M and N are multiples of 256 and K of 32,
// with 16-byte aligned rows.  Same arithmetic as sgemm_kernel.hpp (the
// reference's cblas_sgemm → s_nn over saxpy_avx2, ntensors.pas:2061-2157,
// 2231-2286: every C element an ascending-k fma chain from beta*C with
// A_PART = ALPHA*A rounded once), so bit-identical to it; a leaner main loop:
//
//   * block 256 x 256, 8 waves (2 x 4), wave tile 128 x 64 = 4 x 2
//     v_mfma_f32_32x32x2_f32 accumulators; k-tiles of 32, two LDS stages;
//   * B (n-contiguous rows) streams global -> LDS by LDS-DMA
//     (global_load_lds_dwordx4: one wave-instruction = one 1 KB k-row of the
//     tile), no staging registers, no ds_write;
//   * A (k-contiguous rows) is transposed through registers into a k-major
//     image whose columns are permuted so a lane's four 32-row fragments
//     (rows lc, lc+32, lc+64, lc+96 of its wave tile) sit in one 16-byte slot
//     — one ds_read_b128 per MFMA step instead of four ds_read_b32 — and
//     XOR-swizzled by k/4 so the transposing ds_write_b32 are conflict-free
//     (staging lanes cover rows m, m+32, m+64, m+96 of 8 k-quads);
//   * fragments of step s+1 are read before step s's MFMAs are issued
//     (pinned there by scheduling fences);
//   * interior-only addressing: no bounds tests, no zero page in the loop.
#include <type_traits>

#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// BM x BN block tile, WM x WN waves (wave tile WTM x WTN = TM x TN 32x32
// accumulators), MINB blocks per CU, k-tiles of BK (32, or 16 where two
// blocks share a CU: two LDS stages of each fit beside the other's)
template <int BM, int BN, int WM, int WN, int MINB, int BK = 32>
struct Geo {
  static constexpr int BM_ = BM, BN_ = BN, WN_ = WN, MINB_ = MINB, BK_ = BK;
  static constexpr int KQ = BK / 4;                 // k-quads per tile row
  static constexpr int NT = 64 * WM * WN;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int TM = WTM / 32, TN = WTN / 32;
  static constexpr int LDA = BM, LDB = BN;          // LDS row lengths (k-major)
  static constexpr int A_TILE = BK * LDA, B_TILE = BK * LDB;
  static constexpr int STAGE = A_TILE + B_TILE;
  static constexpr int AU = BM * BK / 4 / NT;       // float4 A staging units / thread
  static constexpr int BROWS = 256 / BN;            // B k-rows per DMA wave-instruction
  static constexpr int BDMA = BK / BROWS / (NT / 64);  // DMA instructions per wave per tile
  static_assert(TM == 2 || TM == 4, "A fragments read as one b64 / b128");
  static_assert(BN == 128 || BN == 256, "B rows of 512 B or 1 KB per DMA");
  static_assert(AU >= 1 && BDMA >= 1 && BM * BK / 4 % NT == 0, "staging split");
  static_assert(BK == 16 || BK == 32, "k-quad swizzle over at most 8 quads");
};

template <class G>
__global__ __launch_bounds__(G::NT, G::MINB_) void sgemm_nn_big_kernel(GemmArgs p) {
  constexpr int BM = G::BM_, BN = G::BN_, NT = G::NT, WN = G::WN_;
  constexpr int WTM = G::WTM, WTN = G::WTN, TM = G::TM, TN = G::TN;
  constexpr int LDA = G::LDA, LDB = G::LDB, A_TILE = G::A_TILE, STAGE = G::STAGE;
  constexpr int AU = G::AU, BK = G::BK_, KQ = G::KQ;
  // column swizzle of k-quad kq: a wave's staging lanes cover 64/KQ
  // consecutive columns of each of the KQ quads; XOR with kq << SW moves
  // each quad's columns to their own bank range (KQ = 8: the 4-column
  // rotation; KQ = 4: 16-column blocks)
  constexpr int SW = KQ == 8 ? 2 : 4;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lc = lane & 31, h = lane >> 5;
  const int wm = wid / WN, wn = wid % WN;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  // XCD-contiguous grouped raster (as sgemm_kernel.hpp map_tile)
  const int tiles_m = (int)(p.M / BM), tiles_n = (int)(p.N / BN);
  int tm, tn;
  {
    const int nb = tiles_m * tiles_n, bid = blockIdx.x;
    const int xcd = bid & 7, q = nb >> 3, r = nb & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    constexpr int GROUP_M = 8;
    const int per_group = GROUP_M * tiles_n;
    const int group = wg / per_group, first_m = group * GROUP_M;
    const int gsize = min(tiles_m - first_m, GROUP_M);
    const int in_group = wg - group * per_group;
    tm = first_m + in_group % gsize;
    tn = in_group / gsize;
  }
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN, bz = blockIdx.y;
  const float* __restrict__ A = p.A + bz * p.strideA;
  const float* __restrict__ B = p.B + bz * p.strideB;
  float* __restrict__ C = p.C + bz * p.strideC;
  const int64_t lda = p.lda, ldb = p.ldb, ldc = p.ldc;

  // ---- accumulators: 0, C or beta*C -------------------------------------
  floatx16 acc[TM][TN];
  const int64_t row_base = m0 + wm * WTM + 4 * h;
  const int64_t col_base = n0 + wn * WTN + lc;
  if (p.beta_mode == BETA_ZERO) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
  } else {  // all loads issued before any use; one branch for the block
    const bool scale = p.beta_mode == BETA_SCALE;
    const float beta = p.beta;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          acc[i][j][e] = C[(row_base + 32 * i + (e & 3) + 8 * (e >> 2)) * ldc + col_base + 32 * j];
    if (scale) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][j][e] = beta * acc[i][j][e];
    }
  }
  // materialise the accumulators here: hipcc would otherwise place the wait
  // for these C loads at their first use inside the k-loop body, where the
  // same vmcnt wait (executed every tile) also drains the next tile's B DMA
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(acc[i][j]));

  // ---- A staging: unit u of this thread = k-quad kq, tile row m ----------
  // LDS column of row m: perm(m) = (m & ~(WTM-1)) | (m & 31)*TM | (m >> 5)%TM,
  // so lane lc's TM fragments (rows lc + 32i of its wave tile) are adjacent;
  // the staging index mm (0..BM-1) IS that column: m(mm) inverts perm
  const float* a_src[AU];
  int a_dst[AU];
#pragma unroll
  for (int u = 0; u < AU; ++u) {
    const int idx = tid + NT * u;
    const int kq = idx % KQ, mm = idx / KQ;
    const int m = (mm & ~(WTM - 1)) | ((mm % TM) << 5) | ((mm & (WTM - 1)) / TM);
    a_src[u] = A + (m0 + m) * lda + 4 * kq;
    a_dst[u] = (4 * kq) * LDA + (mm ^ (kq << SW));  // element c adds c*LDA
  }
  float4 ra[AU];
  const float alpha = p.alpha;
  auto load_a = [&](int64_t k0) {
#pragma unroll
    for (int u = 0; u < AU; ++u) ra[u] = *reinterpret_cast<const float4*>(a_src[u] + k0);
  };
  auto store_a = [&](float* as) {
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      float4 v = ra[u];  // A_PART = ALPHA*A[kk] (1*x == x bit for bit: no branch)
      v.x = alpha * v.x; v.y = alpha * v.y; v.z = alpha * v.z; v.w = alpha * v.w;
      as[a_dst[u]] = v.x;
      as[a_dst[u] + LDA] = v.y;
      as[a_dst[u] + 2 * LDA] = v.z;
      as[a_dst[u] + 3 * LDA] = v.w;
    }
  };
  // ---- B staging: LDS-DMA; one wave-instruction moves BROWS k-rows (1 KB),
  // wave w fetches rows BROWS*BDMA*w .. +BROWS*BDMA-1 -------------------------
  constexpr int BROWS = G::BROWS, BDMA = G::BDMA;
  const int brow = BROWS * BDMA * wid + lane / (BN / 4);
  const float* b_src = B + (int64_t)brow * ldb + n0 + 4 * (lane % (BN / 4));
  const unsigned b_lds0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)(smem + A_TILE +
                                                                      BROWS * BDMA * wid * LDB));
  auto dma_b = [&](int64_t k0, int stage) {
#pragma unroll
    for (int r = 0; r < BDMA; ++r) {
      unsigned keep;
      const float* src = b_src + (k0 + BROWS * r) * ldb;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(src), "s"(b_lds0 + (unsigned)((stage * STAGE + BROWS * r * LDB) * 4))
          : "memory");
    }
  };

  // ---- fragments: step s of a k-tile consumes k = 2s + h ------------------
  const int a_frag = wm * WTM + TM * lc;    // TM floats: rows lc + 32i
  const int b_frag = wn * WTN + lc;         // rows lc + 32j
  auto frag = [&](const float* st, int s, float (&a)[TM], float (&b)[TN]) {
    const int k = 2 * s + h;
#ifdef TNS_NB_NO_FRAG  // (diagnostic: MFMAs on register operands, no LDS reads)
    for (int i = 0; i < TM; ++i) a[i] = (float)(lane + i + s);
    for (int j = 0; j < TN; ++j) b[j] = (float)(lane - j + s);
    (void)st; (void)k;
    return;
#endif
    const float* ap = st + k * LDA + (a_frag ^ (((k >> 2) & (KQ - 1)) << SW));
    if constexpr (TM == 4) {
      const float4 v = *reinterpret_cast<const float4*>(ap);
      a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
    } else {
      const float2 v = *reinterpret_cast<const float2*>(ap);
      a[0] = v.x; a[1] = v.y;
    }
    const float* bp = st + A_TILE + k * LDB + b_frag;
#pragma unroll
    for (int j = 0; j < TN; ++j) b[j] = bp[32 * j];
  };
  auto mma = [&](const float (&a)[TM], const float (&b)[TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
  };

  const int nt = (int)(p.K / BK);
  if (nt > 0) {
    load_a(0);
    dma_b(0, 0);
    store_a(smem);  // (the compiler waits for the A loads; the DMA is older)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // tile t: B DMA and A loads of tile t+1 first, MFMAs of tile t from LDS
  // (fragments one step ahead), A of tile t+1 written mid-tile, barrier.
  // The last tile is peeled so the loop body has no conditional staging
  // (a conditional store made hipcc keep the A loads "pending" across the
  // back-edge and drain vmcnt — the fresh B DMA included — at the loop top).
  auto tile = [&](int t, auto MORE) {
    constexpr bool more = decltype(MORE)::value;
    const float* cur = smem + (t & 1) * STAGE;
    float* nxt = smem + ((t + 1) & 1) * STAGE;
    if constexpr (more) {
#ifndef TNS_NB_NO_DMA  // (diagnostic builds: timing without this part)
      dma_b((int64_t)(t + 1) * BK, (t + 1) & 1);
#endif
#ifndef TNS_NB_NO_AST
      load_a((int64_t)(t + 1) * BK);
#endif
      // keep the A loads at the top of the tile (the scheduler sinks them
      // next to their mid-tile use otherwise, exposing their latency)
      __builtin_amdgcn_sched_barrier(0);
    }
    float a0[TM], b0[TN], a1[TM], b1[TN];
    frag(cur, 0, a0, b0);
#pragma unroll
    for (int s = 0; s < BK / 2; s += 2) {
      // (scheduling fences: hipcc otherwise sinks each fragment read next to
      // its MFMAs and waits on it there; fenced, a step's reads are in flight
      // behind the previous step's 8 MFMAs — 4096^3 1.000 -> 0.996 ms)
      frag(cur, s + 1, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a0, b0);
      if (s + 2 < BK / 2) frag(cur, s + 2, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (more)
        if (s == BK / 4 - 2) {  // mid-tile: A of tile t+1 (its loads' first use)
          __builtin_amdgcn_sched_barrier(0);
#ifndef TNS_NB_NO_AST
          store_a(nxt);
#endif
        }
      mma(a1, b1);
    }
    if constexpr (more) {
#ifndef TNS_NB_NO_BAR
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t+1's B DMA landed
      __syncthreads();
#endif
    }
  };
  for (int t = 0; t + 1 < nt; ++t) tile(t, std::true_type{});
  if (nt > 0) tile(nt - 1, std::false_type{});

  // ---- epilogue ----------------------------------------------------------
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t row = row_base + 32 * i + (e & 3) + 8 * (e >> 2);
#pragma unroll
      for (int j = 0; j < TN; ++j) C[row * ldc + col_base + 32 * j] = acc[i][j][e];
    }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

using G256 = Geo<256, 256, 2, 4, 1>;  // 8 waves, wave tile 128x64, 1 block/CU
using G128 = Geo<128, 128, 2, 2, 2>;  // 4 waves, wave tile 64x64, 2 blocks/CU
using G256x128 = Geo<256, 128, 2, 2, 1>;  // 4 waves, wave tile 128x64
using G256w16 = Geo<256, 256, 4, 4, 1>;   // 16 waves, wave tile 64x64, 4 waves per SIMD
// 4 waves, wave tile 128x64, k-tiles of 16: two blocks per CU (2 x 48 KB of
// LDS), so one block's barrier and staging are covered by the other's MFMAs
using G256x128k16 = Geo<256, 128, 2, 2, 2, 16>;

template <class G>
bool applies(const GemmArgs& a) {
  if (a.conv || a.epi != EPI_NONE || a.beta_mode == BETA_STORE) return false;
  if (a.M % G::BM_ || a.N % G::BN_ || a.K % G::BK_ || a.M <= 0 || a.N <= 0) return false;
  if (a.lda % 4 || a.ldb % 4 || !aligned16(a.A) || !aligned16(a.B)) return false;
  if (a.batch > 1 && (a.strideA % 4 || a.strideB % 4)) return false;
  return (a.M / G::BM_) * (a.N / G::BN_) <= 0x7fffffff;
}

template <class G>
hipError_t launch(const GemmArgs& a, hipStream_t s) {
  if (!applies<G>(a)) return hipErrorInvalidValue;
  const int64_t tiles = (a.M / G::BM_) * (a.N / G::BN_);
  for (int64_t b0 = 0; b0 < a.batch; b0 += 65535) {
    GemmArgs sub = a;
    const int64_t nb = a.batch - b0 < 65535 ? a.batch - b0 : 65535;
    sub.A = a.A + b0 * a.strideA;
    sub.B = a.B + b0 * a.strideB;
    sub.C = a.C + b0 * a.strideC;
    sub.batch = nb;
    hipLaunchKernelGGL(sgemm_nn_big_kernel<G>, dim3((unsigned)tiles, (unsigned)nb), dim3(G::NT), 0,
                       s, sub);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

// (a 4-wave 256x256 form, wave tile 128x128 at one wave per SIMD, spills 67
// registers at the 512 cap — not instantiated)
// (form 5 is the ping-pong schedule of the 256x256 tile, sgemm_nn_pp.hip;
// form 6 the tile at one wave per SIMD with both operands by LDS-DMA and
// interleaved columns, sgemm_nn_w4.hip; form 7, the ping-pong tile with B
// register-staged into k-permuted slots, is compiled into the diagnostics
// build only: measured, not picked)
#ifdef TNS_DIAG_KERNELS
int sgemm_nn_big_count() { return 8; }
#else
int sgemm_nn_big_count() { return 7; }
#endif
const char* sgemm_nn_big_name(int v) {
  static const char* names[] = {"256x256x32_w2x4_nn_big", "128x128x32_w2x2_nn_big",
                                "256x128x32_w2x2_nn_big", "256x256x32_w4x4_nn_big",
                                "256x128x16_w2x2_b2_nn_big", "256x256x32_w2x4_pp_nn_big",
                                "256x256x32_w2x2_dma_nn_big", "256x256x32_w2x4_ppbq_nn_big"};
  return v >= 0 && v < sgemm_nn_big_count() ? names[v] : "";
}

// heuristic: the 256x256 tile when it gives about a block per CU, at one
// wave per SIMD with LDS-DMA operands where it applies (form 6; 4096^3 0.983
// -> 0.950 ms against the ping-pong form 5, which itself took 0.994 -> 0.972
// from form 0; all bit-identical)
int sgemm_nn_big_pick(const GemmArgs& a) {
  if (applies<G256>(a) && (a.M / 256) * (a.N / 256) * a.batch >= 192)
    return sgemm_nn_w4_applies(a) ? 6 : sgemm_nn_pp_applies(a) ? 5 : 0;
  return -1;
}

hipError_t launch_sgemm_nn_big(int v, const GemmArgs& a, hipStream_t s) {
  switch (v) {
    case 0: return launch<G256>(a, s);
    case 1: return launch<G128>(a, s);
    case 2: return launch<G256x128>(a, s);
    case 3: return launch<G256w16>(a, s);
    case 4: return launch<G256x128k16>(a, s);
    case 5: return launch_sgemm_nn_pp(a, s);
    case 6: return launch_sgemm_nn_w4(a, s);
#ifdef TNS_DIAG_KERNELS
    case 7: return launch_sgemm_nn_pp(a, s, true);  // k-permuted B slots
#endif
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tns
