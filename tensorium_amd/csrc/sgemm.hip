// sgemm.hip — fp32 SGEMM on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
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
//   This kernel feeds each accumulator k in ascending order (k-tiles
//   ascending, MFMA steps ascending, lane-half 0 = the lower k of a step),
//   pre-multiplies A by alpha once (the reference's A_PART) and starts the
//   accumulator at beta*C (the reference's mulvs pre-scale).  NT/TT use a
//   different summation order in the reference (8-lane sdot / unfused
//   mul+add) and agree within the componentwise bound documented in DESIGN.md.
//
// Structure: 128x128 block tile, BK=32, 256 threads = 4 waves (2x2), each
// wave owns 64x64 = 2x2 MFMA 32x32 accumulators (64 acc VGPRs).  Operands
// are staged global -> registers (float4 where the layout allows) -> LDS in
// k-major [k][m] / [k][n] images (double-buffered, one barrier per k-tile);
// the next tile's global loads are issued before the current tile's MFMAs.
// Block index is remapped so that the 8 XCDs each get a contiguous, grouped
// region of C (L2 reuse of A/B panels).
#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128;
constexpr int BN = 128;
constexpr int BK = 32;
constexpr int NTHREADS = 256;
constexpr int GROUP_M = 8;

// LDS row length of a k-major operand image.  K-contiguous operands are
// transposed on the way in (4 scalar ds_writes per float4); a row length
// of 129 (≡ 1 mod 8) makes those writes bank-conflict free.  MN-contiguous
// operands are written with ds_write_b128 and keep 128.
template <bool KCONTIG>
struct LdsLd {
  static constexpr int value = KCONTIG ? BM + 1 : BM;
};

// Loads one BK x 128 operand tile (k, mn) into 16 registers per thread.
//   KCONTIG:  element (k, mn) at base[(mn0+mn)*ld + k0+k]   (A NoTrans / B Trans)
//   else   :  element (k, mn) at base[(k0+k)*ld + mn0+mn]   (A Trans / B NoTrans)
// Out-of-range elements read as 0.
template <bool KCONTIG, int VEC>
__device__ __forceinline__ void load_tile(float (&r)[16], const float* __restrict__ base,
                                          int64_t ld, int64_t mn0, int64_t k0, int64_t MN,
                                          int64_t K, int tid) {
  if constexpr (VEC == 4) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = tid + NTHREADS * it;
      int64_t gk, gmn;
      bool full, any;
      if constexpr (KCONTIG) {
        gk = k0 + 4 * (idx & 7);
        gmn = mn0 + (idx >> 3);
        full = (gmn < MN) && (gk + 3 < K);
        any = (gmn < MN);
      } else {
        gk = k0 + (idx >> 5);
        gmn = mn0 + 4 * (idx & 31);
        full = (gk < K) && (gmn + 3 < MN);
        any = (gk < K);
      }
      const float* ptr = KCONTIG ? base + gmn * ld + gk : base + gk * ld + gmn;
      float4 v;
      if (full) {
        v = *reinterpret_cast<const float4*>(ptr);
      } else {
        float t[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          bool ok = any && (KCONTIG ? (gk + c < K) : (gmn + c < MN));
          t[c] = ok ? ptr[c] : 0.0f;
        }
        v = make_float4(t[0], t[1], t[2], t[3]);
      }
      r[4 * it + 0] = v.x;
      r[4 * it + 1] = v.y;
      r[4 * it + 2] = v.z;
      r[4 * it + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int idx = tid + NTHREADS * it;
      int64_t gk, gmn;
      if constexpr (KCONTIG) {
        gk = k0 + (idx & 31);
        gmn = mn0 + (idx >> 5);
      } else {
        gk = k0 + (idx >> 7);
        gmn = mn0 + (idx & 127);
      }
      const float* ptr = KCONTIG ? base + gmn * ld + gk : base + gk * ld + gmn;
      r[it] = (gk < K && gmn < MN) ? *ptr : 0.0f;
    }
  }
}

template <bool KCONTIG, int VEC>
__device__ __forceinline__ void store_tile(const float (&r)[16], float* __restrict__ xs, int tid) {
  constexpr int LD = LdsLd<KCONTIG>::value;
  if constexpr (VEC == 4) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = tid + NTHREADS * it;
      if constexpr (KCONTIG) {
        const int kq = idx & 7, mn = idx >> 3;
#pragma unroll
        for (int c = 0; c < 4; ++c) xs[(4 * kq + c) * LD + mn] = r[4 * it + c];
      } else {
        const int mq = idx & 31, k = idx >> 5;
        *reinterpret_cast<float4*>(xs + k * LD + 4 * mq) =
            make_float4(r[4 * it], r[4 * it + 1], r[4 * it + 2], r[4 * it + 3]);
      }
    }
  } else {
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int idx = tid + NTHREADS * it;
      if constexpr (KCONTIG) {
        xs[(idx & 31) * LD + (idx >> 5)] = r[it];
      } else {
        xs[(idx >> 7) * LD + (idx & 127)] = r[it];
      }
    }
  }
}

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

template <bool TA, bool TB, int AV, int BV>
__global__ __launch_bounds__(NTHREADS, 2) void sgemm_mfma_kernel(GemmArgs p) {
  constexpr bool AKC = !TA;  // A is k-contiguous in memory
  constexpr bool BKC = TB;   // B is k-contiguous in memory
  constexpr int LDA_S = LdsLd<AKC>::value;
  constexpr int LDB_S = LdsLd<BKC>::value;
  constexpr int A_TILE = BK * LDA_S;
  constexpr int B_TILE = BK * LDB_S;
  constexpr int STAGE = A_TILE + B_TILE;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int l31 = lane & 31;
  const int h = lane >> 5;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int tiles_m = (int)((p.M + BM - 1) / BM);
  const int tiles_n = (int)((p.N + BN - 1) / BN);
  int tm, tn;
  map_tile(blockIdx.x, tiles_m, tiles_n, tm, tn);
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t bz = blockIdx.y;

  const float* __restrict__ A = p.A + bz * p.strideA;
  const float* __restrict__ B = p.B + bz * p.strideB;
  float* __restrict__ C = p.C + bz * p.strideC;
  const int64_t M = p.M, N = p.N, K = p.K;

  // ---- accumulator init: 0, C, or beta*C (reference mulvs pre-scale) -----
  floatx16 acc00, acc01, acc10, acc11;
  const int64_t row_base = m0 + wm * 64 + 4 * h;
  const int64_t col_base = n0 + wn * 64 + l31;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    acc00[i] = 0.0f;
    acc01[i] = 0.0f;
    acc10[i] = 0.0f;
    acc11[i] = 0.0f;
  }
  if (p.beta_mode != BETA_ZERO) {
    const bool scale = p.beta_mode == BETA_SCALE;
    const float beta = p.beta;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int rr = (i & 3) + 8 * (i >> 2);
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int64_t row = row_base + r * 32 + rr;
          const int64_t col = col_base + c * 32;
          float v = 0.0f;
          if (row < M && col < N) {
            v = C[row * p.ldc + col];
            if (scale) v = beta * v;
          }
          if (r == 0 && c == 0) acc00[i] = v;
          if (r == 0 && c == 1) acc01[i] = v;
          if (r == 1 && c == 0) acc10[i] = v;
          if (r == 1 && c == 1) acc11[i] = v;
        }
    }
  }

  const int nt = (int)((K + BK - 1) / BK);
  const bool scale_a = p.alpha != 1.0f;
  const float alpha = p.alpha;
  float ra[16], rb[16];

  if (nt > 0) {
    load_tile<AKC, AV>(ra, A, p.lda, m0, 0, M, K, tid);
    load_tile<BKC, BV>(rb, B, p.ldb, n0, 0, N, K, tid);
    if (scale_a) {
#pragma unroll
      for (int i = 0; i < 16; ++i) ra[i] = alpha * ra[i];  // A_PART = ALPHA*A[kk]
    }
    store_tile<AKC, AV>(ra, smem, tid);
    store_tile<BKC, BV>(rb, smem + A_TILE, tid);
    __syncthreads();
  }

  for (int t = 0; t < nt; ++t) {
    const float* as = smem + (t & 1) * STAGE;
    const float* bs = as + A_TILE;
    const bool has_next = (t + 1) < nt;
    if (has_next) {
      const int64_t k0 = (int64_t)(t + 1) * BK;
      load_tile<AKC, AV>(ra, A, p.lda, m0, k0, M, K, tid);
      load_tile<BKC, BV>(rb, B, p.ldb, n0, k0, N, K, tid);
    }
    const float* ap = as + h * LDA_S + wm * 64 + l31;
    const float* bp = bs + h * LDB_S + wn * 64 + l31;
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const float a0 = ap[2 * s * LDA_S];
      const float a1 = ap[2 * s * LDA_S + 32];
      const float b0 = bp[2 * s * LDB_S];
      const float b1 = bp[2 * s * LDB_S + 32];
      acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc00, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc01, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc10, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc11, 0, 0, 0);
    }
    if (has_next) {
      if (scale_a) {
#pragma unroll
        for (int i = 0; i < 16; ++i) ra[i] = alpha * ra[i];
      }
      float* nxt = smem + ((t + 1) & 1) * STAGE;
      store_tile<AKC, AV>(ra, nxt, tid);
      store_tile<BKC, BV>(rb, nxt + A_TILE, tid);
    }
    __syncthreads();
  }

  // ---- epilogue ----------------------------------------------------------
  const bool fuse = p.epi == EPI_BIAS_ACT;
  const int act = p.act;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int rr = (i & 3) + 8 * (i >> 2);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int64_t row = row_base + r * 32 + rr;
      if (row >= M) continue;
      const float bias = fuse ? p.bias[row] : 0.0f;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int64_t col = col_base + c * 32;
        if (col >= N) continue;
        float v = (r == 0) ? (c == 0 ? acc00[i] : acc01[i]) : (c == 0 ? acc10[i] : acc11[i]);
        if (fuse) v = act_apply(v + bias, act);  // forwardBias then activate
        C[row * p.ldc + col] = v;
      }
    }
  }
}

template <bool TA, bool TB, int AV, int BV>
hipError_t launch_variant(const GemmArgs& a, hipStream_t s) {
  const int64_t tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  for (int64_t b0 = 0; b0 < a.batch; b0 += 65535) {
    GemmArgs sub = a;
    const int64_t nb = a.batch - b0 < 65535 ? a.batch - b0 : 65535;
    sub.A = a.A + b0 * a.strideA;
    sub.B = a.B + b0 * a.strideB;
    sub.C = a.C + b0 * a.strideC;
    sub.batch = nb;
    hipLaunchKernelGGL((sgemm_mfma_kernel<TA, TB, AV, BV>), dim3((unsigned)tiles, (unsigned)nb),
                       dim3(NTHREADS), 0, s, sub);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <bool TA, bool TB>
hipError_t launch_trans(const GemmArgs& a, bool av, bool bv, hipStream_t s) {
  if (av && bv) return launch_variant<TA, TB, 4, 4>(a, s);
  if (av) return launch_variant<TA, TB, 4, 1>(a, s);
  if (bv) return launch_variant<TA, TB, 1, 4>(a, s);
  return launch_variant<TA, TB, 1, 1>(a, s);
}

bool vec4_ok(const float* p, int64_t ld, int64_t stride, int64_t batch) {
  if ((reinterpret_cast<uintptr_t>(p) & 15) != 0) return false;
  if (ld % 4 != 0) return false;
  if (batch > 1 && stride % 4 != 0) return false;
  return true;
}

}  // namespace

hipError_t launch_sgemm(const GemmArgs& a, bool transA, bool transB, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0 || a.batch <= 0) return hipSuccess;
  const bool av = vec4_ok(a.A, a.lda, a.strideA, a.batch);
  const bool bv = vec4_ok(a.B, a.ldb, a.strideB, a.batch);
  if (!transA && !transB) return launch_trans<false, false>(a, av, bv, s);
  if (!transA && transB) return launch_trans<false, true>(a, av, bv, s);
  if (transA && !transB) return launch_trans<true, false>(a, av, bv, s);
  return launch_trans<true, true>(a, av, bv, s);
}

}  // namespace tns
