// sgemm_tt.hip — gemm(Trans, Trans) in the reference's scalar s_tt order.
//
// Replaces sgemm_tt / s_tt (ntensors.pas:2159-2206) behind cblas_sgemm
// (2231-2286):  sum := 0; for kk ascending: sum := sum + ALPHA*A[i+kk*lda]*
// B[kk+j*ldb]; C[i,j] := C[i,j] + sum, after the mulvs beta pre-scale.  FPC
// evaluates the product left to right and rounds every operation to single
// (no FMA), so each step is  t1 = rn(alpha*a), t2 = rn(t1*b), sum = rn(sum+t2).
// fp32 MFMA fuses its multiply-add and cannot produce these roundings, so this
// path runs on the VALU: packed v_pk_mul_f32 / v_pk_add_f32 (two outputs per
// instruction; the library is built with -ffp-contract=off, so they are never
// fused into v_pk_fma_f32).
//
// A block owns a BM x BN tile of C (256 threads, RxR outputs per thread split
// into 4x4 quads 64 apart, so the float4 LDS reads of a k-row are
// conflict-free).  Per k-tile of 16 the alpha-scaled A rows (t1, contiguous
// over i in the TT layout) and the B columns (contiguous over kk, transposed
// on the way in) are staged global -> registers -> LDS, double-buffered with
// one barrier per tile.  Zero-filled k >= K adds rn(sum + (+0)) = sum (sum is
// never -0: it starts at +0 and exact cancellation rounds to +0).
#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int TT_NT = 256;
constexpr int TT_BK = 16;

template <int R>  // outputs per thread per dimension (4 or 8)
__global__ __launch_bounds__(TT_NT, R == 8 ? 2 : 4) void sgemm_tt_kernel(GemmArgs p) {
  constexpr int Q = R / 4;             // quads per dimension
  constexpr int BM = 64 * Q, BN = 64 * Q;
  constexpr int LDA_S = BM, LDB_S = BN + 4;  // B transposed: pad the row
  constexpr int EA = TT_BK * BM / TT_NT, EB = TT_BK * BN / TT_NT;
  __shared__ __attribute__((aligned(16))) float as[2][TT_BK * LDA_S];
  __shared__ __attribute__((aligned(16))) float bs[2][TT_BK * LDB_S];

  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int tiles_m = (int)((p.M + BM - 1) / BM);
  const int64_t m0 = (int64_t)(blockIdx.x % tiles_m) * BM;
  const int64_t n0 = (int64_t)(blockIdx.x / tiles_m) * BN;
  const int64_t bz = blockIdx.y;
  const float* __restrict__ A = p.A + bz * p.strideA;
  const float* __restrict__ B = p.B + bz * p.strideB;
  float* __restrict__ C = p.C + bz * p.strideC;
  const int64_t M = p.M, N = p.N, K = p.K;
  const float alpha = p.alpha;

  float ra[EA], rb[EB];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int u = 0; u < EA; ++u) {  // A(kk, i) = A[kk*lda + i]: coalesced over i
      const int idx = tid + TT_NT * u;
      const int64_t kk = k0 + idx / BM, i = m0 + idx % BM;
      ra[u] = (kk < K && i < M) ? alpha * A[kk * p.lda + i] : 0.0f;  // t1
    }
#pragma unroll
    for (int u = 0; u < EB; ++u) {  // B(kk, j) = B[j*ldb + kk]: runs over kk
      const int idx = tid + TT_NT * u;
      const int64_t kk = k0 + idx % TT_BK, j = n0 + idx / TT_BK;
      rb[u] = (kk < K && j < N) ? B[j * p.ldb + kk] : 0.0f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < EA; ++u) {
      const int idx = tid + TT_NT * u;
      as[buf][(idx / BM) * LDA_S + idx % BM] = ra[u];
    }
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      const int idx = tid + TT_NT * u;
      bs[buf][(idx % TT_BK) * LDB_S + idx / TT_BK] = rb[u];
    }
  };

  f2 acc[R][R / 2];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int c = 0; c < R / 2; ++c) acc[r][c] = f2{0.0f, 0.0f};

  const int nt = (int)((K + TT_BK - 1) / TT_BK);
  if (nt > 0) {
    load(0);
    store(0);
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      const int cur = t & 1;
      if (t + 1 < nt) load((int64_t)(t + 1) * TT_BK);
#pragma unroll 2
      for (int kk = 0; kk < TT_BK; ++kk) {
        float a[R], b[R];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const float4 va = *reinterpret_cast<const float4*>(&as[cur][kk * LDA_S + 64 * q + 4 * ty]);
          const float4 vb = *reinterpret_cast<const float4*>(&bs[cur][kk * LDB_S + 64 * q + 4 * tx]);
          a[4 * q + 0] = va.x; a[4 * q + 1] = va.y; a[4 * q + 2] = va.z; a[4 * q + 3] = va.w;
          b[4 * q + 0] = vb.x; b[4 * q + 1] = vb.y; b[4 * q + 2] = vb.z; b[4 * q + 3] = vb.w;
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int c = 0; c < R / 2; ++c) {
            const f2 t2 = f2{a[r], a[r]} * f2{b[2 * c], b[2 * c + 1]};  // rn(t1*b)
            acc[r][c] = acc[r][c] + t2;                               // rn(sum+t2)
          }
      }
      if (t + 1 < nt) store(cur ^ 1);
      __syncthreads();
    }
  }

  const float beta = p.beta;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t m = m0 + 64 * (r / 4) + 4 * ty + (r % 4);
    if (m >= M) continue;
#pragma unroll
    for (int c = 0; c < R; ++c) {
      const int64_t n = n0 + 64 * (c / 4) + 4 * tx + (c % 4);
      if (n >= N) continue;
      const float sum = acc[r][c / 2][c % 2];
      float* cp = C + m * p.ldc + n;
      float c0;
      if (p.beta_mode == BETA_ZERO)
        c0 = 0.0f;
      else if (p.beta_mode == BETA_SCALE)
        c0 = beta * *cp;  // cblas_sgemm's mulvs pre-scale
      else
        c0 = *cp;
      *cp = c0 + sum;  // C[i*ldc+j] := C[i*ldc+j] + sum
    }
  }
}

template <int R>
hipError_t launch_r(const GemmArgs& a, hipStream_t s) {
  constexpr int BT = 16 * R;
  const int64_t tiles = ((a.M + BT - 1) / BT) * ((a.N + BT - 1) / BT);
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  for (int64_t b0 = 0; b0 < a.batch; b0 += 65535) {
    GemmArgs sub = a;
    const int64_t nb = a.batch - b0 < 65535 ? a.batch - b0 : 65535;
    sub.A = a.A + b0 * a.strideA;
    sub.B = a.B + b0 * a.strideB;
    sub.C = a.C + b0 * a.strideC;
    sub.batch = nb;
    hipLaunchKernelGGL((sgemm_tt_kernel<R>), dim3((unsigned)tiles, (unsigned)nb), dim3(TT_NT),
                       0, s, sub);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

// 128x128 tiles (8x8 per thread) when they still give >= 2 blocks per CU,
// else 64x64 (4x4 per thread)
hipError_t launch_sgemm_tt(const GemmArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0 || a.batch <= 0) return hipSuccess;
  const int64_t b128 = ((a.M + 127) / 128) * ((a.N + 127) / 128) * a.batch;
  return b128 >= 512 ? launch_r<8>(a, s) : launch_r<4>(a, s);
}

}  // namespace tns
