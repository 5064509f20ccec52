// sgemm_sdot_chains.hip — gemm(NoTrans, Trans) in the sdot_avx2 order on the
// VALU, one lane per few residue chains.
//
// Same arithmetic as sgemm_sdot.hip (s_nt over sdot_avx2, ntensors.pas:
// 1957-2005, 1233-1306): C[i,j] := C[i,j] + ALPHA * sdot(K, A[i,:], B[j,:]),
// sdot = 8 ascending fma chains over k = l (mod 8) from +0, then
// s_l = lane_l + lane_{l+4} and (s0 + s1) + (s2 + s3).
//
// Why a second form: the MFMA kernel gives one 32x32 output tile's 8 chains
// to 8 waves, so a product with few outputs and a very long k — the conv dW
// GEMMs of the large YOLOv3 layers (layer 0: 32 x 27 outputs per image over
// k = 173056; nConvolutionLayer.pas:636-640) — occupies a handful of CUs that
// stream the whole k alone.  Here every chain (output, residue) is its own
// accumulator in a lane's registers: a lane holds R consecutive residues of
// RM x RN outputs, the block's A and B rows are staged through LDS in k-chunks
// of KC (row-major, k contiguous, row stride KC + 8 so the 8 rows a half-wave
// reads fall in distinct bank octets), and per 8 k the lane reads its R
// residues of each row as one ds_read_b64 / b128 and issues RM*RN*R fma
// (packed pairs).  55296 independent chains on layer 0 instead of 64 MFMA
// waves.  The chain order (ascending k per residue, zero-filled k >= K adds
// fma(0, 0, x) = x) and the fold are the reference's, so the result is bit
// for bit the MFMA kernel's.
#include "tns_internal.hpp"

namespace tns {
namespace {

constexpr int KC = 256;      // k per staged chunk (32 steps per residue)
constexpr int KP = KC + 8;   // LDS row stride (= 8 mod 64 dwords)

typedef float f2 __attribute__((ext_vector_type(2)));

template <int R>
struct Vec;
template <>
struct Vec<2> {
  typedef float2 T;
  static __device__ inline void get(const float* p, float (&v)[2]) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    v[0] = t.x; v[1] = t.y;
  }
};
template <>
struct Vec<4> {
  static __device__ inline void get(const float* p, float (&v)[4]) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
};
template <>
struct Vec<8> {
  static __device__ inline void get(const float* p, float (&v)[8]) {
    const float4 t = reinterpret_cast<const float4*>(p)[0];
    const float4 u = reinterpret_cast<const float4*>(p)[1];
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    v[4] = u.x; v[5] = u.y; v[6] = u.z; v[7] = u.w;
  }
};

// stages of KC k per row in the LDS ring: as many as fit in ~80 KB (two
// blocks per CU), at least 2
template <int ROWS>
constexpr int ring_stages() {
  constexpr int st = ROWS * KP * 4;
  constexpr int n = 80 * 1024 / st;
  return n < 2 ? 2 : (n > 8 ? 8 : n);
}

// NT threads; a group of 8/R consecutive lanes owns RM x RN outputs (rows
// gm + GM*i of A, gn + GN*j of B), lane s of the group residues R*s..R*s+R-1.
// GL: operands 16-byte aligned with K % 4 == 0 — full k-chunks stream into an
// LDS ring of S stages by LDS-DMA (global_load_lds_dwordx4: one wave-
// instruction = one row's 1 KB chunk, lane-linear), S-1 chunks in flight
// behind counted vmcnt waits and raw barriers; the ragged last chunk and the
// !GL form load through registers with zero fill.
template <int NT, int R, int RM, int RN, int GM, bool GL>
__global__ __launch_bounds__(NT) void sdot_chains_kernel(GemmArgs p, int tiles_m, int tiles) {
  constexpr int LPO = 8 / R;
  constexpr int NG = NT / LPO;
  constexpr int GN = NG / GM;
  static_assert(NG % GM == 0, "groups");
  constexpr int TM = GM * RM, TN = GN * RN, ROWS = TM + TN;
  constexpr int W = NT / 64;
  static_assert(ROWS % W == 0, "rows per wave");
  constexpr int I = ROWS / W;            // DMA instructions per wave per chunk
  constexpr int UNITS = ROWS * KC / 4;   // float4 staging units per chunk
  static_assert(UNITS % NT == 0, "staging split");
  constexpr int U = UNITS / NT;
  constexpr int STAGE = ROWS * KP;
  constexpr int S = GL ? ring_stages<ROWS>() : 2;
  static_assert((S - 2) * I <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) float lds[S * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int s = tid % LPO, grp = tid / LPO, gm = grp % GM, gn = grp / GM;
  // XCD-contiguous order: the blocks one XCD runs (blockIdx.x = xcd + 8j)
  // take a contiguous range of (image, tile), so an image's rows are shared
  // in that XCD's L2 (bijective for any grid size)
  const int nwg = gridDim.x, xcd = blockIdx.x & 7, q = nwg >> 3, r8 = nwg & 7;
  const int wid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (blockIdx.x >> 3);
  const int tile = wid % tiles;
  const int64_t bz = wid / tiles;
  const int64_t m0 = (int64_t)(tile % tiles_m) * TM;
  const int64_t n0 = (int64_t)(tile / tiles_m) * TN;
  const float* __restrict__ A = p.A + bz * p.strideA;
  const float* __restrict__ B = p.B + bz * p.strideB;
  const int64_t M = p.M, N = p.N, K = p.K;

  // register staging of chunk k0 (zero fill past K and past the last row)
  auto stage_regs = [&](int64_t k0, float* buf) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = tid + NT * u;
      const int row = idx / (KC / 4);
      const int64_t k = k0 + 4 * (idx % (KC / 4));
      const bool isa = row < TM;
      const int64_t g = isa ? m0 + row : n0 + row - TM;
      const bool rok = g < (isa ? M : N);
      const float* src = (isa ? A + g * p.lda : B + g * p.ldb) + k;
      float4 v;
      if (GL && rok && k + 4 <= K) {
        v = *reinterpret_cast<const float4*>(src);
      } else {
        float e4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) e4[e] = (rok && k + e < K) ? src[e] : 0.0f;
        v = make_float4(e4[0], e4[1], e4[2], e4[3]);
      }
      *reinterpret_cast<float4*>(buf + (idx / (KC / 4)) * KP + 4 * (idx % (KC / 4))) = v;
    }
  };
  // LDS-DMA of full chunk c into its ring stage: wave wv fetches rows
  // wv*I .. wv*I+I-1 (rows past M / N re-read a valid row; never stored)
  const float* rowp[I];
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const int row = wv * I + i;
    const bool isa = row < TM;
    int64_t g = isa ? m0 + row : n0 + row - TM;
    const int64_t lim = isa ? M : N;
    g = g < lim ? g : lim - 1;
    rowp[i] = (isa ? A + g * p.lda : B + g * p.ldb) + 4 * lane;
  }
  // issued as inline asm: hipcc tracks a builtin LDS-DMA as a pending LDS
  // write and drains vmcnt(0) before every ds_read; the ring's own counted
  // waits order it instead (M0 = the wave-uniform LDS destination)
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)(lds + wv * I * KP));
  auto dma = [&](int c) {
    const unsigned base = lds0 + (unsigned)((c % S) * STAGE * 4);
#pragma unroll
    for (int i = 0; i < I; ++i) {
      unsigned keep;
      const float* src = rowp[i] + (int64_t)c * KC;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(src), "s"(base + (unsigned)(i * KP * 4))
          : "memory");
    }
  };

  float acc[RM][RN][R];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int e = 0; e < R; ++e) acc[i][j][e] = 0.0f;

  // one chunk: KC/8 steps per residue in groups of G, the next group's LDS
  // reads issued before the current group's fma (one wave per SIMD is the
  // common case here, so the read latency must overlap the fma)
  constexpr int OPS = (RM + RN) * R;           // floats read per step
  constexpr int G = OPS >= 16 ? 2 : (OPS >= 8 ? 4 : 8);
  constexpr int NGR = KC / 8 / G;
  auto fetch = [&](const float* pa, const float* pb, int g, float (&a)[G][RM][R],
                   float (&b)[G][RN][R]) {
#pragma unroll
    for (int q = 0; q < G; ++q) {
#pragma unroll
      for (int i = 0; i < RM; ++i) Vec<R>::get(pa + i * GM * KP + 8 * (g * G + q), a[q][i]);
#pragma unroll
      for (int j = 0; j < RN; ++j) Vec<R>::get(pb + j * GN * KP + 8 * (g * G + q), b[q][j]);
    }
  };
  auto fmas = [&](const float (&a)[G][RM][R], const float (&b)[G][RN][R]) {
#pragma unroll
    for (int q = 0; q < G; ++q)
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int e = 0; e < R; e += 2) {
            // residues R*s+e, R*s+e+1: one packed fma, each lane exact
            const f2 x = {a[q][i][e], a[q][i][e + 1]}, y = {b[q][j][e], b[q][j][e + 1]};
            f2 c = {acc[i][j][e], acc[i][j][e + 1]};
            c = __builtin_elementwise_fma(x, y, c);
            acc[i][j][e] = c.x;
            acc[i][j][e + 1] = c.y;
          }
  };
  auto compute = [&](const float* cur) {
    const float* pa = cur + gm * KP + R * s;
    const float* pb = cur + (TM + gn) * KP + R * s;
    float a0[G][RM][R], b0[G][RN][R], a1[G][RM][R], b1[G][RN][R];
    fetch(pa, pb, 0, a0, b0);
#pragma unroll
    for (int g = 0; g < NGR; g += 2) {
      if (g + 1 < NGR) fetch(pa, pb, g + 1, a1, b1);
      fmas(a0, b0);
      if (g + 2 < NGR) fetch(pa, pb, g + 2, a0, b0);
      if (g + 1 < NGR) fmas(a1, b1);
    }
  };

  const int nt = (int)((K + KC - 1) / KC);
  int t0 = 0;
  if constexpr (GL) {
    const int nf = (int)(K / KC);  // full chunks by DMA
#pragma unroll
    for (int c = 0; c < S - 1; ++c)
      if (c < nf) dma(c);
    for (int t = 0; t < nf; ++t) {
      if (t + S - 2 < nf)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((S - 2) * I) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // chunk t landed for every wave; stage
                                     // (t-1)%S no longer read by anyone
      if (t + S - 1 < nf) dma(t + S - 1);
      compute(lds + (t % S) * STAGE);
    }
    t0 = nf;
    if (t0 < nt) {  // ragged last chunk
      __syncthreads();
      stage_regs((int64_t)t0 * KC, lds + (t0 % S) * STAGE);
      __syncthreads();
      compute(lds + (t0 % S) * STAGE);
    }
  } else {
    for (int t = 0; t < nt; ++t) {
      __syncthreads();
      stage_regs((int64_t)t * KC, lds + (t & 1) * STAGE);
      __syncthreads();
      compute(lds + (t & 1) * STAGE);
    }
  }

  // fold the 8 residue chains of each output as sdot_avx2: s_l = l + l+4,
  // then (s0 + s1) + (s2 + s3); the partners live in the same lane (R = 8)
  // or in lanes of the same group (shuffles within LPO lanes)
  const float alpha = p.alpha, beta = p.beta;
  float* __restrict__ C = p.C + bz * p.strideC;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      float dot;
      const float* l = acc[i][j];
      if constexpr (R == 8) {
        dot = ((l[0] + l[4]) + (l[1] + l[5])) + ((l[2] + l[6]) + (l[3] + l[7]));
      } else if constexpr (R == 4) {
        // lane s=0: residues 0..3, s=1: 4..7
        float u[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) u[e] = l[e] + __shfl_down(l[e], 1, 2);
        dot = (u[0] + u[1]) + (u[2] + u[3]);
      } else {  // R == 2: lane s holds residues 2s, 2s+1
        // s_{2s} = l_{2s} + l_{2s+4} (lane s + lane s+2), same for 2s+1
        const float v0 = l[0] + __shfl_down(l[0], 2, 4);
        const float v1 = l[1] + __shfl_down(l[1], 2, 4);
        const float h = v0 + v1;  // lane 0: s0 + s1, lane 1: s2 + s3
        dot = h + __shfl_down(h, 1, 4);
      }
      const int64_t m = m0 + gm + GM * i, n = n0 + gn + GN * j;
      if (s != 0 || m >= M || n >= N) continue;
      const float sum = alpha * dot;
      float* cp = C + m * p.ldc + n;
      if (p.beta_mode == BETA_STORE) {
        *cp = sum;
        continue;
      }
      float c0;
      if (p.beta_mode == BETA_ZERO)
        c0 = 0.0f;
      else if (p.beta_mode == BETA_SCALE)
        c0 = beta * *cp;
      else
        c0 = *cp;
      *cp = c0 + sum;
    }
}

struct ChainsVariant {
  int nt, r, rm, rn, gm;
  hipError_t (*launch)(const GemmArgs&, bool, hipStream_t);
  const char* name;
};

template <int NT, int R, int RM, int RN, int GM>
hipError_t launch_chains(const GemmArgs& a, bool gl, hipStream_t s) {
  constexpr int NG = NT * R / 8, GN = NG / GM, TM = GM * RM, TN = GN * RN;
  const int64_t tm = (a.M + TM - 1) / TM, tn = (a.N + TN - 1) / TN;
  const int64_t per = 0x7fffffff / (tm * tn);  // images per launch (1-D grid)
  if (per < 1) return hipErrorInvalidValue;
  for (int64_t b0 = 0; b0 < a.batch; b0 += per) {
    GemmArgs sub = a;
    const int64_t nb = a.batch - b0 < per ? a.batch - b0 : per;
    sub.A = a.A + b0 * a.strideA;
    sub.B = a.B + b0 * a.strideB;
    sub.C = a.C + b0 * a.strideC;
    sub.batch = nb;
    const dim3 grid((unsigned)(tm * tn * nb));
    if (gl)
      hipLaunchKernelGGL((sdot_chains_kernel<NT, R, RM, RN, GM, true>), grid, dim3(NT), 0, s, sub,
                         (int)tm, (int)(tm * tn));
    else
      hipLaunchKernelGGL((sdot_chains_kernel<NT, R, RM, RN, GM, false>), grid, dim3(NT), 0, s,
                         sub, (int)tm, (int)(tm * tn));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

#define TNS_CHAINS(NT, R, RM, RN, GM)                                                   \
  {NT, R, RM, RN, GM, launch_chains<NT, R, RM, RN, GM>,                                \
   "chains<nt" #NT ",r" #R "," #RM "x" #RN ",gm" #GM ">"}
const ChainsVariant kChains[] = {
    TNS_CHAINS(64, 2, 1, 1, 4),    // 0: tile 4x4
    TNS_CHAINS(128, 2, 1, 1, 8),   // 1: tile 8x4
    TNS_CHAINS(256, 2, 1, 1, 8),   // 2: tile 8x8
    TNS_CHAINS(64, 2, 2, 2, 4),    // 3: tile 8x8
    TNS_CHAINS(256, 2, 2, 2, 8),   // 4: tile 16x16
    TNS_CHAINS(128, 4, 2, 2, 8),   // 5: tile 16x16
    TNS_CHAINS(256, 4, 2, 2, 8),   // 6: tile 16x32
    TNS_CHAINS(256, 8, 2, 2, 16),  // 7: tile 32x32 (in-lane fold)
    TNS_CHAINS(256, 2, 4, 4, 8),   // 8: tile 32x32
};
#undef TNS_CHAINS
constexpr int kChainsCount = sizeof(kChains) / sizeof(kChains[0]);

bool chains_vec4(const float* p, int64_t ld, int64_t stride, int64_t batch, int64_t K) {
  if ((reinterpret_cast<uintptr_t>(p) & 15) != 0) return false;
  if (ld % 4 != 0 || K % 4 != 0) return false;
  return batch <= 1 || stride % 4 == 0;
}

}  // namespace

int sdot_chains_variant_count() { return kChainsCount; }
const char* sdot_chains_variant_name(int v) {
  return v >= 0 && v < kChainsCount ? kChains[v].name : "";
}

hipError_t launch_sdot_chains(const GemmArgs& a, int variant, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0 || a.batch <= 0) return hipSuccess;
  if (variant < 0 || variant >= kChainsCount) return hipErrorInvalidValue;
  const bool gl = chains_vec4(a.A, a.lda, a.strideA, a.batch, a.K) &&
                  chains_vec4(a.B, a.ldb, a.strideB, a.batch, a.K);
  return kChains[variant].launch(a, gl, s);
}

}  // namespace tns
