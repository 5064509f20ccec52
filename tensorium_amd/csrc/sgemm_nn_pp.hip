// sgemm_nn_pp.hip — large aligned gemm(NoTrans, NoTrans), ping-pong form.
//
// Same tile and arithmetic as sgemm_nn_big.hip (256 x 256 block, 8 waves of
// 128 x 64 = 4 x 2 v_mfma_f32_32x32x2_f32 accumulators, k-tiles of 32, two
// LDS stages, B by LDS-DMA, A transposed through registers into the permuted
// k-major image), so bit-identical to it and to the reference's s_nn chain
// (ntensors.pas:2061-2157: every C element an ascending-k fma chain from
// beta*C, A_PART = ALPHA*A rounded once).  What changes is the schedule.
//
// The 8 waves form two groups of 4, one wave of each group per SIMD (waves
// i and i + 4 share a SIMD): group 0 owns block rows 0..127, group 1 rows
// 128..255.  Each k-tile runs in two phases separated by a barrier; in each
// phase one group computes (128 MFMAs per wave, fragment reads one step
// ahead) while the other stages half of the NEXT k-tile:
//
//   phase A:  group 0 computes tile t     group 1 stages k 0..15 of tile t+1
//                                          and reads its step-0 fragments of t
//   phase B:  group 1 computes tile t     group 0 stages k 16..31 of tile t+1
//                                          and reads its step-0 fragments of
//                                          t+1 (k 0..1: staged in phase A)
//
// so every SIMD's matrix pipe always has one wave with MFMAs to issue: the
// staging (global loads, the transposing ds_writes, the B DMA), the barrier
// wait and the first fragment reads of a phase sit under the partner's
// MFMAs instead of stalling both waves of a SIMD at once, as the lock-step
// schedule does at every k-tile (0.87 -> target >= 0.92 of peak).
// Two stages suffice: in phase A of tile t group 1 writes stage (t+1)&1,
// which both groups finished reading in tile t-1.
#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BM = 256, BN = 256, BK = 32, NT = 512;
constexpr int WTM = 128, WTN = 64, TM = 4, TN = 2;  // wave tile, 32x32 accumulators
constexpr int LDA = BM, LDB = BN;                     // k-major LDS rows
constexpr int A_TILE = BK * LDA, B_TILE = BK * LDB, STAGE = A_TILE + B_TILE;

// BP: B register-staged into a k-permuted slot image instead of the row
// image by LDS-DMA: slot (g, h, column) holds the four k = 8g + h + 2i
// (i = 0..3) a lane consumes over MFMA steps 4g..4g+3, so a wave reads its
// two B fragments once per four steps (two ds_read_b128) instead of two
// ds_read_b32 per step (the bare loop: 0.923 -> see scripts/mfma_probe.hip
// m32_lds4); a group thread owns one column of the half's 16 k-rows (16
// coalesced dword loads, four ds_write_b128)
template <bool BP>
__global__ __launch_bounds__(NT, 1) void sgemm_nn_pp_kernel(GemmArgs p) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches
  const int lc = lane & 31, h = lane >> 5;
  const int g = wid >> 2, wq = wid & 3;  // group (= block-row half), wave in group
  const int tg = tid & 255;              // thread index in the group
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  // XCD-contiguous grouped raster (as sgemm_nn_big.hip)
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
  const int64_t row_base = m0 + g * WTM + 4 * h;
  const int64_t col_base = n0 + wq * WTN + lc;
  if (p.beta_mode == BETA_ZERO) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
  } else {
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
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(acc[i][j]));

  // ---- staging of one k-half (16 k) of a tile by one group ----------------
  // A: unit u of this thread = k-quad kq (of the half), permuted row mm; LDS
  // column of row m as sgemm_nn_big.hip (a lane's four 32-row fragments in
  // one 16-byte slot), XOR-swizzled by (k-quad & 3) << 3: a 32-lane store
  // group covers 8 consecutive columns x 4 k-quads -> 32 distinct banks.
  constexpr int AU = 4;
  const float* a_src[AU];
  int a_dst[AU];
#pragma unroll
  for (int u = 0; u < AU; ++u) {
    const int idx = tg + 256 * u;
    const int kq = idx & 3, mm = idx >> 2;
    const int m = (mm & ~(WTM - 1)) | ((mm % TM) << 5) | ((mm & (WTM - 1)) / TM);
    a_src[u] = A + (m0 + m) * lda + 4 * kq;
    a_dst[u] = (4 * kq) * LDA + (mm ^ (kq << 3));  // + half*16*LDA; element c adds c*LDA
  }
  const float alpha = p.alpha;
  // B: wave wq of the group moves k-rows 16*half + 4*wq + r (one 1 KB row
  // per global_load_lds_dwordx4 wave-instruction)
  const float* b_src = B + (int64_t)(4 * wq) * ldb + n0 + 4 * lane;
  const unsigned b_lds0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)(smem + A_TILE +
                                                                      4 * wq * LDB));
  // issue: the half's B DMA (straight into LDS) and A loads (into ra);
  // finish: wait for both, scale A, transposing ds_writes.  Both run in the
  // group's memory phase.  (Issued a phase earlier instead — loads carried in
  // registers across the partner's compute phase, the DMA into rows the group
  // had finished reading — hipcc copies the loop-carried registers right
  // after the loads and waits on them there: 4096^3 0.972 -> 1.137 ms.)
  float4 ra[AU];
  float rbp[BP ? 16 : 1];
  // (BP) buffer loads: the column in the VGPR offset, the row in the
  // uniform SGPR offset (no 64-bit address registers per row)
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(B), 0, BP ? 0x7fffffff : 0, 0x00020000);
  const unsigned b_voff = 4u * (unsigned)(n0 + tg);
  auto issue_half = [&](int64_t k0, int st, int half) {
    if constexpr (BP) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const unsigned so = __builtin_amdgcn_readfirstlane((unsigned)((k0 + 16 * half + r) * ldb * 4));
        rbp[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(brs, b_voff, so, 0));
      }
    } else {
#ifndef TNS_PP_NO_B  // (diagnostic builds: timing without this part, wrong results)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      unsigned keep;
      const float* src = b_src + (k0 + 16 * half + r) * ldb;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(src), "s"(b_lds0 + (unsigned)((st * STAGE + (16 * half + r) * LDB) * 4))
          : "memory");
    }
#endif
    }
#ifndef TNS_PP_NO_A
#pragma unroll
    for (int u = 0; u < AU; ++u)
      if constexpr (BP)  // unit u = unit 0 shifted by rows {0, 16, 128, 144}[u] (fewer live registers)
        ra[u] = *reinterpret_cast<const float4*>(a_src[0] + (int64_t)((u & 1) * 16 + (u >> 1) * 128) * lda + k0 + 16 * half);
      else
        ra[u] = *reinterpret_cast<const float4*>(a_src[u] + k0 + 16 * half);
#endif
  };
  auto finish_half = [&](int st, int half) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // A loads and B DMA landed
    if constexpr (BP) {
      float* bs = smem + st * STAGE + A_TILE;
#pragma unroll
      for (int gl = 0; gl < 2; ++gl)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
          *reinterpret_cast<float4*>(bs + (((2 * half + gl) * 2 + hh) * BN + tg) * 4) =
              make_float4(rbp[8 * gl + hh], rbp[8 * gl + hh + 2], rbp[8 * gl + hh + 4],
                          rbp[8 * gl + hh + 6]);
    }
#ifndef TNS_PP_NO_A
    float* as = smem + st * STAGE + 16 * half * LDA;
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      float4 v = ra[u];  // A_PART = ALPHA*A[kk] (1*x == x bit for bit)
      v.x = alpha * v.x; v.y = alpha * v.y; v.z = alpha * v.z; v.w = alpha * v.w;
      const int d = BP ? a_dst[0] + 64 * u : a_dst[u];  // (mm + 64u) ^ x = (mm ^ x) + 64u
      as[d] = v.x;
      as[d + LDA] = v.y;
      as[d + 2 * LDA] = v.z;
      as[d + 3 * LDA] = v.w;
    }
#endif
  };

  // ---- fragments: step s of a k-tile consumes k = 2s + h ------------------
  const int a_frag = g * WTM + TM * lc;  // 4 floats: rows lc + 32i of the wave tile
  const int b_frag = wq * WTN + lc;      // rows lc + 32j
  auto frag = [&](const float* st, int s, float (&a)[TM], float (&b)[TN]) {
    const int k = 2 * s + h;
    const float* ap = st + k * LDA + (a_frag ^ (((k >> 2) & 3) << 3));
    const float4 v = *reinterpret_cast<const float4*>(ap);
    a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
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
  float a0[TM], b0[TN];
  // (BP) the B slots of four steps: bq[j] = column b_frag + 32j of group g
  float4 bq0[TN];
  auto fragA = [&](const float* st, int s, float (&a)[TM]) {
    const int k = 2 * s + h;
    const float4 v = *reinterpret_cast<const float4*>(st + k * LDA + (a_frag ^ (((k >> 2) & 3) << 3)));
    a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
  };
  auto fragBq = [&](const float* st, int g4, float4 (&bq)[TN]) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bq[j] = *reinterpret_cast<const float4*>(st + A_TILE + ((g4 * 2 + h) * BN + b_frag + 32 * j) * 4);
  };
  // step-0 fragments of a stage into a0 / b0 (or a0 / bq0)
  auto frag0 = [&](const float* st) {
    if constexpr (BP) {
      fragA(st, 0, a0);
      fragBq(st, 0, bq0);
    } else {
      frag(st, 0, a0, b0);
    }
  };
  // one k-tile of this wave's MFMAs from stage cur, step 0's fragments
  // already in a0/b0
  auto compute = [&](const float* cur) {
    if constexpr (BP) {
      float a1[TM];
      float4 bq1[TN];
#pragma unroll
      for (int g4 = 0; g4 < BK / 8; ++g4) {
        float4 (&bc)[TN] = (g4 & 1) ? bq1 : bq0;
        float4 (&bn)[TN] = (g4 & 1) ? bq0 : bq1;
#pragma unroll
        for (int c = 0; c < 4; c += 2) {
          const int s = 4 * g4 + c;
          fragA(cur, s + 1, a1);
          if (c == 0 && g4 + 1 < BK / 8) fragBq(cur, g4 + 1, bn);
          __builtin_amdgcn_sched_barrier(0);
          {
            const float bb[TN] = {bc[0][c], bc[1][c]};
            mma(a0, bb);
          }
          if (s + 2 < BK / 2) fragA(cur, s + 2, a0);
          __builtin_amdgcn_sched_barrier(0);
          {
            const float bb[TN] = {bc[0][c + 1], bc[1][c + 1]};
            mma(a1, bb);
          }
        }
      }
    } else {
      float a1[TM], b1[TN];
#pragma unroll
      for (int s = 0; s < BK / 2; s += 2) {
        frag(cur, s + 1, a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, b0);
        if (s + 2 < BK / 2) frag(cur, s + 2, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1);
      }
    }
  };

  // Staging jobs: group 1 fills k 0..15 of tile t+1 in phase A(t), group 0
  // k 16..31 in phase B(t); every job's rows were last read in tile t-1.
  const int nt = (int)(p.K / BK);
  if (nt > 0) {
    issue_half(0, 0, 1 - g);  // group 1: k 0..15, group 0: k 16..31
    finish_half(0, 1 - g);
    __syncthreads();
    if (g == 0) frag0(smem);
  }
  for (int t = 0; t < nt; ++t) {
    const float* cur = smem + (t & 1) * STAGE;
    const int nxt = (t + 1) & 1;
    const bool more = t + 1 < nt;
    // phase A
    if (g == 0) {
      compute(cur);
    } else {
      if (more) {
        issue_half((int64_t)(t + 1) * BK, nxt, 0);
        finish_half(nxt, 0);
      }
      frag0(cur);
    }
    __syncthreads();
    // phase B
    if (g == 1) {
      compute(cur);
    } else if (more) {
      issue_half((int64_t)(t + 1) * BK, nxt, 1);
      finish_half(nxt, 1);
      frag0(smem + nxt * STAGE);  // k 0..1 (BP: 0..7) of tile t+1: staged in phase A
    }
    if (more) __syncthreads();
  }

  // ---- epilogue (group 0 stores while group 1 computes the last tile) ----
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t row = row_base + 32 * i + (e & 3) + 8 * (e >> 2);
#pragma unroll
      for (int j = 0; j < TN; ++j) C[row * ldc + col_base + 32 * j] = acc[i][j][e];
    }
}

bool aligned16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

}  // namespace

bool sgemm_nn_pp_applies(const GemmArgs& a) {
  if (a.conv || a.epi != EPI_NONE || a.beta_mode == BETA_STORE) return false;
  if (a.M % BM || a.N % BN || a.K % BK || a.M <= 0 || a.N <= 0) return false;
  if (a.lda % 4 || a.ldb % 4 || !aligned16(a.A) || !aligned16(a.B)) return false;
  if (a.batch > 1 && (a.strideA % 4 || a.strideB % 4)) return false;
  return (a.M / BM) * (a.N / BN) <= 0x7fffffff;
}

hipError_t launch_sgemm_nn_pp(const GemmArgs& a, hipStream_t s, bool bperm) {
  if (!sgemm_nn_pp_applies(a)) return hipErrorInvalidValue;
  // (k-permuted B form: one buffer resource over each B, 31-bit byte offsets)
  if (bperm && (a.K * a.ldb + a.N) * 4 > 0x7fffffffLL) return hipErrorInvalidValue;
  const int64_t tiles = (a.M / BM) * (a.N / BN);
  for (int64_t b0 = 0; b0 < a.batch; b0 += 65535) {
    GemmArgs sub = a;
    const int64_t nb = a.batch - b0 < 65535 ? a.batch - b0 : 65535;
    sub.A = a.A + b0 * a.strideA;
    sub.B = a.B + b0 * a.strideB;
    sub.C = a.C + b0 * a.strideC;
    sub.batch = nb;
#ifdef TNS_DIAG_KERNELS  // (the k-permuted B form: diagnostics build only)
    if (bperm)
      hipLaunchKernelGGL(sgemm_nn_pp_kernel<true>, dim3((unsigned)tiles, (unsigned)nb), dim3(NT), 0,
                         s, sub);
    else
#else
    if (bperm) return hipErrorInvalidValue;
#endif
      hipLaunchKernelGGL(sgemm_nn_pp_kernel<false>, dim3((unsigned)tiles, (unsigned)nb), dim3(NT),
                         0, s, sub);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace tns
