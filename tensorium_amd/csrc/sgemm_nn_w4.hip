// sgemm_nn_w4.hip — large aligned gemm(NoTrans, NoTrans), one wave per SIMD.
//
// The 256 x 256 x 32 block of sgemm_nn_big.hip / sgemm_nn_pp.hip with the
// same arithmetic (the reference's cblas_sgemm -> s_nn over saxpy_avx2,
// ntensors.pas:2061-2157, 2231-2286: every C element an ascending-k fma chain
// from beta*C, A_PART = ALPHA*A rounded once; v_mfma_f32_32x32x2_f32 step s
// consumes k = 2s + h, lane half h), so bit-identical to them; the block is
// laid out for one wave per SIMD instead of two:
//
//   * 4 waves (2 x 2), wave tile 128 x 128 = 4 x 4 accumulators of 32 x 32
//     (256 accumulator registers per lane: the wave has the SIMD's whole
//     register file to itself), so a step is 16 MFMAs = 1024 matrix-pipe
//     cycles fed by 8 ds_read_b32 — no partner wave's staging on the SIMD;
//   * BOTH operands stream global -> LDS by LDS-DMA (global_load_lds_dwordx4,
//     SGPR base + one per-lane VGPR offset for the whole launch): no staging
//     registers, no VALU transposes, no ds_write;
//   * A lands as row images [m][32 k] whose 16-byte k-chunks are XOR-swizzled
//     by row on the source side (chunk slot = chunk ^ ((m >> 1) & 7)), B as
//     [k][256 n] rows rotated by 32 floats on odd k: both fragment reads are
//     conflict-free or 2-way (A: lanes m and m + 16 share a bank);
//   * two LDS stages (2 x 64 KB); the barrier that publishes tile t+1 sits
//     before tile t's last step, whose 16 MFMAs each carry one of the 16 DMA
//     instructions of tile t+2 (into tile t's stage): the DMA goes out a whole
//     tile ahead of its use; fragments of step s+1 are read before step s's
//     MFMAs (scheduling fences);
//   * interleaved columns: accumulator tile j's column lc is block column
//     wn*128 + 4 lc + j (not 32 j + lc), so a lane's four B fragments of a
//     step are one ds_read_b128 and its four tiles' values of one row are 4
//     consecutive columns of C: beta loads and epilogue stores move 16 bytes
//     per lane.
//
// Measured at 4096^3 (scripts/nn_big_ab.py, profiles/r04_sgemm_w4_ab.json): 0.950 ms
// vs 0.983 for the ping-pong form on the same box, bit-identical.  (The
// forms with 32 j + lc columns and 4-byte B reads, with the DMA issued as one
// burst, measured 0.988-0.992 ms and did not reproduce the ping-pong bits at
// 4096^3; dropped.)
//
// alpha != 1 multiplies the A fragments after the read (one rounding, as the
// reference's A_PART = ALPHA*A[kk]).
#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef int int4v __attribute__((ext_vector_type(4)));

constexpr int BM = 256, BN = 256, BK = 32, NT = 256;
constexpr int A_TILE = BM * BK, B_TILE = BK * BN, STAGE = A_TILE + B_TILE;  // floats

__device__ __forceinline__ void dma16(const float* sbase, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

template <bool ALPHA1>
__global__ __launch_bounds__(NT, 1) void sgemm_nn_w4_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lc = lane & 31, h = lane >> 5;
  const int wm = wid >> 1, wn = wid & 1;

  // XCD-contiguous grouped raster (as sgemm_nn_big.hip)
  const int tiles_m = (int)(p.M / BM), tiles_n = (int)(p.N / BN);
  int tm, tn;
  const int64_t bz = blockIdx.y;
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
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const float* __restrict__ A = p.A + bz * p.strideA;
  const float* __restrict__ B = p.B + bz * p.strideB;
  float* __restrict__ C = p.C + bz * p.strideC;
  const int64_t lda = p.lda, ldb = p.ldb, ldc = p.ldc;

  // ---- LDS-DMA staging: wave w moves A row groups 8q..8q+7 (q = 8w + u,
  // u < 8: 1 KB each) and B k-rows r = 8w + u of a tile ----------------------
  // A: lane i -> row 8q + (i >> 3), LDS chunk slot i & 7 <- k-chunk
  //    (i & 7) ^ ((row >> 1) & 7)
  // B: lane i -> LDS chunk i of row r <- n-chunk (i + 8 (r & 1)) & 63
  const int arow = lane >> 3;  // row within the group (group rows are 8-aligned)
  const unsigned a_voff = (unsigned)(arow * lda * 4) + 16u * (unsigned)((lane & 7) ^ ((arow >> 1) & 7));
  // ((8q + arow) >> 1) & 7 = (4q + (arow >> 1)) & 7: q even -> (arow >> 1),
  // q odd -> (arow >> 1) ^ 4; odd groups use the second offset
  const unsigned a_voff1 = (unsigned)(arow * lda * 4) +
                           16u * (unsigned)((lane & 7) ^ (((arow >> 1) & 7) ^ 4));
  const unsigned b_voff0 = 16u * (unsigned)lane;
  const unsigned b_voff1 = 16u * (unsigned)((lane + 8) & 63);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)smem;
  const float* a_row0 = A + m0 * lda;  // + (8q) * lda + k0
  const float* b_row0 = B + n0;        // + (k0 + r) * ldb
  // DMA instruction u (0..15) of this wave for tile k0 into stage st
  auto issue1 = [&](int u, int64_t k0, int st) {
    const unsigned sb = lds0 + (unsigned)(st * STAGE * 4);
    if (u < 8) {
      const int q = 8 * wid + u;
      dma16(a_row0 + (int64_t)(8 * q) * lda + k0, (u & 1) ? a_voff1 : a_voff,
            sb + (unsigned)(q * 1024));
    } else {
      const int r = 8 * wid + (u - 8);
      dma16(b_row0 + (k0 + r) * ldb, (u & 1) ? b_voff1 : b_voff0,
            sb + (unsigned)(A_TILE * 4 + r * 1024));
    }
  };
  auto issue = [&](int64_t k0, int st) {
    const unsigned sb = lds0 + (unsigned)(st * STAGE * 4);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int q = 8 * wid + u;
      dma16(a_row0 + (int64_t)(8 * q) * lda + k0, (u & 1) ? a_voff1 : a_voff,
            sb + (unsigned)(q * 1024));
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = 8 * wid + u;
      dma16(b_row0 + (k0 + r) * ldb, (u & 1) ? b_voff1 : b_voff0,
            sb + (unsigned)(A_TILE * 4 + r * 1024));
    }
  };

  // the first two tiles' DMA goes out before the beta*C loads, so the two
  // latencies overlap (the C loads are younger: waiting for them waits for
  // the DMA too)
  const int nt = (int)(p.K / BK);
#ifdef TNS_W4_DMA_LATE  // (A/B side builds: round 4's order, DMA after the C loads)
  constexpr bool kDmaFirst = false;
#else
  constexpr bool kDmaFirst = true;
#endif
  if (kDmaFirst && nt > 0) issue(0, 0);
  if (kDmaFirst && nt > 1) issue(BK, 1);

  // ---- accumulators: 0, C or beta*C ---------------------------------------
  // C through a buffer resource over this block's rows: the lane's column in
  // a 32-bit VGPR offset, the row (wave-uniform: i, e) in the SGPR offset,
  // the column tile j in the instruction offset — no 64-bit row addresses
  // held across the loop
  floatx16 acc[4][4];
  const int64_t row_base = m0 + wm * 128;
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
      C + row_base * ldc, 0, 0x7fffffff, 0x00020000);
  const unsigned c_voff = 4u * (unsigned)(4 * h * ldc + n0 + wn * 128 + 4 * lc);
  auto c_soff = [&](int i, int e) {
    return (unsigned)(4 * (32 * i + (e & 3) + 8 * (e >> 2)) * ldc);
  };
  if (p.beta_mode == BETA_ZERO) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
  } else {
    // tile (i, j) = g: its 16 loads in flight while tile g-1 is moved into
    // its accumulator registers
    const bool scale = p.beta_mode == BETA_SCALE;
    const float beta = p.beta;
    {
      // row group g = (i, e-block of 4): 4 float4 loads = tiles 0..3 of 4 rows
      floatx4 v[2][4];
      auto ldv = [&](int g, floatx4 (&t)[4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          t[u] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 crs, c_voff, c_soff(g >> 2, 4 * (g & 3) + u), 0));
      };
      ldv(0, v[0]);
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        if (g + 1 < 16) ldv(g + 1, v[(g + 1) & 1]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float c = v[g & 1][u][j];
            acc[g >> 2][j][4 * (g & 3) + u] = scale ? beta * c : c;
          }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[i][j]));
  if (!kDmaFirst && nt > 0) issue(0, 0);
  if (!kDmaFirst && nt > 1) issue(BK, 1);

  // ---- fragments: step s (k = 2s + h) --------------------------------------
  // A tile i: row wm*128 + 32 i + lc, chunk (k >> 2) ^ swz, swz = (lc >> 1) & 7
  // B tile j: n = wn*128 + 32 j + lc at LDS column (n - 32 h) & 255 of row k
  const int swz = (lc >> 1) & 7;
  int b_col[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    b_col[j] = A_TILE + h * BN + ((wn * 128 + 4 * lc + j - 32 * h) & 255);
  const float alpha = p.alpha;
  auto mma = [&](const float (&a)[4], const float (&b)[4]) {
    float aa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) aa[i] = ALPHA1 ? a[i] : alpha * a[i];  // A_PART = ALPHA*A
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(aa[i], b[j], acc[i][j], 0, 0, 0);
  };
  // a step's 16 MFMAs with the 16 DMA instructions of tile k0 issued
  // one after each: the DMA issue (SALU + VMEM) fills the 64-cycle gaps the
  // matrix pipe leaves between this wave's MFMAs instead of delaying them
  auto mma_dma = [&](const float (&a)[4], const float (&b)[4], int64_t k0, int st, bool dma) {
    float aa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) aa[i] = ALPHA1 ? a[i] : alpha * a[i];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = u >> 2, j = u & 3;
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(aa[i], b[j], acc[i][j], 0, 0, 0);
      if (dma) issue1(u, k0, st);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const int a_lane = (wm * 128 + lc) * BK + h;
  auto frag = [&](const float* st, int s, float (&a)[4], float (&b)[4]) {
    const int ka = 4 * ((s >> 1) ^ swz) + 2 * (s & 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = st[a_lane + 32 * BK * i + ka];
    const floatx4 v = *reinterpret_cast<const floatx4*>(st + b_col[0] + 2 * s * BN);
    b[0] = v[0]; b[1] = v[1]; b[2] = v[2]; b[3] = v[3];
  };
  float a0[4], b0[4], a1[4], b1[4];
  {
    // the barrier that publishes tile t+1 sits before step 15 of tile
    // t, so tile t+1's first fragments are read under step 15's MFMAs and the
    // DMA of tile t+2 (into tile t's stage, whose reads all completed before
    // the barrier) goes out a whole tile ahead of its use
    if (nt > 0) {
      if (nt > 1) {
        // tile 0's 16 DMAs of this wave (with beta*C loaded: all of them)
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      frag(smem, 0, a0, b0);
    }
    for (int t = 0; t < nt; ++t) {
      const float* cur = smem + (t & 1) * STAGE;
      const float* nxt = smem + ((t + 1) & 1) * STAGE;
#pragma unroll
      for (int s = 0; s < BK / 2 - 2; s += 2) {  // steps 0 .. 13
        frag(cur, s + 1, a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, b0);
        frag(cur, s + 2, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1);
      }
      frag(cur, BK / 2 - 1, a1, b1);  // step 15's fragments
      __builtin_amdgcn_sched_barrier(0);
      mma(a0, b0);                     // step 14
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 < nt) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile t+1
        __syncthreads();  // every wave's; every read of tile t complete
        frag(nxt, 0, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
      }
      mma_dma(a1, b1, (int64_t)(t + 2) * BK, t & 1, t + 2 < nt);  // step 15 + tile t+2's DMA
    }
  }

  // ---- epilogue ----------------------------------------------------------------
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const floatx4 v = {acc[i][0][e], acc[i][1][e], acc[i][2][e], acc[i][3][e]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(int4v, v), crs, c_voff,
                                             c_soff(i, e), 0);
    }
}

bool aligned16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

}  // namespace

bool sgemm_nn_w4_applies(const GemmArgs& a) {
  if (a.conv || a.epi != EPI_NONE || a.beta_mode == BETA_STORE) return false;
  if (a.M % BM || a.N % BN || a.K % BK || a.M <= 0 || a.N <= 0) return false;
  if (a.lda % 4 || a.ldb % 4 || !aligned16(a.A) || !aligned16(a.B)) return false;
  if (a.batch > 1 && (a.strideA % 4 || a.strideB % 4)) return false;
  // (32-bit byte offsets: 7 rows of A per DMA lane offset, a block's 256
  // rows of C from its first row)
  if (a.lda * 4 * 8 > 0x7fffffffLL || (256 * a.ldc + a.N) * 4 > 0x7fffffffLL) return false;
  return (a.M / BM) * (a.N / BN) <= 0x7fffffff;
}

hipError_t launch_sgemm_nn_w4(const GemmArgs& a, hipStream_t s) {
  if (!sgemm_nn_w4_applies(a)) return hipErrorInvalidValue;
  const int64_t tiles = (a.M / BM) * (a.N / BN);
  const bool alpha1 = a.alpha == 1.0f;
  for (int64_t b0 = 0; b0 < a.batch; b0 += 65535) {
    GemmArgs sub = a;
    const int64_t nb = a.batch - b0 < 65535 ? a.batch - b0 : 65535;
    sub.A = a.A + b0 * a.strideA;
    sub.B = a.B + b0 * a.strideB;
    sub.C = a.C + b0 * a.strideC;
    sub.batch = nb;
    const dim3 grid((unsigned)tiles, (unsigned)nb);
    if (alpha1)
      hipLaunchKernelGGL((sgemm_nn_w4_kernel<true>), grid, dim3(NT), 0, s, sub);
    else
      hipLaunchKernelGGL((sgemm_nn_w4_kernel<false>), grid, dim3(NT), 0, s, sub);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace tns
