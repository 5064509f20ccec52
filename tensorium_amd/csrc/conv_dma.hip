// conv_dma.hip — implicit-GEMM convolution fed by an LDS-DMA ring
// (TConvolutionalLayer.forward → Conv2D + forwardBias + activate after
// fuseBatchNorm: nConvolutionLayer.pas:457-569, ntensors.pas:8252-8349; the
// im2col column order of sim2Col, 11415-11532).
//
// Same arithmetic as conv_tile.hip / the ConvBIO path of sgemm_kernel.hpp:
// each output an ascending-k fma chain over k = (c, kr, kc) from +0 through
// the v_mfma_f32_16x16x4_f32 lane-quarter order (lane quarter q = the q-th k
// of a step), then bias add and activation, each rounded once — so
// bit-identical to sim2Col + the reference GEMM.  What changes is how the
// operands reach LDS: no staging registers, no ds_write, no transposes.
//
//   * B (the im2col matrix, never materialised) is GATHERED straight into
//     LDS by dword LDS-DMA (buffer_load_dword ... lds): one wave-instruction
//     writes 64 consecutive pixels of one k-row of the tile, each lane
//     sourcing its pixel's tap of that k from the unpadded image; taps
//     outside the window get an out-of-range offset and land as 0 (the
//     buffer resource's range check).  k is uniform per instruction, so the
//     (c, kr, kc) walk is scalar.
//   * A (weights, k-contiguous rows) arrives by 16-byte LDS-DMA
//     (global_load_lds_dwordx4): 16-byte slots of 4 consecutive k of a row,
//     the slot index XOR-swizzled by row so a step's A fragment reads
//     (16 rows x 2 lane quarters per 32-lane group) are at worst 2-way.
//   * a 3-stage LDS ring: tile t+2 is issued at the top of tile t, so every
//     gather has two tiles of MFMAs to land in; one raw barrier per tile
//     after a counted vmcnt (a __syncthreads() would drain the ring).
//   * WM x WN waves, wave tile 16 rows x BN/WN columns (J 16x16 MFMA
//     accumulators), fragments read one step ahead.
#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
// Measured and not picked (profiles/): compiled only into the
// diagnostics build (TNS_DIAG=1 python -m tensorium_amd.build); the default
// library reports no forms of this family.
#ifdef TNS_DIAG_KERNELS

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32, NT = 512, NSTAGE = 3;

template <int BM_, int BN_>
struct DGeo {
  static constexpr int BM = BM_, BN = BN_;
  static constexpr int WM = BM / 16, WN = 8 / WM;  // waves: 16-row strips x column groups
  static constexpr int WTN = BN / WN, J = WTN / 16;
  static constexpr int SEG = (BN + 63) / 64;          // 64-pixel DMA segments per B row
  static constexpr int LDB = SEG * 64 + 16;           // rows k and k+1 16 banks apart
  static constexpr int A_FL = BM * BK;                // A floats per stage (slots of 4)
  static constexpr int STAGE = A_FL + BK * LDB;       // floats
  static constexpr int ADMA = A_FL / 4 / 64 / 8;      // A DMA wave-instructions per wave
  static constexpr int BROWS = BK / 8;                // B k-rows per wave
  static constexpr int BDMA = BROWS * SEG;            // B DMA wave-instructions per wave
  static constexpr int NDMA = ADMA + BDMA;
  static_assert(WM * WN == 8 && BN % (16 * WN) == 0 && ADMA >= 1, "geometry");
  static_assert(NSTAGE * STAGE * 4 <= 160 * 1024, "LDS");
};

template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
#ifdef TNS_CD_NO_BAR  // (diagnostic builds)
  asm volatile("" ::: "memory");
#else
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
#endif
}

template <class G, int KS>
__global__ __launch_bounds__(NT, 1) void conv_dma_kernel(GemmArgs p, int dil) {
  constexpr int BM = G::BM, BN = G::BN, WN = G::WN, WTN = G::WTN, J = G::J, SEG = G::SEG;
  constexpr int LDB = G::LDB, A_FL = G::A_FL, STAGE = G::STAGE, ADMA = G::ADMA;
  constexpr int BROWS = G::BROWS, NDMA = G::NDMA;
  __shared__ __attribute__((aligned(16))) float smem[NSTAGE * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;
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
  const unsigned lds0 =
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)smem;  // byte address

  // ---- B gather state: this lane's pixel in each 64-pixel segment --------
  unsigned vbase[SEG];
  int ir0[SEG], ic0[SEG];
#pragma unroll
  for (int c = 0; c < SEG; ++c) {
    int n = n0 + 64 * c + lane;
    n = n < N ? n : N - 1;  // past N (or past the tile's BN): any valid pixel, never used
    const int img = n / p.conv_ohw, pix = n - img * p.conv_ohw;
    const int orow = pix / p.conv_ow, ocol = pix - orow * p.conv_ow;
    ir0[c] = orow * p.conv_sY - p.conv_pH;
    ic0[c] = ocol * p.conv_sX - p.conv_pW;
    vbase[c] = 4u * (unsigned)(img * (int)p.strideB + ir0[c] * W + ic0[c]);
  }
  const __amdgpu_buffer_rsrc_t brsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.B), 0, p.conv_bytes, 0x00020000);
  // wave wid gathers k-rows BROWS*wid .. +BROWS-1 of every tile: (c, kr, kc)
  // of each, wave-uniform, advanced by BK per tile
  int bc[BROWS], bkr[BROWS], bkc[BROWS];
#pragma unroll
  for (int r = 0; r < BROWS; ++r) {
    const int k = BROWS * wid + r;
    bc[r] = k / (KS * KS);
    const int rem = k - bc[r] * KS * KS;
    bkr[r] = rem / KS;
    bkc[r] = rem - bkr[r] * KS;
  }
  auto advance = [&]() {  // k += BK on every row
#pragma unroll
    for (int r = 0; r < BROWS; ++r) {
      if constexpr (KS == 1) {
        bc[r] += BK;
      } else {
        constexpr int DC = BK / (KS * KS), DR = BK % (KS * KS);
        int rem = bkr[r] * KS + bkc[r] + DR;
        int c = bc[r] + DC;
        if (rem >= KS * KS) { rem -= KS * KS; ++c; }
        bc[r] = c;
        bkr[r] = rem >= 2 * KS ? 2 : (rem >= KS ? 1 : 0);
        bkc[r] = rem - bkr[r] * KS;
      }
    }
  };

  // ---- A DMA sources: slot s of wave-instruction i holds 4 k of one row ---
  const float* a_src[ADMA];
#pragma unroll
  for (int i = 0; i < ADMA; ++i) {
    const int slot = 64 * (ADMA * wid + i) + lane;
    const int row = slot >> 3, kq = (slot & 7) ^ (row & 7);
    a_src[i] = p.A + (m0 + row) * p.lda + 4 * kq;
  }

  // ---- this wave's DMAs of a tile: index 0..ADMA-1 the A slots, then the
  // B rows r x segments c; dma(i, st) issues one of them for the tile whose
  // k-state is current into stage st
  int cur_tile = 0;
  auto dma = [&](int i, int st) {
#ifdef TNS_CD_NO_DMA  // (diagnostic builds: timing without the staging, wrong results)
    return;
#endif
    const unsigned sbase = lds0 + (unsigned)(st * STAGE) * 4u;
#ifdef TNS_CD_NO_A
    if (i < ADMA) return;
#endif
#ifdef TNS_CD_NO_B
    if (i >= ADMA) return;
#endif
    if (i < ADMA) {
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(a_src[i] + (int64_t)cur_tile * BK), "s"(sbase + (unsigned)((ADMA * wid + i) * 1024))
          : "memory");
      return;
    }
    const int r = (i - ADMA) / SEG, c = (i - ADMA) % SEG;
    const int y = bkr[r] * dil, z = bkc[r] * dil;
    const unsigned x = 4u * (unsigned)(bc[r] * HW + y * W + z);
    const unsigned rowb = sbase + (unsigned)((A_FL + (BROWS * wid + r) * LDB + 64 * c) * 4);
    const bool ok = ((unsigned)(ir0[c] + y) < (unsigned)H) & ((unsigned)(ic0[c] + z) < (unsigned)W);
    const unsigned off = ok ? vbase[c] + x : 0x80000000u;
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(off), "s"(brsrc), "s"(rowb)
        : "memory");
  };
  auto issue = [&](int tile, int st) {  // the whole tile at once (prologue)
    cur_tile = tile;
#pragma unroll
    for (int i = 0; i < NDMA; ++i) dma(i, st);
  };

  // ---- MFMA: step s consumes k = 4s + q ----------------------------------
  floatx4 acc[J];
#pragma unroll
  for (int j = 0; j < J; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int arow = wr * 16 + r16;
  const int b_frag = wc * WTN + r16;
  auto frag = [&](const float* st, int s, float& a, float (&b)[J]) {
    a = st[(arow * 8 + (s ^ (arow & 7))) * 4 + q];
    const float* bp = st + A_FL + (4 * s + q) * LDB + b_frag;
#pragma unroll
    for (int j = 0; j < J; ++j) b[j] = bp[16 * j];
  };
  auto mma = [&](float a, const float (&b)[J]) {
#pragma unroll
    for (int j = 0; j < J; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[j], acc[j], 0, 0, 0);
  };

  const int nt = K / BK;
  if (nt > 0) {
    issue(0, 0);
    if (nt > 1) {
      advance();
      issue(1, 1);
      wait_vm_barrier<NDMA>();  // tile 0 landed (tile 1 may still be in flight)
    } else {
      wait_vm_barrier<0>();
    }
  }
  for (int t = 0; t < nt; ++t) {
    const float* cur = smem + (t % NSTAGE) * STAGE;
    const bool ahead = t + 2 < nt;
    // tile t+2's DMAs into stage (t+2)%3 = (t-1)%3 (every wave left it at the
    // last barrier), spread over the four step pairs of this tile behind
    // their MFMAs, waves 4..7 two pairs later than waves 0..3, so a wave
    // blocked issuing a DMA leaves its SIMD partner's MFMAs the pipe
    if (ahead) {
      advance();
      cur_tile = t + 2;
    }
    const int st2 = (t + 2) % NSTAGE;
    const int rot = (wid >> 2) * 2;
    float a0, b0[J], a1, b1[J];
    frag(cur, 0, a0, b0);
#pragma unroll
    for (int s = 0; s < BK / 4; s += 2) {
      frag(cur, s + 1, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a0, b0);
      if (s + 2 < BK / 4) frag(cur, s + 2, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      if (ahead) {
        const int grp = ((s >> 1) + rot) & 3;  // wave-uniform
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
          if (gg == grp) {
#pragma unroll
            for (int i = gg * NDMA / 4; i < (gg + 1) * NDMA / 4; ++i) dma(i, st2);
          }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t + 1 < nt) {  // tile t+1 landed (own DMAs), then everyone's
      if (ahead)
        wait_vm_barrier<NDMA>();
      else
        wait_vm_barrier<0>();
    }
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
    for (int e = 0; e < 4; ++e) {
      const int64_t row = m0 + wr * 16 + 4 * q + e;
      float v = acc[j][e];
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
    hipLaunchKernelGGL((conv_dma_kernel<G, 3>), dim3((unsigned)tiles), dim3(NT), 0, s, a, dil);
  else if (ks == 1)
    hipLaunchKernelGGL((conv_dma_kernel<G, 1>), dim3((unsigned)tiles), dim3(NT), 0, s, a, dil);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

struct TileInfo {
  int bm, bn;
  hipError_t (*fn)(const GemmArgs&, int, int, hipStream_t);
  const char* name;
};
#define TNS_CD(BMv, BNv) {BMv, BNv, launch_g<DGeo<BMv, BNv>>, "conv_dma<" #BMv "x" #BNv ">"}
const TileInfo kTiles[] = {
    TNS_CD(128, 176),  // 0: 52^2 / 104^2 3x3 (every wave all 11 column strips)
    TNS_CD(128, 96),   // 1: 26^2 layers (4 x 57 blocks)
    TNS_CD(64, 96),    // 2: 13^2 / 208^2 layers (2 column groups of 48)
    TNS_CD(64, 192),   // 3
    TNS_CD(128, 128),  // 4
};
#undef TNS_CD
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

}  // namespace

int conv_dma_count() { return kNumTiles; }
const char* conv_dma_name(int v) { return v >= 0 && v < kNumTiles ? kTiles[v].name : ""; }

// not picked by default until measured (TNS_OPT_CONV_VARIANT = 300 + v)
int conv_dma_pick(const GemmArgs& a, int ks) {
  (void)a; (void)ks;
  return -1;
}

hipError_t launch_conv_dma(int v, const GemmArgs& a, int ks, int dil, hipStream_t s) {
  if (v < 0 || v >= kNumTiles) return hipErrorInvalidValue;
  return kTiles[v].fn(a, ks, dil, s);
}

#else
int conv_dma_count() { return 0; }
const char* conv_dma_name(int) { return ""; }
int conv_dma_pick(const GemmArgs&, int) { return -1; }
hipError_t launch_conv_dma(int, const GemmArgs&, int, int, hipStream_t) { return hipErrorInvalidValue; }
#endif  // TNS_DIAG_KERNELS

}  // namespace tns
