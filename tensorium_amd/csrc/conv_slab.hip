// conv_slab.hip — the conv layers with few output pixels per filter (the
// 13^2 / 26^2 planes of YOLOv3: M = 512 / 1024 filters, K = 2304 / 4608) as
// a two-pass implicit GEMM: the im2col matrix written ONCE per layer in the
// exact order the GEMM's LDS images want it (the "slab"), then a GEMM whose B
// operand streams global -> LDS by LDS-DMA (global_load_lds_dwordx4, one
// 1 KB wave-instruction per 64 slots) — no per-tile gather, no address
// arithmetic, no transposing stores on the B side.
// (TConvolutionalLayer.forward -> Conv2D + forwardBias + activate after
// fuseBatchNorm: nConvolutionLayer.pas:457-569, ntensors.pas:8252-8349;
// sim2Col's column order, 11415-11532.)
//
// Arithmetic: exactly conv_tile4.hip's — every output an ascending-k fma chain
// over k = (c, kr, kc) from +0 (v_mfma_f32_16x16x4_f32: step s of a k-tile
// consumes k = 4s + q, lane quarter q), then bias add and activation, each
// rounded once — so bit-identical to it, to sim2Col + the reference GEMM.
//
// Slab layout (floats): for column tile ct (BN output pixels of the
// batch-folded N) and k-tile t (BK values of k) a contiguous chunk of
// ROWS = BK/4 slot rows x BN slots x 4: slot row 4g + q, slot c, component i
// holds col[k = t*BK + 16g + 4i + q][n = ct*BN + c] (0 past the window or
// past N) — the LDS image conv_tile4 builds by gathering, so a lane's
// ds_read_b128 of one slot feeds four MFMA steps.  Chunks of one column tile
// follow each other along k: a block streams K*BN contiguous floats.
//
// Why a second pass pays here: on these planes the col matrix is small
// (13^2: 4608 x 1352 floats = 25 MB, written in ~5 us) while the GEMM runs
// ~100 us, and the gather stages it replaces are where conv_tile4's k-loop
// loses time (block stamps: waves waiting at the tile barrier for late
// gathered operands, profiles/r05_conv_fwd_stamps.json).  The 52^2 and larger
// planes keep conv_tile4 (their col matrix is 100+ MB).
//
// GEMM schedule (per block: BM x BN outputs, 2 waves per SIMD): two LDS
// stages; A (weights, k-contiguous rows) through registers (float4 loads,
// each value stored into its k-permuted slot row); B by DMA.  One barrier per
// k-tile, before the tile's last 4-step group: before it each wave stores the
// next tile's A and waits for its own DMA of the next tile's B (both issued a
// whole tile earlier); after it the next tile's first fragments are read and
// the DMA of tile t+2 goes out into tile t's stage (whose last reads preceded
// the barrier), interleaved with the last group's MFMAs.
#include <algorithm>
#include <type_traits>

#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void slab_dma16(const float* sbase, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

struct SlabFillArgs {
  const float* x;   // images [batch][C][H][W]
  int64_t strideX;  // floats per image
  float* slab;
  int C, H, W, stride, pad, dil, ow, ohw, N, K, KT;
  float inv_ohw, inv_ow;  // (1 + 2^-20) / ohw, ... / ow: quotients by one multiply
  unsigned bytes;         // the images' extent (buffer range: loads past it read 0)
  int64_t units;          // CT * KT * NG * BN
};

// n / d for 0 <= n < 2^22 by a float multiply (the host rounds 1/d up a
// little), then exact corrections (none or one step for d >= 5)
__device__ __forceinline__ int slab_div(int n, int d, float inv) {
  int qq = (int)((float)n * inv);
  while (qq * d > n) --qq;
  while ((qq + 1) * d <= n) ++qq;
  return qq;
}

// one (column, 4-step group) per thread: the 16 consecutive k of group g of
// k-tile t at column n — four 16-byte slots (slot rows 4g + q), each a
// store of 64 consecutive slots across the wave; the column's window is
// decoded once, the 16 k walk (channel, tap) incrementally, and every value
// is one buffer load (taps outside the image read 0 through the range check:
// no branches, all 16 loads in flight together)
template <int KS, int BK, int BN>
__global__ __launch_bounds__(256) void slab_fill_kernel(SlabFillArgs a) {
  constexpr int NG = BK / 16, KK = KS * KS;
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (x >= a.units) return;
  const int c = (int)(x % BN);
  const int64_t r1 = x / BN;
  const int g = (int)(r1 % NG);
  const int64_t r2 = r1 / NG;
  const int t = (int)(r2 % a.KT), ct = (int)(r2 / a.KT);
  const int n = ct * BN + c;
  float v[16];
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x), 0, a.bytes, 0x00020000);
  {
    const int nn = n < a.N ? n : a.N - 1;  // (past N: any column, stored as 0)
    const int img = slab_div(nn, a.ohw, a.inv_ohw), pix = nn - img * a.ohw;
    const int oy = slab_div(pix, a.ow, a.inv_ow), ox = pix - oy * a.ow;
    const int iy0 = oy * a.stride - a.pad, ix0 = ox * a.stride - a.pad;
    const int HW = a.H * a.W;
    // the window's taps: validity bits and byte offsets from the origin
    unsigned mask = 0;
    int toff[KK];
#pragma unroll
    for (int kr = 0; kr < KS; ++kr)
#pragma unroll
      for (int kc = 0; kc < KS; ++kc) {
        const int iy = iy0 + kr * a.dil, ix = ix0 + kc * a.dil;
        mask |= (unsigned)(((unsigned)iy < (unsigned)a.H) & ((unsigned)ix < (unsigned)a.W))
                << (kr * KS + kc);
        toff[kr * KS + kc] = 4 * (kr * a.dil * a.W + kc * a.dil);
      }
    if (n >= a.N) mask = 0;
    const unsigned base = 4u * (unsigned)(img * (int)a.strideX + iy0 * a.W + ix0);
    const int k0 = t * BK + 16 * g;
    int ch = k0 / KK, tap = k0 - ch * KK;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      int off = toff[0];
#pragma unroll
      for (int u = 1; u < KK; ++u) off = tap == u ? toff[u] : off;
      const unsigned o = ((mask >> tap) & 1u) ? base + 4u * (unsigned)(ch * HW) + (unsigned)off
                                              : 0x80000000u;
      v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, o, 0, 0));
      if (++tap == KK) {
        tap = 0;
        ++ch;
      }
    }
  }
  // slot row 4g + q holds k = 16g + 4i + q: v[4i + q]
  float* dst = a.slab + ((r2 * NG + g) * 4 * BN + c) * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<floatx4*>(dst + q * BN * 4) = floatx4{v[q], v[4 + q], v[8 + q], v[12 + q]};
}

// The same fill with the (column tile, k-tile, group) of a block uniform:
// one block of BN (rounded up to whole waves) threads per (ct, t, g), a
// thread one column — so the 16 k's (channel, tap) walk and the taps' byte
// offsets are scalar, and a value costs the lane its window bit test, one
// address add and its load (the per-lane form selected each tap's offset
// out of nine registers: ~25 VALU instructions a value)
template <int KS, int BK, int BN>
__global__ __launch_bounds__((BN + 63) / 64 * 64) void slab_fill_u_kernel(SlabFillArgs a) {
  constexpr int NG = BK / 16, KK = KS * KS;
  const int c = threadIdx.x;
  if (c >= BN) return;
  const int64_t r1 = blockIdx.x;  // (ct * KT + t) * NG + g
  const int g = (int)(r1 % NG);
  const int64_t r2 = r1 / NG;
  const int t = (int)(r2 % a.KT), ct = (int)(r2 / a.KT);
  const int n = ct * BN + c;
  float v[16];
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x), 0, a.bytes, 0x00020000);
  {
    const int nn = n < a.N ? n : a.N - 1;  // (past N: any column, stored as 0)
    const int img = slab_div(nn, a.ohw, a.inv_ohw), pix = nn - img * a.ohw;
    const int oy = slab_div(pix, a.ow, a.inv_ow), ox = pix - oy * a.ow;
    const int iy0 = oy * a.stride - a.pad, ix0 = ox * a.stride - a.pad;
    const int HW = a.H * a.W;
    unsigned mask = 0;
#pragma unroll
    for (int kr = 0; kr < KS; ++kr)
#pragma unroll
      for (int kc = 0; kc < KS; ++kc) {
        const int iy = iy0 + kr * a.dil, ix = ix0 + kc * a.dil;
        mask |= (unsigned)(((unsigned)iy < (unsigned)a.H) & ((unsigned)ix < (unsigned)a.W))
                << (kr * KS + kc);
      }
    if (n >= a.N) mask = 0;
    const unsigned base = 4u * (unsigned)(img * (int)a.strideX + iy0 * a.W + ix0);
    // (block-uniform from here: k0, the channel / tap walk, the tap offsets)
    const int k0 = __builtin_amdgcn_readfirstlane(t * BK + 16 * g);
    int ch = k0 / KK, tap = k0 - ch * KK;
    int kr = tap / KS, kc = tap - kr * KS;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const unsigned uoff = 4u * (unsigned)(ch * HW + kr * a.dil * a.W + kc * a.dil);
      const unsigned o = ((mask >> tap) & 1u) ? base + uoff : 0x80000000u;
      v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, o, 0, 0));
      ++tap;
      if (++kc == KS) {
        kc = 0;
        ++kr;
      }
      if (tap == KK) {
        tap = 0;
        kr = 0;
        ++ch;
      }
    }
  }
  float* dst = a.slab + ((r2 * NG + g) * 4 * BN + c) * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    *reinterpret_cast<floatx4*>(dst + q * BN * 4) = floatx4{v[q], v[4 + q], v[8 + q], v[12 + q]};
}

struct SlabGemmArgs {
  const float* A;  // weights [M][K]
  const float* slab;
  float* C;        // [img][M][ohw]
  const float* bias;
  int M, N, K, KT, tiles_m, ohw, act;
  bool fuse;
};

// BM x BN block tile, BK-deep k-tiles, NS LDS stages (the B DMA runs NS - 1
// tiles ahead); WM x WN waves, each a 16-row strip of JA (wave columns < NA)
// or JB 16-column fragments (uneven splits keep the two waves of a SIMD —
// w and w + NW/2 — at the same fragment count)
template <int BM_, int BN_, int BK_, int WM_, int WN_, int JA_, int NA_, int NS_, int DG_ = 0,
          int MAP_ = 0>
struct SG {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_, JA = JA_, NA = NA_;
  static constexpr int NS = NS_;
  // DG (timing diagnostics, wrong results): 1 no B DMA, 2 no A loads / stores,
  // 4 no k-loop barrier; MAP 1: row tiles outer in the XCD order
  static constexpr int DG = DG_, MAP = MAP_;
  static constexpr int NW = WM * WN, NT = 64 * NW, J = BN / 16, NG = BK / 16, ROWS = BK / 4;
  static constexpr int JB = NA < WN ? (J - NA * JA) / (WN - NA) : 0;
  static constexpr int A_TILE = ROWS * BM * 4, B_TILE = ROWS * BN * 4, STAGE = A_TILE + B_TILE;
  static constexpr int AU = BM * BK / 4 / NT;       // float4 A units per thread and tile
  static constexpr int BDMA = 4 * BK * BN / 1024;   // 1 KB B DMA instructions per tile
  static constexpr int DPW = (BDMA + NW - 1) / NW;  // ... per wave (padded: uniform count)
  static_assert(BM == 16 * WM && BN % 16 == 0 && BK % 16 == 0, "geometry");
  static_assert(NA * JA + (WN - NA) * JB == J && NA >= 1 && NA <= WN, "wave column split");
  static_assert(AU >= 1 && BM * BK / 4 % NT == 0, "A units");
  static_assert(4 * BK * BN % 1024 == 0, "whole DMA instructions");
  static_assert(NS >= 2 && NS * STAGE * 4 <= 163840, "LDS");
  static_assert(NG >= 2 && NG % 2 == 0, "groups: f0 holds group 0 at every tile start");
  static_assert(DPW * (NS - 2) <= 63 && DPW <= 63, "vmcnt immediates");
};

template <int JW>
struct SFrag {
  floatx4 a, b[JW];
};

// s_waitcnt vmcnt(N) for a runtime choice between N and 0 (immediates only)
template <int N>
__device__ __forceinline__ void wait_vm(bool keep_n) {
  if (keep_n)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <class G>
__global__ __launch_bounds__(G::NT, 1) void slab_gemm_kernel(SlabGemmArgs p) {
  constexpr int BM = G::BM, BN = G::BN, BK = G::BK, NG = G::NG, NS = G::NS;
  constexpr int A_TILE = G::A_TILE, STAGE = G::STAGE, AU = G::AU, DPW = G::DPW;
  __shared__ __attribute__((aligned(16))) float smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), wm = w % G::WM, wn = w / G::WM;
  const int r16 = lane & 15, q = lane >> 4;
  // XCD-contiguous order, column tiles outer: the row blocks of one column
  // tile stream the same slab through one XCD's L2
  int tm, tn;
  {
    const int nb = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, qq = nb >> 3, rr = nb & 7;
    const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    if constexpr (G::MAP == 1) {
      const int tiles_n = (p.N + BN - 1) / BN;
      tn = wg % tiles_n;
      tm = wg / tiles_n;
    } else {
      tm = wg % p.tiles_m;
      tn = wg / p.tiles_m;
    }
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int N = p.N, K = p.K, nt = p.KT;
  const float* slabT = p.slab + (int64_t)tn * K * BN;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)smem;
  const unsigned voff = 16u * (unsigned)lane;
  // B: this wave's DMA instructions of tile t into stage st (u = w + NW v;
  // past the tile's last one a wave repeats an instruction of another wave:
  // the same bytes to the same place, so every wave issues DPW)
  auto dma_b = [&](int t, int st, int v) {
    if constexpr (G::DG & 1) return;
    int u = w + G::NW * v;
    if (G::BDMA % G::NW != 0 && u >= G::BDMA) u -= G::NW;
    slab_dma16(slabT + (int64_t)t * (BK * BN) + 256 * u, voff,
               lds0 + 4u * (unsigned)(st * STAGE + A_TILE) + 1024u * (unsigned)u);
  };
  auto dma_all = [&](int t, int st) {
#pragma unroll
    for (int v = 0; v < DPW; ++v) dma_b(t, st, v);
  };
  // A staging: unit = k-quad kq4 of row m (8 k-quads per 8 lanes: 128
  // contiguous bytes of a row); its values go to slot rows 4(kq4>>2) + 0..3,
  // component kq4 & 3.  The loads are asm (SGPR base + lane offset): the
  // compiler cannot see the DMA in the vmcnt queue, so the waits are counted
  // by hand — a load is waited for with the younger DMA still in flight
  unsigned a_off[AU];
  int a_dst[AU];
#pragma unroll
  for (int u = 0; u < AU; ++u) {
    const int idx = tid + G::NT * u;
    const int lo = idx & 7, rest = idx >> 3;
    const int m = rest % BM, kq4 = lo + 8 * (rest / BM);
    a_off[u] = 4u * (unsigned)(m * K + 4 * kq4);
    a_dst[u] = (4 * (kq4 >> 2)) * BM * 4 + m * 4 + (kq4 & 3);
  }
  const float* a_row0 = p.A + (int64_t)m0 * K;
  floatx4 ra[AU];
  auto load_a = [&](int t) {
    if constexpr (G::DG & 2) return;
    const float* sb = a_row0 + t * BK;
#pragma unroll
    for (int u = 0; u < AU; ++u)
      asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(ra[u]) : "v"(a_off[u]), "s"(sb) : "memory");
  };
  auto store_a = [&](int st) {
    if constexpr (G::DG & 2) return;
    float* as = smem + st * STAGE;
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      asm volatile("" : "+v"(ra[u]));  // (after the wait: the loaded values)
      as[a_dst[u]] = ra[u][0];
      as[a_dst[u] + BM * 4] = ra[u][1];
      as[a_dst[u] + 2 * BM * 4] = ra[u][2];
      as[a_dst[u] + 3 * BM * 4] = ra[u][3];
    }
  };

  auto run = [&](auto JWC, const int coff) {
    constexpr int JW = decltype(JWC)::value;
    floatx4 acc[JW];
#pragma unroll
    for (int j = 0; j < JW; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    using Frag = SFrag<JW>;
    auto frag = [&](int st, int g, Frag& f) {
      const float* ap = smem + st * STAGE + ((4 * g + q) * BM + wm * 16 + r16) * 4;
      f.a = *reinterpret_cast<const floatx4*>(ap);
      const float* bp = smem + st * STAGE + A_TILE + ((4 * g + q) * BN + coff * 16 + r16) * 4;
#pragma unroll
      for (int j = 0; j < JW; ++j) f.b[j] = *reinterpret_cast<const floatx4*>(bp + 64 * j);
    };
    auto mma = [&](const Frag& f) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < JW; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[i], f.b[j][i], acc[j], 0, 0, 0);
    };
    // the last group's MFMAs with this wave's DMA instructions of tile tb
    // spread over them
    auto mma_dma = [&](const Frag& f, int tb, int st) {
      constexpr int NM = 4 * JW, STEP = NM / DPW > 0 ? NM / DPW : 1;
#pragma unroll
      for (int x = 0; x < NM; ++x) {
        const int i = x / JW, j = x % JW;
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[i], f.b[j][i], acc[j], 0, 0, 0);
        if (x % STEP == 0 && x / STEP < DPW) dma_b(tb, st, x / STEP);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (NM / STEP < DPW) {  // (more DMA instructions than MFMAs)
#pragma unroll
        for (int v = NM / STEP; v < DPW; ++v) dma_b(tb, st, v);
      }
    };

    Frag f0, f1;
    // prologue: tiles 0 .. NS-1's B DMA into stages 0 .. NS-1, tile 0's A
    // stored, tile 1's A loads in flight (issued before tile 1's DMA)
    load_a(0);
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      if (t == 1 && nt > 1) {
        wait_vm<0>(false);  // (tile 0's A and B)
        store_a(0);
        load_a(1);
      }
      if (t < nt) dma_all(t, t);
    }
    if (nt == 1) {
      wait_vm<0>(false);
      store_a(0);
    } else {
      // tile 0's B: the DMA of tiles 1 .. NS-1 (and tile 1's A) may fly on
      if (nt >= NS)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AU + (NS - 1) * DPW) : "memory");
      else
        wait_vm<0>(false);
    }
    __syncthreads();
    frag(0, 0, f0);
    for (int t = 0; t < nt; ++t) {
      const int cur = t % NS;
#pragma unroll
      for (int g = 0; g + 1 < NG; ++g) {
        Frag& fc = (g & 1) ? f1 : f0;
        Frag& fn = (g & 1) ? f0 : f1;
        frag(cur, g + 1, fn);
        __builtin_amdgcn_sched_barrier(0);
        mma(fc);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (t + 1 < nt) {
        // tile t+1: A (loaded after barrier t-1) and B (DMA'd after barrier
        // t+1-NS, older); younger in the queue: tile t-1+NS's DMA, issued
        // after A(t+1) (NS >= 3, where that tile exists)
        const int nxt = (t + 1) % NS;
        if constexpr (NS == 2)
          wait_vm<0>(false);
        else
          wait_vm<DPW>(t + NS - 1 < nt);
        store_a(nxt);
        if constexpr (!(G::DG & 4))
          __syncthreads();  // every wave's tile t+1 in; every read of tile t done
        frag(nxt, 0, f0);
        // tile t+2's A loads, then tile t+NS's B DMA into tile t's stage
        if (t + 2 < nt) load_a(t + 2);
        __builtin_amdgcn_sched_barrier(0);
        if (t + NS < nt)
          mma_dma(f1, t + NS, cur);
        else
          mma(f1);
      } else {
        mma(f1);
      }
    }

    // epilogue: forwardBias + activate, conv output [img][filter][pixel]
    const int row0 = m0 + wm * 16 + 4 * q;
    float bias[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[e] = p.fuse ? p.bias[row0 + e] : 0.0f;
#pragma unroll
    for (int j = 0; j < JW; ++j) {
      const int n = n0 + coff * 16 + 16 * j + r16;
      if (n >= N) continue;
      const int img = n / p.ohw, pix = n - img * p.ohw;
      float* cp = p.C + ((int64_t)img * p.M + row0) * p.ohw + pix;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[j][e];
        if (p.fuse) v = act_apply_cheap(v + bias[e], p.act);
        cp[(int64_t)e * p.ohw] = v;
      }
    }
  };
  if constexpr (G::NA == G::WN) {
    run(std::integral_constant<int, G::JA>{}, wn * G::JA);
  } else {
    if (wn < G::NA)
      run(std::integral_constant<int, G::JA>{}, wn * G::JA);
    else
      run(std::integral_constant<int, G::JB>{}, G::NA * G::JA + (wn - G::NA) * G::JB);
  }
}

struct SlabForm {
  int bm, bn, bk;
  hipError_t (*gemm)(const SlabGemmArgs&, hipStream_t);
  hipError_t (*fill)(const SlabFillArgs&, int ks, hipStream_t);
  const char* name;
};

template <class G>
hipError_t launch_slab_gemm(const SlabGemmArgs& a, hipStream_t s) {
  const int64_t blocks = (int64_t)(a.M / G::BM) * ((a.N + G::BN - 1) / G::BN);
  hipLaunchKernelGGL((slab_gemm_kernel<G>), dim3((unsigned)blocks), dim3(G::NT), 0, s, a);
  return hipGetLastError();
}

template <int BK, int BN>
hipError_t launch_slab_fill(const SlabFillArgs& a, int ks, hipStream_t s) {
#ifndef TNS_SLAB_FILL_LANE  // (A/B side builds: the per-lane form)
  {
    constexpr int NT = (BN + 63) / 64 * 64;
    const int64_t nb = a.units / BN;  // (ct, t, g) triples
    if (nb > 0x7fffffffLL) return hipErrorInvalidValue;
    if (ks == 3)
      hipLaunchKernelGGL((slab_fill_u_kernel<3, BK, BN>), dim3((unsigned)nb), dim3(NT), 0, s, a);
    else if (ks == 1)
      hipLaunchKernelGGL((slab_fill_u_kernel<1, BK, BN>), dim3((unsigned)nb), dim3(NT), 0, s, a);
    else
      return hipErrorInvalidValue;
    return hipGetLastError();
  }
#endif
  const unsigned blocks = (unsigned)((a.units + 255) / 256);
  if (ks == 3)
    hipLaunchKernelGGL((slab_fill_kernel<3, BK, BN>), dim3(blocks), dim3(256), 0, s, a);
  else if (ks == 1)
    hipLaunchKernelGGL((slab_fill_kernel<1, BK, BN>), dim3(blocks), dim3(256), 0, s, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

#define TNS_SLAB(BMv, BNv, BKv, WMv, WNv, JAv, NAv, NSv)                                       \
  {BMv, BNv, BKv, launch_slab_gemm<SG<BMv, BNv, BKv, WMv, WNv, JAv, NAv, NSv>>,                   \
   launch_slab_fill<BKv, BNv>,                                                                   \
   "conv_slab<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",j" #JAv "x" #NAv ",s" #NSv ">"}
#define TNS_SLABD(BMv, BNv, BKv, WMv, WNv, JAv, NAv, NSv, DGv, MAPv)                             \
  {BMv, BNv, BKv, launch_slab_gemm<SG<BMv, BNv, BKv, WMv, WNv, JAv, NAv, NSv, DGv, MAPv>>,       \
   launch_slab_fill<BKv, BNv>,                                                                   \
   "conv_slab<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",j" #JAv "x" #NAv ",s" #NSv ",dg" #DGv \
   ",map" #MAPv ">"}
const SlabForm kSlab[] = {
    TNS_SLAB(32, 176, 64, 2, 4, 3, 3, 3),   // 0: form 3 with three stages (DMA two tiles ahead)
    TNS_SLAB(64, 176, 32, 4, 2, 6, 1, 3),   // 1
    TNS_SLAB(64, 176, 32, 4, 2, 6, 1, 4),   // 2
    TNS_SLAB(32, 176, 64, 2, 4, 3, 3, 2),   // 3: the 13^2 planes (8 x 32 blocks) — picked
    TNS_SLAB(64, 176, 64, 4, 2, 6, 1, 2),   // 4: the 26^2 planes (31 x 8 blocks) — picked
    TNS_SLAB(32, 176, 32, 2, 2, 6, 1, 4),   // 5: one wave per SIMD
    TNS_SLABD(32, 176, 64, 2, 4, 3, 3, 2, 0, 1),  // 6: form 3, row tiles outer
    TNS_SLABD(64, 176, 64, 4, 2, 6, 1, 2, 0, 1),  // 7: form 4, row tiles outer
};
#undef TNS_SLAB
#undef TNS_SLABD
constexpr int kNumSlab = sizeof(kSlab) / sizeof(kSlab[0]);

}  // namespace

int conv_slab_count() { return kNumSlab; }
const char* conv_slab_name(int v) { return v >= 0 && v < kNumSlab ? kSlab[v].name : ""; }

// the form for a layer, -1: conv_tile4 stays.  Measured at batch 8, warm
// clock, kernel trace (scripts/slab_prof.sh, profiles/r06_conv_slab.json):
// the 13^2 planes (1024 filters, K = 4608 / 2304 stride 2) on 32 x 176 x 64
// (fill 10.1 + GEMM 116.5 us against conv_tile4's 133.7), the 26^2 planes
// (512 filters, K = 2304) on 64 x 176 x 64 (15.5 + 108.2 against 130.8); the
// 1x1 layers stay (the fill and the short k: 13^2 0.035 against 0.023 ms)
int conv_slab_pick(int64_t M, int64_t N, int64_t K, int64_t ks) {
  if (ks != 3 || K % 64) return -1;
  if (M == 1024 && N >= 1024) return 3;
  if (M == 512 && N >= 4096) return 4;
  return -1;
}

int64_t conv_slab_floats(int v, int64_t N, int64_t K) {
  if (v < 0 || v >= kNumSlab) return -1;
  const int64_t bn = kSlab[v].bn;
  return (N + bn - 1) / bn * bn * K;
}

hipError_t launch_conv_slab(int v, const ConvSlabArgs& c, float* slab, hipStream_t s) {
  if (v < 0 || v >= kNumSlab) return hipErrorInvalidValue;
  const SlabForm& f = kSlab[v];
  const int64_t N = c.batch * c.ohw;
  // (32-bit buffer offsets over the images; columns below 2^22 for slab_div)
  if (c.M % f.bm || c.K % f.bk || (c.ks != 1 && c.ks != 3) || N >= (1LL << 22) ||
      4 * c.batch * c.C * c.H * c.W > 0x7fffffffLL ||
      c.K > 0x7fffffffLL / f.bn || (reinterpret_cast<uintptr_t>(c.weights) & 15) || c.K % 4 ||
      (reinterpret_cast<uintptr_t>(slab) & 15) || c.M * c.K > 0x7fffffffLL)
    return hipErrorInvalidValue;
  const int64_t CT = (N + f.bn - 1) / f.bn, KT = c.K / f.bk;
  if (CT * (c.M / f.bm) > 0x7fffffffLL) return hipErrorInvalidValue;
  SlabFillArgs fa{};
  fa.x = c.input; fa.strideX = c.C * c.H * c.W; fa.slab = slab;
  fa.C = (int)c.C; fa.H = (int)c.H; fa.W = (int)c.W; fa.stride = (int)c.stride;
  fa.pad = (int)c.pad; fa.dil = (int)c.dil; fa.ow = (int)c.ow; fa.ohw = (int)c.ohw;
  fa.N = (int)N; fa.K = (int)c.K; fa.KT = (int)KT;
  fa.inv_ohw = (float)((1.0 + 1.0 / 1048576.0) / (double)c.ohw);
  fa.inv_ow = (float)((1.0 + 1.0 / 1048576.0) / (double)c.ow);
  fa.bytes = (unsigned)(4 * c.batch * c.C * c.H * c.W);
  fa.units = CT * KT * (f.bk / 16) * f.bn;
  if (hipError_t e = f.fill(fa, (int)c.ks, s)) return e;
  SlabGemmArgs ga{};
  ga.A = c.weights; ga.slab = slab; ga.C = c.out; ga.bias = c.bias;
  ga.M = (int)c.M; ga.N = (int)N; ga.K = (int)c.K; ga.KT = (int)KT;
  ga.tiles_m = (int)(c.M / f.bm); ga.ohw = (int)c.ohw; ga.act = c.act; ga.fuse = c.bias != nullptr;
  return f.gemm(ga, s);
}

}  // namespace tns
