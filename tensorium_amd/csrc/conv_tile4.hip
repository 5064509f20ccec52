// conv_tile4.hip — conv_tile.hip's plane-sized implicit-GEMM convolution with
// k-permuted LDS images: one ds_read_b128 per operand fragment feeds four
// v_mfma_f32_16x16x4_f32 steps (TConvolutionalLayer.forward → Conv2D +
// forwardBias + activate after fuseBatchNorm: nConvolutionLayer.pas:457-569,
// ntensors.pas:8252-8349; sim2Col's column order, 11415-11532).
//
// Same arithmetic as conv_tile.hip (each output an ascending-k fma chain over
// k = (c, kr, kc) from +0 in the 16x16x4 lane-quarter order, then bias add
// and activation, each rounded once), so bit-identical to it and to sim2Col +
// the reference GEMM.  What changes is how the operands reach the MFMAs:
//
//   * MFMA step s of a k-tile consumes k = 4s + q (lane quarter q).  Steps
//     4g .. 4g+3 form group g; a lane's four values of one group sit in one
//     16-byte LDS slot: image row 4g + q, slot = column, component i holds
//     k = 16g + 4i + q.  A wave reads 1 A slot + J B slots per group (12
//     ds_read_b128 per 44 MFMAs on the 128x176 tile, against 12 ds_read_b32
//     per 11 MFMAs): the bare wave loop measured 0.968 of the MFMA peak in
//     this form against 0.857 with per-step b32 reads (scripts/mfma_probe.hip).
//     Row strides are multiples of 64 dwords, so the b128 reads are
//     conflict-free;
//   * B is gathered as in conv_tile (lanes of a quarter take 16 consecutive
//     output pixels of one k, out-of-window taps read 0 through the buffer
//     range check), but a lane quarter takes the component i, not q, so the
//     transposing ds_write_b32 stores are 2-way (free); each column's window
//     validity is a 9-bit tap mask computed once, one bfe per element;
//   * A (weights, k-contiguous) float4 loads are spread into the four slot
//     rows of their k-quad (2-way stores, no swizzle needed);
//   * one barrier per k-tile, placed before the last group's MFMAs: the next
//     tile's first fragments are read right after it, under those MFMAs, so
//     no LDS latency is exposed at the tile boundary; the next tile's global
//     loads are issued at the top of a tile and stored after group SG.
//
// Two other B staging forms, bit-identical, kept selectable (TNS_CT4D): BD
// gathers by dword LDS-DMA straight into the slots, BW lets a lane fill whole
// slots (four loads along k, one ds_write_b128, lanes along 64 pixels).  On
// YOLOv3 layer 11 at a warm clock (scripts/ct4_stamps.py: 13.3 k cycles per
// 64-deep tile, 11.26 k of them MFMA) both are slower: BD 0.127 ms (the DMA
// issue doubles the tile-top phase), BW 0.123 ms (last group +0.86 k
// cycles), against 0.115 ms — although a diagnostic build without the b32 B
// stores runs 11.6 k cycles per tile (0.100 ms).  Likewise AP (A by 16-byte
// LDS-DMA from a slot-ordered copy of the weights made per call): 0.120 ms.
#include <algorithm>
#include <cstring>
#include <type_traits>

#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int I, int N, class F>
__device__ __forceinline__ void cfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    cfor<I + 1, N>(f);
  }
}

// ds_write_addtid_b32: LDS[M0 + OFF + 4 * lane] = v (M0 saved and restored)
template <int OFF>
__device__ __forceinline__ void st_addtid(float v, unsigned m0v) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "ds_write_addtid_b32 %1 offset:%3\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v), "s"(m0v), "i"(OFF)
      : "memory");
}

// one group's fragments of a wave: the A slot and JW B slots (4 steps each)
template <int JW>
struct Frag4 {
  floatx4 a, b[JW];
};

template <int BM_, int BN_, int WM_, int WN_, int BK_, int SG_, int IL_ = 0, bool SI_ = false,
          int RI_ = 0, bool ST_ = false, int JA_ = 0, int NA_ = 0, bool TA_ = false,
          bool BD_ = false, bool BW_ = false, bool AP_ = false, bool AT_ = false,
          bool DX_ = false, bool PF_ = false>
struct Geo4 {
  // PF: the register-staged operands of tile t+2 are loaded at the top of
  // tile t (two register sets, the tile pairs unrolled), so a gather has a
  // whole tile to land before its stores (the 2-group 26^2 / 13^2 forms
  // otherwise wait at the barrier for their loads: block stamps,
  // profiles/r05_conv_fwd_stamps.json)
  static constexpr bool PF = PF_;
  // DX: the conv backward's state.delta of a stride-1 layer as one implicit
  // transposed convolution — A = the weights tap-major, wt[t][f][c] (k-major,
  // TA), B = the delta planes gathered through the flipped window, k = t*F + f:
  // every tap's ascending-f chain from +0 is added to the image pixel at the
  // tap's end, in scol2im's (kr, kc) order, skipping the taps it skips — the
  // reference's TN GEMM + col2im sums, no col matrix (F % BK == 0: a k-tile
  // never straddles taps)
  static constexpr bool DX = DX_;
  // AT: B stored by ds_write_addtid_b32 (address M0 + offset + 4 * lane: no
  // address VGPR, 2 cycles a store against 4 for ds_write_b32): the gather
  // lanes are (pixel = lane >> 2, slot component = lane & 3), so a wave's 64
  // stores of one (slot row, fragment) are 64 consecutive dwords; the two
  // stages' B images sit below the A images (M0 + offset reach them)
  static constexpr bool AT = AT_;
  // AP: A read from a pre-permuted copy of the weights (conv_tile4_permute:
  // slot row R = 4g + q of the whole K, then m, then the slot's 4 values), so
  // a tile's slot row is contiguous and arrives by 16-byte LDS-DMA
  // (global_load_lds_dwordx4, 64 slots per wave-instruction): no A staging
  // registers and no transposing stores
  static constexpr bool AP = AP_;
  // BW: a B gather lane fills whole 16-byte slots (its pixel's four k of one
  // slot row: four dword loads, one ds_write_b128); lanes along 64
  // consecutive pixels, the slot row wave-uniform (scalar k walk)
  static constexpr bool BW = BW_;
  // BD: B gathered straight into its LDS slots by dword LDS-DMA
  // (buffer_load_dword ... lds; lanes = 16 pixels x the 4 slot components, so
  // one wave-instruction fills 16 slots of a slot row): no staging registers,
  // no ds_write, no wait on the gather before the mid-tile stores
  static constexpr bool BD = BD_;
  // TA: A stored k-major ([K][M], gemm(Trans, ...)): a thread fills whole
  // 16-byte slots (four dword loads down k, one ds_write_b128); used for the
  // conv backward's col = W^T . delta as a 1x1 "convolution" over delta
  static constexpr bool TA = TA_;
  // WM x WN waves, each a 16-row strip of BN / WN columns; or, with JA > 0,
  // wave columns 0..NA-1 of JA 16-column fragments and the rest of JB (176 =
  // 6 + 5 fragments: waves w and w + NW/2 share a SIMD, so a SIMD's two waves
  // carry 11 fragments either way)
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BK = BK_, SG = SG_;
  // instruction placement (sched_group_barrier) inside each group's MFMAs:
  //   IL > 0: the next tile's loads and their address arithmetic in group 0
  //           (IL VALU per MFMA) instead of a block at the tile top
  //   SI:     the LDS stores of the next tile in group SG, one per MFMA,
  //           instead of a block after it
  //   RI > 0: the next group's fragment reads one per RI MFMAs instead of a
  //           block in front of them
  //   ST:     staging staggered by wave half (waves w and w + NW/2 share a
  //           SIMD): half h issues its loads in front of group h's MFMAs and
  //           stores after group SG + h, so one wave of a SIMD runs MFMAs
  //           while the other stages
  static constexpr int IL = IL_, RI = RI_;
  static constexpr bool SI = SI_, ST = ST_;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int J = BN / 16;             // 16-column fragments of the tile
  static constexpr int JA = JA_ > 0 ? JA_ : J / WN;  // ... of one wave (columns < NA)
  static constexpr int NA = JA_ > 0 ? NA_ : WN;
  static constexpr int JB = NA < WN ? (J - NA * JA) / (WN - NA) : 0;  // ... of the others
  static constexpr int NG = BK / 16;            // 4-step groups per k-tile
  static constexpr int ROWS = BK / 4;           // slot rows per image (4g + q)
  static constexpr int A_TILE = ROWS * BM * 4;  // floats
  static constexpr int STAGE = ROWS * (BM + BN) * 4;
  static constexpr int B_TILE = ROWS * BN * 4;  // floats
  static constexpr int AU = BM * BK / 4 / NT;   // float4 A units per thread
  static constexpr int KI = BK / 4 / NW;        // B k-slots per thread
  // ATA: with AT, the A stores too by ds_write_addtid_b32 where both stages'
  // A images lie within M0 + offset reach (lanes = 16 rows x the 4 slot
  // components of one k group: each of a float4's values goes to one slot row
  // as 64 consecutive dwords)
  static constexpr bool ATA = AT && (2 * B_TILE + 2 * A_TILE) * 4 <= 126976 &&
                              NG * (BM / 16) % NW == 0 && NG * (BM / 16) / NW == AU;
  static_assert(BM == 16 * WM, "one 16-row strip per wave");
  static_assert(BM % 16 == 0 && BN % 16 == 0, "b128 slot rows: 64-dword multiples");
  static_assert(BK % 16 == 0 && SG <= NG - 2, "stores precede the barrier");
  static_assert(!(IL && SI) || SG >= 1 || PF_, "interleaved stores need a group after the loads");
  static_assert(!ST || (!IL && !SI && SG + 1 <= NG - 2 && NW % 2 == 0), "staggered staging");
  static_assert(AU >= 1 && BM * BK / 4 % NT == 0 && KI >= 1 && BK / 4 % NW == 0, "geometry");
  static_assert(NA * JA + (WN - NA) * JB == J && NA >= 1 && NA <= WN, "wave column split");
  static_assert(2 * STAGE * 4 + 64 <= 163840, "LDS");
  static_assert(!BD || (!IL && !ST && !TA), "DMA gather: tile-top issue only");
  static_assert(!(BD && BW), "one gather form");
  static_assert(!AT || (!BD && !BW && !TA && !AP && !SI && 2 * B_TILE * 4 <= 98304),
                "addtid B stores: register-staged gather, block-placed stores, B images below 96 KB");
  static_assert(!AP || (!IL && !ST && !TA && BM % 64 == 0 && ROWS * BM % (64 * NW) == 0),
                "A DMA: tile-top issue, whole 64-slot pieces");
  static_assert(!DX || (TA && !AT && !BD && !BW && !AP), "DX: k-major weights, b32 gather");
  static_assert(!PF || (!AT && !AP && !BD && !BW && !ST), "PF: register staging");
  static constexpr int ADM = AP ? ROWS * BM / 64 / NW : 0;  // A DMA instructions per wave
  static constexpr int AST = AP ? 0 : 4 * AU;                // A LDS stores per thread
  static constexpr int CH = (BN + 63) / 64;  // (BW) 64-pixel chunks of a slot row
  static constexpr int BLD = BW ? KI * CH * 4 : KI * J;            // B loads per thread
  static constexpr int BST = BW ? KI * CH : (BD ? 0 : KI * J);      // B LDS stores per thread
};

template <class G, int KS>
__global__ __launch_bounds__(G::NT) void conv_tile4_kernel(GemmArgs p, int dil) {
  constexpr int BM = G::BM, BN = G::BN, BK = G::BK, J = G::J, NG = G::NG;
  constexpr int A_TILE = G::A_TILE, STAGE = G::STAGE, AU = G::AU, KI = G::KI;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
#ifdef TNS_CT4_STAMPS
  const unsigned long long rt_entry = __builtin_amdgcn_s_memrealtime();
#endif
  // stage st: A image and B image (AT: [B0][B1][A0][A1], else [A0 B0][A1 B1])
  auto a_st = [&](int st) -> float* {
    return G::AT ? smem + 2 * G::B_TILE + st * A_TILE : smem + st * STAGE;
  };
  auto b_st = [&](int st) -> float* {
    return G::AT ? smem + st * G::B_TILE : smem + st * STAGE + A_TILE;
  };

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w % G::WM, wn = w / G::WM;
  const int half = __builtin_amdgcn_readfirstlane(w >= G::NW / 2 ? 1 : 0);  // (ST)
  const int r16 = lane & 15, q = lane >> 4;
  const int tiles_m = (int)(p.M / BM);
  // XCD-contiguous order, column tiles outer (blocks of one XCD share the
  // images' rows in its L2); tile rows inner
  int tm, tn;
  {
    const int nb = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, qq = nb >> 3, rr = nb & 7;
    const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
#if defined(TNS_CT4_MAP) && TNS_CT4_MAP == 1  // (A/B side builds: row tiles outer)
    const int tiles_n = (int)((p.N + BN - 1) / BN);
    tn = wg % tiles_n;
    tm = wg / tiles_n;
#elif defined(TNS_CT4_MAP) && TNS_CT4_MAP == 2  // (groups of 4 row tiles, column-major within)
    const int tiles_n = (int)((p.N + BN - 1) / BN);
    const int gm = min(4, tiles_m), per = gm * tiles_n, grp = wg / per;
    const int gs = min(gm, tiles_m - grp * gm), in = wg - grp * per;
    tm = grp * gm + in % gs;
    tn = in / gs;
#else
    tm = wg % tiles_m;
    tn = wg / tiles_m;
#endif
  }
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;
  const int N = (int)p.N, K = (int)p.K;
  const int H = p.conv_H, W = p.conv_W, HW = H * W;
  // (DX) column pixel -> image pixel: itself, or a stride-2 class pixel
  auto dx_pix = [&](int pix) -> int {
    if (!p.dx_cls) return pix;
    const int qy = pix / p.conv_ow, qx = pix - qy * p.conv_ow;
    return (2 * qy + ((p.dx_cls >> 1) & 1)) * p.dx_imgW + 2 * qx + ((p.dx_cls >> 2) & 1);
  };

  // ---- per-column state: window origin and the 9-bit tap validity mask ----
  // gather lanes: pixel gp of a 16-column fragment, slot component gq
  // (BD: the DMA writes lane L to float 4 * (L >> 2) + (L & 3) of its row)
  // (BW: lane = pixel of a 64-pixel chunk)
  // (AT: the same lane split, for consecutive-dword stores)
  const int gp = (G::BD || G::AT) ? lane >> 2 : r16, gq = (G::BD || G::AT) ? lane & 3 : q;
  constexpr int NCOL = G::BW ? G::CH : J;
  // output column n (clamped below N): its window's base offset and tap mask
  auto col_geo = [&](int n, unsigned& vb, unsigned& m) {
    n = n < N ? n : N - 1;  // past N: any valid pixel, never stored
    const int img = n / p.conv_ohw, pix = n - img * p.conv_ohw;
    const int orow = pix / p.conv_ow, ocol = pix - orow * p.conv_ow;
    const int ir0 = orow * p.conv_sY - p.conv_pH, ic0 = ocol * p.conv_sX - p.conv_pW;
    vb = 4u * (unsigned)(img * (int)p.strideB + ir0 * W + ic0);
    m = 0;
#pragma unroll
    for (int kr = 0; kr < KS; ++kr)
#pragma unroll
      for (int kc = 0; kc < KS; ++kc)
        m |= (unsigned)(((unsigned)(ir0 + kr * dil) < (unsigned)H) &
                        ((unsigned)(ic0 + kc * dil) < (unsigned)W))
             << (kr * KS + kc);
  };
  unsigned vbase[NCOL], tmask[NCOL];
#pragma unroll
  for (int j = 0; j < NCOL; ++j) col_geo(n0 + (G::BW ? 64 * j + lane : 16 * j + gp), vbase[j], tmask[j]);
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.B), 0, p.conv_bytes, 0x00020000);

  // ---- B k-slots: slot sl = wm*KI + ii = 4g + r takes k = 16g + 4q + r (the
  // lane quarter is the slot component), advanced by BK per tile -------------
  // (BW: entry 4 ii + i = component i of slot row w*KI + ii, wave-uniform)
  const int wu = __builtin_amdgcn_readfirstlane(w);
  constexpr int NKS = G::BW ? 4 * KI : KI;
  int kc_[NKS], kr_[NKS], cc_[NKS];
#pragma unroll
  for (int ii = 0; ii < NKS; ++ii) {
    const int sl = G::BW ? wu * KI + ii / 4 : w * KI + ii;
    const int k = 16 * (sl >> 2) + 4 * (G::BW ? ii % 4 : gq) + (sl & 3);
    if constexpr (G::DX) {  // (k < BK <= F: tap 0, filter k)
      cc_[ii] = k;
      kr_[ii] = kc_[ii] = 0;
      continue;
    }
    cc_[ii] = k / (KS * KS);
    const int rem = k - cc_[ii] * KS * KS;
    kr_[ii] = rem / KS;
    kc_[ii] = rem - kr_[ii] * KS;
  }
  // (DX) the tile's first filter and its tap t in the forward window's
  // terms: reference tap (kr, kc) = t reads the delta pixel at forward tap
  // (KS-1-kr, KS-1-kc) of a window padded by KS-1-pad
  // (a stride-2 pixel class: its dx_taps >> 16 taps)
  const int F_ = G::DX ? K / (p.dx_cls ? (p.dx_taps >> 16) : KS * KS) : 0;
  int d_f0 = 0, d_t = 0;
  auto advance = [&]() {  // k += BK
    if constexpr (G::DX) {
      d_f0 += BK;
      if (d_f0 == F_) {
        d_f0 = 0;
        ++d_t;
      }
      return;
    }
#pragma unroll
    for (int ii = 0; ii < NKS; ++ii) {
      if constexpr (KS == 1) {
        cc_[ii] += BK;
      } else {
        constexpr int DC = BK / (KS * KS), DR = BK % (KS * KS);
        int rem = kr_[ii] * KS + kc_[ii] + DR;
        int c = cc_[ii] + DC;
        if (rem >= KS * KS) { rem -= KS * KS; ++c; }
        cc_[ii] = c;
        kr_[ii] = rem >= 2 * KS ? 2 : (rem >= KS ? 1 : 0);
        kc_[ii] = rem - kr_[ii] * KS;
      }
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  float rbs[G::PF ? 2 : 1][KI][J];  // (unused with BD / BW; PF: one set a tile parity)
  floatx4 rw[G::BW ? KI : 1][G::BW ? G::CH : 1];  // (BW)
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)smem;
  auto gather_b = [&](const float* bs, auto SET) {
    auto& rb = rbs[decltype(SET)::value];
    if constexpr (G::BW) {
#pragma unroll
      for (int ii = 0; ii < KI; ++ii)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = 4 * ii + i;
          const unsigned x = 4u * (unsigned)(cc_[e] * HW + kr_[e] * dil * W + kc_[e] * dil);
          const int tap = kr_[e] * KS + kc_[e];
#pragma unroll
          for (int c = 0; c < G::CH; ++c) {
            const bool ok = __builtin_amdgcn_ubfe(tmask[c], tap, 1) != 0;
            const unsigned off = ok ? vbase[c] + x : 0x80000000u;
            rw[ii][c][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0));
          }
        }
      return;
    }
#pragma unroll
    for (int ii = 0; ii < KI; ++ii) {
      int y = kr_[ii] * dil, z = kc_[ii] * dil, tap = kr_[ii] * KS + kc_[ii], cc = cc_[ii];
      if constexpr (G::DX) {
        int fr = KS - 1 - d_t / KS, fc = KS - 1 - d_t % KS;  // wave-uniform
        if (p.dx_cls) {
          const int fb = (p.dx_taps >> (4 * d_t)) & 15;
          fr = fb / KS;
          fc = fb - fr * KS;
        }
        y = fr;
        z = fc;
        tap = fr * KS + fc;
        cc = d_f0 + cc_[ii];
      }
      const unsigned x = 4u * (unsigned)(cc * HW + y * W + z);
#pragma unroll
      for (int j = 0; j < J; ++j) {
        if constexpr (G::BD) {
          const bool ok = __builtin_amdgcn_ubfe(tmask[j], tap, 1) != 0;
          const unsigned off = ok ? vbase[j] + x : 0x80000000u;
          const unsigned row = lds0 + 4u * (unsigned)((bs - smem) + ((wu * KI + ii) * BN + 16 * j) * 4);
          unsigned keep;
          // (a copy: an asm operand alone does not make the generic lambda
          // capture rsrc)
          const __amdgpu_buffer_rsrc_t rs = rsrc;
          asm volatile(
              "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
              "buffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
              : "=&s"(keep)
              : "v"(off), "s"(rs), "s"(row)
              : "memory");
        } else {
#if defined(TNS_CT4_DIAG) && (TNS_CT4_DIAG & 1)
          rb[ii][j] = (float)(x + j);  // diagnostic build: no B loads (timing only)
#else
          const bool ok = __builtin_amdgcn_ubfe(tmask[j], tap, 1) != 0;
          const unsigned off = ok ? vbase[j] + x : 0x80000000u;
          rb[ii][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0));
#endif
        }
      }
    }
  };
  // slot (row 4g + r, column n), component q
  int b_dst[KI];
#pragma unroll
  for (int ii = 0; ii < KI; ++ii) b_dst[ii] = (w * KI + ii) * BN * 4 + r16 * 4 + q;
  auto store_b = [&](float* bs, auto SET) {
    auto& rb = rbs[decltype(SET)::value];
#if defined(TNS_CT4_DIAG) && (TNS_CT4_DIAG & 2)
    return;  // diagnostic build: no B stores (timing only)
#endif
    if constexpr (G::BW) {
#pragma unroll
      for (int ii = 0; ii < KI; ++ii)
#pragma unroll
        for (int c = 0; c < G::CH; ++c)
          if (64 * (c + 1) <= BN || 64 * c + lane < BN)
            *reinterpret_cast<floatx4*>(bs + ((wu * KI + ii) * BN + 64 * c + lane) * 4) = rw[ii][c];
    } else if constexpr (G::AT) {
#pragma unroll
      for (int ii = 0; ii < KI; ++ii) {
        // slot row w*KI + ii: fragment j's 64 dwords at row start + 256 j bytes
        const unsigned base = lds0 + 4u * (unsigned)((bs - smem) + (wu * KI + ii) * BN * 4);
        if (base < 65536u - 256u * J)
          cfor<0, J>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            st_addtid<256 * j>(rb[ii][j], base);
          });
        else
          cfor<0, J>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            st_addtid<32768 + 256 * j>(rb[ii][j], base - 32768u);
          });
      }
    } else if constexpr (!G::BD) {  // (BD: landed by the DMA)
#pragma unroll
      for (int ii = 0; ii < KI; ++ii)
#pragma unroll
        for (int j = 0; j < J; ++j) bs[b_dst[ii] + 64 * j] = rb[ii][j];
    }
  };

  // ---- A staging (weights [M][K]): unit = k-quad kq4 of row m; its four
  // values go to rows 4g + 0..3, component i = kq4 & 3 (g = kq4 >> 2) --------
  // (TA, A = [K][M]: unit = slot (row 4g + q, column m), the values of
  // k = 16g + 4i + q for i = 0..3, lanes along m)
  const float* a_src[AU];
  int a_dst[AU];
#pragma unroll
  for (int u = 0; u < AU; ++u) {
    const int idx = tid + G::NT * u;
    if constexpr (G::TA) {
      const int m = idx % BM, row = idx / BM;
      a_src[u] = p.A + (int64_t)(16 * (row >> 2) + (row & 3)) * p.lda + m0 + m;
      a_dst[u] = (row * BM + m) * 4;
    } else if constexpr (G::ATA) {
      // unit u of wave w: group g and 16-row block mb, lane = (row, component i)
      const int pair = u * G::NW + w, g = pair / (BM / 16), mb = 16 * (pair % (BM / 16));
      const int m = mb + (lane >> 2), i = lane & 3;
      a_src[u] = p.A + (m0 + m) * p.lda + 16 * g + 4 * i;
      a_dst[u] = ((4 * g) * BM + mb) * 4;  // slot row 4g + c: + c * BM * 4 (in floats)
    } else {
      // 8 k-quads of one row per 8 lanes (128 contiguous bytes per row)
      const int lo = idx & 7, rest = idx >> 3;
      const int m = rest % BM, kq4 = lo + 8 * (rest / BM);
      a_src[u] = p.A + (m0 + m) * p.lda + 4 * kq4;
      a_dst[u] = (4 * (kq4 >> 2)) * BM * 4 + m * 4 + (kq4 & 3);
    }
  }
  float4 ras[G::PF ? 2 : 1][AU];  // (unused with AP)
  auto load_a = [&](int k0, float* as, auto SET) {
    auto& ra = ras[decltype(SET)::value];
    if constexpr (G::AP) {
#pragma unroll
      for (int u = 0; u < G::ADM; ++u) {
        const int idx = wu * G::ADM + u, R = idx / (BM / 64), c = idx % (BM / 64);
        const float* src = p.A + ((int64_t)(k0 / 4 + R) * p.M + m0 + 64 * c + lane) * 4;
        const unsigned dst = lds0 + 4u * (unsigned)((as - smem) + (R * BM + 64 * c) * 4);
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src), "s"(dst)
            : "memory");
      }
      return;
    } else {
      (void)as;
    }
#if defined(TNS_CT4_DIAG) && (TNS_CT4_DIAG & 4)
    for (int u = 0; u < AU; ++u) ra[u] = make_float4(k0, k0 + 1, k0 + 2, k0 + 3);
    return;  // diagnostic build: no A loads (timing only)
#endif
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      if constexpr (G::TA) {
        const float* q0 = a_src[u] + (int64_t)k0 * p.lda;
        ra[u] = make_float4(q0[0], q0[4 * p.lda], q0[8 * p.lda], q0[12 * p.lda]);
      } else {
        ra[u] = *reinterpret_cast<const float4*>(a_src[u] + k0);
      }
    }
  };
  auto store_a = [&](float* as, auto SET) {
    auto& ra = ras[decltype(SET)::value];
    if constexpr (G::AP) return;  // (landed by the DMA)
#if defined(TNS_CT4_DIAG) && (TNS_CT4_DIAG & 8)
    return;  // diagnostic build: no A stores (timing only)
#endif
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      if constexpr (G::TA) {
        *reinterpret_cast<float4*>(as + a_dst[u]) = ra[u];
      } else if constexpr (G::ATA) {
        const float v[4] = {ra[u].x, ra[u].y, ra[u].z, ra[u].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const unsigned base =
              lds0 + 4u * (unsigned)((as - smem) + __builtin_amdgcn_readfirstlane(a_dst[u]) + c * BM * 4);
          if (base < 65536u)
            st_addtid<0>(v[c], base);
          else
            st_addtid<32768>(v[c], base - 32768u);
        }
      } else {
        as[a_dst[u]] = ra[u].x;
        as[a_dst[u] + BM * 4] = ra[u].y;
        as[a_dst[u] + 2 * BM * 4] = ra[u].z;
        as[a_dst[u] + 3 * BM * 4] = ra[u].w;
      }
    }
  };

  // ---- MFMA: group g, step i consumes k = 16g + 4i + q; the main loop and
  // epilogue for a wave of JW fragments from fragment column coff ------------
  auto run = [&](auto JWC, const int coff) {
  constexpr int JW = decltype(JWC)::value;
  floatx4 acc[JW];
#pragma unroll
  for (int j = 0; j < JW; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // (DX) the image pixels' running sums, state.delta on entry, and the
  // columns' tap masks; a tap's chains are added at its last k-tile
  floatx4 rs[G::DX ? JW : 1];
  unsigned omask[G::DX ? JW : 1];
  int fl_cnt = 0, fl_tap = 0;
  const int fl_tiles = G::DX ? F_ / BK : 0;
  if constexpr (G::DX) {
    const int64_t row0 = m0 + wm * 16 + 4 * q;
#pragma unroll
    for (int j = 0; j < JW; ++j) {
      const int n = n0 + coff * 16 + 16 * j + r16, nc = n < N ? n : N - 1;
      unsigned vb;
      col_geo(n, vb, omask[j]);
      const int img = nc / p.conv_ohw, pix = dx_pix(nc - img * p.conv_ohw);
      const float* cp = p.C + (int64_t)img * p.strideC + pix + row0 * p.ldc;
#pragma unroll
      for (int e = 0; e < 4; ++e) rs[j][e] = cp[e * p.ldc];
    }
  }
  auto flush = [&]() {
    if (++fl_cnt < fl_tiles) return;
    fl_cnt = 0;
    // reference tap fl_tap's forward-window bit (a class: its tap table)
    const int bit = p.dx_cls ? (p.dx_taps >> (4 * fl_tap)) & 15 : KS * KS - 1 - fl_tap;
    ++fl_tap;
#pragma unroll
    for (int j = 0; j < JW; ++j) {
      const bool ok = __builtin_amdgcn_ubfe(omask[j], bit, 1) != 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) rs[j][e] = ok ? rs[j][e] + acc[j][e] : rs[j][e];
      acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };
  using Frag = Frag4<JW>;
  auto frag = [&](int stg, int g, Frag& f) {
    const float* ap = a_st(stg) + ((4 * g + q) * BM + wm * 16 + r16) * 4;
    f.a = *reinterpret_cast<const floatx4*>(ap);
    const float* bp = b_st(stg) + ((4 * g + q) * BN + coff * 16 + r16) * 4;
#pragma unroll
    for (int j = 0; j < JW; ++j) f.b[j] = *reinterpret_cast<const floatx4*>(bp + 64 * j);
  };
  auto mma = [&](const Frag& f) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < JW; ++j)
        if constexpr (G::AT)  // (transposed tile: rows = pixels, columns = filters)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.b[j][i], f.a[i], acc[j], 0, 0, 0);
        else
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[i], f.b[j][i], acc[j], 0, 0, 0);
  };

#ifdef TNS_CT4_STAMPS
  // diagnostic build only: per-phase cycle sums of wave 0 (tile top / groups
  // before the stores / stores / up to the barrier / last group)
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0}, tl = __builtin_amdgcn_s_memtime();
  const unsigned long long tk0 = tl, rt0 = __builtin_amdgcn_s_memrealtime();
#define TNS_PH(i)                                                   \
  do {                                                              \
    const unsigned long long tn_ = __builtin_amdgcn_s_memtime();    \
    ph[i] += tn_ - tl;                                              \
    tl = tn_;                                                       \
  } while (0)
#else
#define TNS_PH(i) \
  do {            \
  } while (0)
#endif
  const int nt = K / BK;
  Frag f0, f1;
  if (nt > 0) {
    load_a(0, a_st(0), S0{});
    gather_b(b_st(0), S0{});
    if constexpr (G::PF) {  // (tile 1 into set 1, in flight past the barrier)
      if (nt > 1) {
        advance();
        load_a(BK, nullptr, S1{});
        gather_b(nullptr, S1{});
      }
    }
    store_a(a_st(0), S0{});
    store_b(b_st(0), S0{});
    if constexpr (G::BD || G::AP) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (G::AT) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (asm stores)
    __syncthreads();
    frag(0, 0, f0);
  }
  auto tile = [&](int t, auto MORE, auto PAR) {
    constexpr bool more = decltype(MORE)::value;
    // (PF) tile t's set parity: the loads of tile t+2 go into set PAR at
    // the top, the stores of tile t+1 come from set PAR ^ 1
    constexpr int par = decltype(PAR)::value;
    using SL = std::integral_constant<int, G::PF ? par : 0>;
    using SS = std::integral_constant<int, G::PF ? par ^ 1 : 0>;
    const int tc = t & 1, tx = (t + 1) & 1;
    TNS_PH(5);
    if constexpr (more && G::PF && !G::IL) {
      // (unconditional: past the last tile the weight rows' k is clamped
      // and the gather's offsets run past the images' range — read, unused)
      advance();
      load_a(min((t + 2) * BK, K - BK), nullptr, SL{});
      gather_b(nullptr, SL{});
      __builtin_amdgcn_sched_barrier(0);  // keep the loads at the top of the tile
    } else if constexpr (more && !G::IL && !G::ST && !G::PF) {
      advance();
      if constexpr (G::BD) {
        gather_b(b_st(tx), S0{});
        load_a((t + 1) * BK, a_st(tx), S0{});
      } else {
        load_a((t + 1) * BK, a_st(tx), S0{});
        gather_b(b_st(tx), S0{});
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the loads at the top of the tile
    }
    TNS_PH(0);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      Frag& fc = (g & 1) ? f1 : f0;
      Frag& fn = (g & 1) ? f0 : f1;
      if constexpr (more)
        if (g == NG - 1) {
          // every wave's stores of tile t+1 are in; its first group is read
          // under this group's MFMAs
          TNS_PH(3);
          if constexpr (G::BD || G::AP) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if constexpr (G::AT) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (asm stores)
#ifdef TNS_CT4_STAMPS
          // every wave's arrival at tile 8's barrier (words 16 + w, realtime
          // ticks after block entry) — who the barrier waits for
          if (t == 8 && lane == 0 && p.stamps != nullptr && blockIdx.x < (1u << 16) && w < 16)
            p.stamps[32 * blockIdx.x + 16 + w] =
                (unsigned)(__builtin_amdgcn_s_memtime() & 0xffffffffu);
#endif
          __syncthreads();
          TNS_PH(4);
        }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (more && G::ST)
        if (g < 2 && half == g) {
          advance();
          load_a((t + 1) * BK, a_st(tx), S0{});
          gather_b(b_st(tx), S0{});
          __builtin_amdgcn_sched_barrier(0);
        }
      // one scheduling region per group: the next group's fragment reads,
      // interleaved staging (LI / SI) and this group's MFMAs
      const bool reads = g + 1 < NG || more;
      if (g + 1 < NG)
        frag(tc, g + 1, fn);
      else if (more)
        frag(tx, 0, fn);
      if constexpr (more && G::IL) {
        if (g == 0) {
          advance();
          if constexpr (G::PF) {  // (tile t+2 into this tile's set, as above)
            load_a(min((t + 2) * BK, K - BK), nullptr, SL{});
            gather_b(nullptr, SL{});
          } else {
            load_a((t + 1) * BK, a_st(tx), S0{});
            gather_b(b_st(tx), S0{});
          }
        }
      }
      if constexpr (more && G::SI) {
        if (g == G::SG) {
          store_a(a_st(tx), SS{});
          store_b(b_st(tx), SS{});
        }
      }
      mma(fc);
      if constexpr (G::RI > 0 || G::IL > 0 || G::SI) {
#pragma unroll
        for (int i = 0; i < 4 * JW; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
          if constexpr (G::RI > 0)
            if (reads && i % G::RI == 0 && i / G::RI < JW + 1)
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // a fragment read
          if constexpr (more && G::IL > 0)
            if (g == 0) {
              __builtin_amdgcn_sched_group_barrier(0x002, G::IL, 0);  // IL VALU
              if (i < AU + G::BLD) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // a load
            }
          if constexpr (more && G::SI)
            if (g == G::SG && i < G::AST + G::BST)
              __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // a store
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (more && G::ST)
        if (g >= G::SG && g <= G::SG + 1 && g == G::SG + half) {
          store_a(a_st(tx), S0{});
          store_b(b_st(tx), S0{});
          __builtin_amdgcn_sched_barrier(0);
        }
      if constexpr (more && !G::SI && !G::ST)
        if (g == G::SG) {
          TNS_PH(1);
          store_a(a_st(tx), SS{});
          store_b(b_st(tx), SS{});
          __builtin_amdgcn_sched_barrier(0);
          TNS_PH(2);
        }
    }
    if constexpr (G::DX) flush();
  };
  static_assert(NG % 2 == 0, "f0 holds group 0 at every tile start");
  if constexpr (G::PF) {  // (tile pairs: the set parity a compile-time constant)
    int t = 0;
    for (; t + 2 < nt; t += 2) {
      tile(t, std::true_type{}, S0{});
      tile(t + 1, std::true_type{}, S1{});
    }
    if (t + 1 < nt) {
      tile(t, std::true_type{}, S0{});
      tile(t + 1, std::false_type{}, S1{});
    } else if (t < nt) {
      tile(t, std::false_type{}, S0{});
    }
  } else {
    for (int t = 0; t + 1 < nt; ++t) tile(t, std::true_type{}, S0{});
    if (nt > 0) tile(nt - 1, std::false_type{}, S0{});
  }

#ifdef TNS_CT4_STAMPS
  TNS_PH(5);
  if (tid == 0 && p.stamps != nullptr && blockIdx.x < (1u << 16)) {
    unsigned* st = p.stamps + 32 * blockIdx.x;
    for (int i = 0; i < 6; ++i) st[i] = (unsigned)ph[i];
    st[6] = (unsigned)(tl - tk0);
    const unsigned long long rt_loop = __builtin_amdgcn_s_memrealtime();
    st[7] = (unsigned)nt | (unsigned)(rt_loop - rt0) << 8;
    // (realtime, 100 MHz: block entry, loop start, loop end; the epilogue's
    // end in word 11, written below)
    st[8] = (unsigned)rt_entry;
    st[9] = (unsigned)(rt_entry >> 32);
    st[10] = (unsigned)(rt0 - rt_entry);
    st[12] = (unsigned)(rt_loop - rt_entry);
  }
#endif
#undef TNS_PH
  // ---- epilogue: forwardBias + activate, conv output [img][filter][pixel] --
  const bool fuse = p.epi == EPI_BIAS_ACT;
  const int act = p.act;
  if constexpr (G::AT) {
    // the MFMAs ran with the operands swapped (same products, same k order:
    // bit-identical): lane (r16, q) holds filter m0 + wm*16 + r16 at the four
    // consecutive pixels 16j + 4q + e, one 16-byte store where they are in
    // one image (every image's pixel count a multiple of 4)
    const int64_t row = m0 + wm * 16 + r16;
    const float bi = fuse ? p.bias[row] : 0.0f;
    const bool v4 = (p.conv_ohw & 3) == 0 && (p.strideC & 3) == 0 && (p.ldc & 3) == 0 &&
                    (reinterpret_cast<uintptr_t>(p.C) & 15) == 0;
#pragma unroll
    for (int j = 0; j < JW; ++j) {
      const int nb = n0 + coff * 16 + 16 * j + 4 * q;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fuse ? act_apply_cheap(acc[j][e] + bi, act) : acc[j][e];
      if (v4) {
        if (nb < N) {
          const int img = nb / p.conv_ohw, pix = nb - img * p.conv_ohw;
          *reinterpret_cast<float4*>(p.C + (int64_t)img * p.strideC + pix + row * p.ldc) =
              make_float4(v[0], v[1], v[2], v[3]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = nb + e;
          if (n < N) {
            const int img = n / p.conv_ohw, pix = n - img * p.conv_ohw;
            p.C[(int64_t)img * p.strideC + pix + row * p.ldc] = v[e];
          }
        }
      }
    }
    return;
  }
  if constexpr (G::DX) {
    const int64_t row0 = m0 + wm * 16 + 4 * q;
#pragma unroll
    for (int j = 0; j < JW; ++j) {
      const int n = n0 + coff * 16 + 16 * j + r16;
      if (n >= N) continue;
      const int img = n / p.conv_ohw, pix = dx_pix(n - img * p.conv_ohw);
      float* cp = p.C + (int64_t)img * p.strideC + pix + row0 * p.ldc;
#pragma unroll
      for (int e = 0; e < 4; ++e) cp[e * p.ldc] = rs[j][e];
    }
    return;
  }
  const bool add = p.epi == EPI_ADD;  // dX of a 1x1 layer: col2im fused (C += col)
  const int64_t row0 = m0 + wm * 16 + 4 * q;
  float bias[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) bias[e] = fuse ? p.bias[row0 + e] : 0.0f;
#pragma unroll
  for (int j = 0; j < JW; ++j) {
    const int n = n0 + coff * 16 + 16 * j + r16;
    if (n >= N) continue;
    const int img = n / p.conv_ohw, pix = n - img * p.conv_ohw;
    float* cp = p.C + (int64_t)img * p.strideC + pix + row0 * p.ldc;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = acc[j][e];
      if (fuse) v = act_apply_cheap(v + bias[e], act);
      if (add) v = cp[e * p.ldc] + v;
      cp[e * p.ldc] = v;
    }
  }
#ifdef TNS_CT4_STAMPS
  if (tid == 0 && p.stamps != nullptr && blockIdx.x < (1u << 16)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (this wave's stores done)
    p.stamps[32 * blockIdx.x + 11] = (unsigned)(__builtin_amdgcn_s_memrealtime() - rt_entry);
  }
#endif
  };
  if constexpr (G::NA == G::WN) {
    run(std::integral_constant<int, G::JA>{}, wn * G::JA);
  } else {
    if (__builtin_amdgcn_readfirstlane(wn) < G::NA)
      run(std::integral_constant<int, G::JA>{}, wn * G::JA);
    else
      run(std::integral_constant<int, G::JB>{}, G::NA * G::JA + (wn - G::NA) * G::JB);
  }
}

#ifdef TNS_CT4_STAMPS
unsigned* g_ct4_stamps = nullptr;
#endif

template <class G>
hipError_t launch_g4(const GemmArgs& a_in, int ks, int dil, hipStream_t s) {
  GemmArgs a = a_in;
#ifdef TNS_CT4_STAMPS
  a.stamps = g_ct4_stamps;
#endif
  if (a.M % G::BM || a.K % G::BK || a.K <= 0) return hipErrorInvalidValue;
  if (!G::TA && (a.lda % 4 || (reinterpret_cast<uintptr_t>(a.A) & 15))) return hipErrorInvalidValue;
  if (G::TA && (a.lda < a.M || a.K * a.lda > 0x7fffffffLL)) return hipErrorInvalidValue;
  const int64_t tiles = (a.M / G::BM) * ((a.N + G::BN - 1) / G::BN);
  if (tiles > 0x7fffffff || a.N > 0x7fffffff || a.K > 0x7fffffff) return hipErrorInvalidValue;
  if (ks == 3)
    hipLaunchKernelGGL((conv_tile4_kernel<G, 3>), dim3((unsigned)tiles), dim3(G::NT), 0, s, a, dil);
  else if (ks == 1)
    hipLaunchKernelGGL((conv_tile4_kernel<G, 1>), dim3((unsigned)tiles), dim3(G::NT), 0, s, a, dil);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

struct TileInfo4 {
  int bm, bn, bk;
  hipError_t (*fn)(const GemmArgs&, int, int, hipStream_t);
  const char* name;
};
#define TNS_CT4(BMv, BNv, WMv, WNv, BKv, SGv, ILv, SIv, RIv, STv)                      \
  {BMv, BNv, BKv, launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, ILv, SIv, RIv, STv>>,    \
   "conv_tile4<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",il" #ILv ",si" #SIv \
   ",ri" #RIv ",st" #STv ">"}
#define TNS_CT4U(BMv, BNv, WMv, WNv, BKv, SGv, SIv, RIv, JAv, NAv)                      \
  {BMv, BNv, BKv, launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, 0, SIv, RIv, false, JAv, NAv>>, \
   "conv_tile4<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",si" #SIv ",ri" #RIv    \
   ",j" #JAv "x" #NAv ">"}
#define TNS_CT4D(BMv, BNv, WMv, WNv, BKv, SGv, SIv, RIv, BDv, BWv)                          \
  {BMv, BNv, BKv,                                                                            \
   launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, 0, SIv, RIv, false, 0, 0, false, BDv, BWv>>, \
   "conv_tile4<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",si" #SIv ",ri" #RIv    \
   ",bd" #BDv ",bw" #BWv ">"}
#define TNS_CT4UD(BMv, BNv, WMv, WNv, BKv, SGv, SIv, RIv, JAv, NAv, BDv, BWv)                 \
  {BMv, BNv, BKv,                                                                              \
   launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, 0, SIv, RIv, false, JAv, NAv, false, BDv, BWv>>, \
   "conv_tile4<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",si" #SIv ",ri" #RIv      \
   ",j" #JAv "x" #NAv ",bd" #BDv ",bw" #BWv ">"}
#define TNS_CT4A(BMv, BNv, WMv, WNv, BKv, SGv, SIv, RIv, JAv, NAv)                                 \
  {BMv, BNv, BKv,                                                                                \
   launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, 0, SIv, RIv, false, JAv, NAv, false, false, false, \
                  true>>,                                                                        \
   "conv_tile4_ap<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",si" #SIv ",ri" #RIv      \
   ",j" #JAv "x" #NAv ">"}
#define TNS_CT4X(BMv, BNv, WMv, WNv, BKv, SGv, RIv, JAv, NAv)                                  \
  {BMv, BNv, BKv,                                                                             \
   launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, 0, false, RIv, false, JAv, NAv, false, false, \
                  false, false, true>>,                                                       \
   "conv_tile4_at<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",ri" #RIv ",j" #JAv   \
   "x" #NAv ">"}
#define TNS_CT4P(BMv, BNv, WMv, WNv, BKv, SGv, SIv, RIv, JAv, NAv)                           \
  {BMv, BNv, BKv,                                                                             \
   launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, 0, SIv, RIv, false, JAv, NAv, false, false,  \
                  false, false, false, false, true>>,                                        \
   "conv_tile4_pf<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",si" #SIv ",ri" #RIv \
   ",j" #JAv "x" #NAv ">"}
#define TNS_CT4PI(BMv, BNv, WMv, WNv, BKv, SGv, ILv, SIv, RIv, JAv, NAv)                     \
  {BMv, BNv, BKv,                                                                             \
   launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, ILv, SIv, RIv, false, JAv, NAv, false, false, \
                  false, false, false, false, true>>,                                        \
   "conv_tile4_pf<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",il" #ILv ",si" #SIv  \
   ",ri" #RIv ",j" #JAv "x" #NAv ">"}
const TileInfo4 kTiles4[] = {
    TNS_CT4(128, 176, 8, 1, 32, 0, 0, false, 0, false),  // 0
    TNS_CT4(128, 176, 8, 1, 64, 2, 0, false, 0, false),  // 1
    TNS_CT4(128, 176, 8, 1, 64, 1, 0, true, 3, false),   // 2: stores and reads interleaved
    TNS_CT4(128, 176, 8, 1, 64, 1, 0, true, 2, false),   // 3
    TNS_CT4(128, 176, 8, 1, 64, 1, 0, false, 3, true),   // 4: staggered halves
    TNS_CT4(128, 176, 8, 1, 64, 1, 0, false, 0, true),   // 5
    TNS_CT4(128, 176, 8, 1, 64, 1, 0, false, 2, true),   // 6
    TNS_CT4(64, 96, 4, 1, 32, 0, 0, false, 0, false),    // 7
    TNS_CT4(64, 96, 4, 1, 32, 0, 0, false, 3, false),    // 8
    TNS_CT4(64, 192, 4, 2, 64, 1, 0, false, 3, true),    // 9
    TNS_CT4(64, 96, 4, 2, 64, 1, 0, false, 3, true),     // 10
    // multi-block tiles for the 512 / 1024-filter layers (26^2, 13^2 planes)
    TNS_CT4(64, 64, 4, 2, 32, 0, 0, false, 0, false),    // 11
    TNS_CT4(64, 64, 4, 1, 32, 0, 0, false, 0, false),    // 12
    TNS_CT4(64, 32, 4, 1, 32, 0, 0, false, 0, false),    // 13
    TNS_CT4(64, 32, 4, 2, 32, 0, 0, false, 0, false),    // 14
    TNS_CT4(64, 64, 4, 1, 64, 2, 0, false, 0, false),    // 15
    TNS_CT4(64, 32, 4, 1, 64, 2, 0, false, 0, false),    // 16
    // uneven wave columns: 26^2 (8 x 31 blocks of 64 x 176), 13^2 (32 x 8 of 32 x 176)
    TNS_CT4U(64, 176, 4, 2, 64, 1, true, 2, 6, 1),       // 17
    TNS_CT4U(64, 176, 4, 2, 32, 0, false, 3, 6, 1),      // 18
    TNS_CT4U(32, 176, 2, 4, 64, 1, true, 2, 3, 3),       // 19
    // 13^2 planes (N = 1352): 8 x 29 blocks of 128 x 48 (1024 filters), 8 x 29 of 64 x 48 (512)
    TNS_CT4(128, 48, 8, 1, 32, 0, 0, false, 3, false),   // 20
    TNS_CT4(128, 48, 8, 1, 64, 1, 0, true, 2, false),    // 21
    TNS_CT4(64, 48, 4, 1, 32, 0, 0, false, 3, false),    // 22
    TNS_CT4(64, 48, 4, 1, 64, 1, 0, true, 2, false),     // 23
    TNS_CT4(128, 96, 8, 1, 64, 1, 0, true, 2, false),    // 24
    // round 5, loads two tiles ahead (PF: two register sets, tile pairs
    // unrolled) — the picked ones (profiles/r05_conv_fwd_sweep.json)
    TNS_CT4P(64, 32, 4, 1, 32, 0, false, 0, 0, 0),       // 25 (13: 26^2 1x1 layers)
    TNS_CT4PI(64, 176, 4, 2, 32, 0, 2, false, 3, 6, 1),  // 26 (18 + loads interleaved: stride 2)
    TNS_CT4PI(64, 176, 4, 2, 32, 0, 0, true, 3, 6, 1),   // 27 (18 + stores interleaved: stride 1)
#ifdef TNS_DIAG_KERNELS  // (diagnostics build only: measured, not picked)
    // PF forms measured and not picked (sweeps: profiles/r05_conv_fwd_sweep.json):
    // 26^2 0.1296 (PF alone) / 0.1311 (IL + SI) / 0.1273 (64-deep) against
    // 0.1268 for 27; 13^2 0.141 / 0.143 / 0.136 against 0.134 for 21; the
    // 64-deep 128 x 176 PF form spills, the 32-deep ones 2-3 % behind 3
    TNS_CT4P(64, 176, 4, 2, 32, 0, false, 3, 6, 1),      // 28 (18)
    TNS_CT4P(128, 48, 8, 1, 64, 1, true, 2, 0, 0),       // 29 (21)
    TNS_CT4P(64, 96, 4, 1, 32, 0, false, 3, 0, 0),       // 30 (8)
    TNS_CT4PI(64, 176, 4, 2, 32, 0, 2, true, 3, 6, 1),   // 31 (18, IL + SI)
    TNS_CT4PI(64, 176, 4, 2, 64, 1, 2, true, 2, 6, 1),   // 32 (17, IL + SI)
    TNS_CT4PI(128, 48, 8, 1, 64, 1, 2, true, 2, 0, 0),   // 33 (21, IL + SI)
    TNS_CT4PI(128, 48, 8, 1, 64, 0, 2, true, 2, 0, 0),   // 34 (21, IL + SI in group 0)
    TNS_CT4PI(128, 176, 8, 1, 32, 0, 0, false, 3, 0, 0), // 35 (0, PF)
    TNS_CT4PI(128, 176, 8, 1, 32, 0, 0, true, 3, 0, 0),  // 36 (0, PF + SI)
    TNS_CT4PI(128, 176, 8, 1, 32, 0, 2, false, 3, 0, 0), // 37 (0, PF + IL)
    // B by dword LDS-DMA (BD) / slot-wise (BW): bit-exact, measured slower
    // than the register-staged b32 stores on every class (kept selectable)
    TNS_CT4D(128, 176, 8, 1, 64, 1, true, 2, true, false),          // 38 (3, BD)
    TNS_CT4D(128, 176, 8, 1, 64, 1, true, 2, false, true),          // 39 (3, BW)
    TNS_CT4UD(64, 176, 4, 2, 32, 0, false, 3, 6, 1, false, true),   // 40 (18, BW)
    // A by 16-byte LDS-DMA from the pre-permuted weights (AP): bit-exact,
    // slower on every class measured (52^2 0.114 -> 0.120 ms, 26^2 0.128 ->
    // 0.138, 13^2 0.138 -> 0.155, 1x1 0.021 -> 0.023; permute pass included)
    TNS_CT4A(128, 176, 8, 1, 64, 1, true, 2, 0, 0),                 // 41 (3)
    // B stored by ds_write_addtid_b32 with operands swapped in the MFMA (AT:
    // gather lanes 16 pixels x 4 k, 16-byte epilogue stores), the picked
    // shapes: timed slower on every layer class (profiles/r04_conv_at_sweep.json:
    // 104^2 3x3 0.123 -> 0.137 ms, 52^2 0.117 -> 0.127,
    // 26^2 0.133 -> 0.163, 13^2 0.147 -> 0.218, 1x1 52^2 0.022 -> 0.024) —
    // the gather's 4 k rows per load instruction touch 4x the cache lines
    TNS_CT4X(128, 176, 8, 1, 64, 2, 0, 0, 0),    // 42 (1)
    TNS_CT4X(128, 176, 8, 1, 64, 1, 2, 0, 0),    // 43
    TNS_CT4X(64, 176, 4, 2, 32, 0, 3, 6, 1),     // 44 (18)
    TNS_CT4X(128, 48, 8, 1, 64, 1, 2, 0, 0),     // 45 (21)
    TNS_CT4X(64, 96, 4, 1, 32, 0, 3, 0, 0),      // 46 (8)
    TNS_CT4X(64, 32, 4, 1, 32, 0, 0, 0, 0),      // 47 (13)
    TNS_CT4X(64, 64, 4, 2, 32, 0, 0, 0, 0),      // 48 (11)
#endif
};
// A k-major (TA): col = W^T . delta of the conv backward (conv_tile4_dx_*)
#define TNS_CT4T(BMv, BNv, WMv, WNv, BKv, SGv, SIv, RIv, JAv, NAv)                      \
  {BMv, BNv, BKv,                                                                      \
   launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, 0, SIv, RIv, false, JAv, NAv, true>>,  \
   "conv_tile4_ta<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",si" #SIv     \
   ",ri" #RIv ",j" #JAv "x" #NAv ">"}
#define TNS_CT4TP(BMv, BNv, WMv, WNv, BKv, SGv, SIv, RIv, JAv, NAv)                      \
  {BMv, BNv, BKv,                                                                      \
   launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, 0, SIv, RIv, false, JAv, NAv, true, false, \
                  false, false, false, false, true>>,                                   \
   "conv_tile4_ta_pf<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",si" #SIv   \
   ",ri" #RIv ",j" #JAv "x" #NAv ">"}
const TileInfo4 kTiles4T[] = {
    TNS_CT4T(128, 176, 8, 1, 64, 1, true, 2, 0, 0),   // 0
    TNS_CT4T(128, 96, 8, 1, 64, 1, true, 2, 0, 0),    // 1
    TNS_CT4T(128, 48, 8, 1, 64, 1, true, 2, 0, 0),    // 2
    TNS_CT4T(64, 176, 4, 2, 32, 0, false, 3, 6, 1),   // 3
    TNS_CT4T(64, 96, 4, 1, 32, 0, false, 3, 0, 0),    // 4
    TNS_CT4T(64, 32, 4, 1, 32, 0, false, 0, 0, 0),    // 5
    TNS_CT4T(128, 176, 8, 1, 32, 0, false, 3, 0, 0),  // 6
    TNS_CT4T(64, 64, 4, 2, 32, 0, false, 3, 0, 0),    // 7: multi-block forms for the short-k dX
    TNS_CT4T(64, 64, 4, 1, 32, 0, false, 3, 0, 0),    // 8
    TNS_CT4T(128, 64, 8, 1, 32, 0, false, 3, 0, 0),   // 9
    TNS_CT4T(64, 128, 4, 2, 32, 0, false, 3, 0, 0),   // 10
    // PF twins (operands of tile t+2 loaded at the top of tile t) of 4, 7, 2
    TNS_CT4TP(64, 96, 4, 1, 32, 0, false, 3, 0, 0),   // 11 (4)
    TNS_CT4TP(64, 64, 4, 2, 32, 0, false, 3, 0, 0),   // 12 (7)
    TNS_CT4TP(128, 48, 8, 1, 64, 1, true, 2, 0, 0),   // 13 (2)
};
constexpr int kNumTiles4T = sizeof(kTiles4T) / sizeof(kTiles4T[0]);
// k-major A, tap-major k (DX): state.delta of stride-1 3x3 layers
#define TNS_CT4DX(BMv, BNv, WMv, WNv, BKv, SGv, SIv, RIv, JAv, NAv)                          \
  {BMv, BNv, BKv,                                                                          \
   launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, 0, SIv, RIv, false, JAv, NAv, true, false,  \
                  false, false, false, true>>,                                             \
   "conv_tile4_dx<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",si" #SIv         \
   ",ri" #RIv ",j" #JAv "x" #NAv ">"}
#define TNS_CT4DXP(BMv, BNv, WMv, WNv, BKv, SGv, SIv, RIv, JAv, NAv)                         \
  {BMv, BNv, BKv,                                                                          \
   launch_g4<Geo4<BMv, BNv, WMv, WNv, BKv, SGv, 0, SIv, RIv, false, JAv, NAv, true, false,  \
                  false, false, false, true, true>>,                                       \
   "conv_tile4_dx_pf<" #BMv "x" #BNv "x" #BKv ",w" #WMv "x" #WNv ",g" #SGv ",si" #SIv      \
   ",ri" #RIv ",j" #JAv "x" #NAv ">"}
const TileInfo4 kTiles4DX[] = {
    TNS_CT4DX(64, 176, 4, 2, 32, 0, false, 3, 6, 1),   // 0: >= 52^2 planes
    TNS_CT4DX(64, 96, 4, 1, 32, 0, false, 3, 0, 0),    // 1: 26^2
    TNS_CT4DX(64, 48, 4, 1, 32, 0, false, 3, 0, 0),    // 2: 13^2
    TNS_CT4DX(128, 96, 8, 1, 64, 1, true, 2, 0, 0),    // 3
    TNS_CT4DX(64, 64, 4, 2, 32, 0, false, 3, 0, 0),    // 4
    TNS_CT4DX(128, 48, 8, 1, 64, 1, true, 2, 0, 0),    // 5
    TNS_CT4DX(32, 176, 2, 4, 64, 1, true, 2, 3, 3),    // 6: 32-channel planes (208^2)
    // the same with the operands of tile t+2 loaded at the top of tile t (PF)
    TNS_CT4DXP(64, 176, 4, 2, 32, 0, false, 3, 6, 1),  // 7 (0)
    TNS_CT4DXP(64, 64, 4, 2, 32, 0, false, 3, 0, 0),   // 8 (4)
    TNS_CT4DXP(32, 176, 2, 4, 64, 1, true, 2, 3, 3),   // 9 (6)
    TNS_CT4DXP(64, 48, 4, 1, 32, 0, false, 3, 0, 0),   // 10 (2)
    // (128 x 176: the running sums take it past 256 VGPRs — spills; not built.
    // Eight-wave 64 x 96 / 32 x 96 forms for the 26^2 / 13^2 row counts
    // measured no better than these: 26^2 0.369 / 0.378 ms a call against
    // 0.352 for TN + col2im, 13^2 0.446 / 0.453 against 0.424 — not built)
};
constexpr int kNumTiles4DX = sizeof(kTiles4DX) / sizeof(kTiles4DX[0]);
#undef TNS_CT4DX
#undef TNS_CT4DXP
#undef TNS_CT4
#undef TNS_CT4U
#undef TNS_CT4D
#undef TNS_CT4A
#undef TNS_CT4UD
#undef TNS_CT4X
#undef TNS_CT4T
#undef TNS_CT4TP
#undef TNS_CT4P
#undef TNS_CT4PI
constexpr int kNumTiles4 = sizeof(kTiles4) / sizeof(kTiles4[0]);

}  // namespace

__global__ void permute_weights_kernel(const float* __restrict__ A, float* __restrict__ Ap, int M,
                                       int K, int64_t n) {
  // Ap[((R * M) + m) * 4 + i] = A[m][16 (R >> 2) + 4 i + (R & 3)]
  for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < n;
       o += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(o & 3);
    const int64_t rest = o >> 2;
    const int m = (int)(rest % M), R = (int)(rest / M);
    Ap[o] = A[(int64_t)m * K + 16 * (R >> 2) + 4 * i + (R & 3)];
  }
}

int conv_tile4_count() { return kNumTiles4; }
bool conv_tile4_is_ap(int v) { return v >= 0 && v < kNumTiles4 && std::strstr(kTiles4[v].name, "_ap<"); }
hipError_t conv_tile4_permute(const float* A, float* Ap, int64_t M, int64_t K, hipStream_t s) {
  if (M <= 0 || K % 16 || M * K > 0x7fffffffLL) return hipErrorInvalidValue;
  const int64_t n = M * K;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(permute_weights_kernel, dim3(blocks), dim3(256), 0, s, A, Ap, (int)M, (int)K, n);
  return hipGetLastError();
}
const char* conv_tile4_name(int v) { return v >= 0 && v < kNumTiles4 ? kTiles4[v].name : ""; }
int conv_tile4_bk(int v) { return v >= 0 && v < kNumTiles4 ? kTiles4[v].bk : 0; }

#ifdef TNS_CT4_STAMPS
// diagnostic build only (not in include/tns.h): per-block phase cycle sums
// of wave 0 into dev_buf (32 words per block), or nothing when NULL
extern "C" int tns_debug_ct4_stamps(unsigned* dev_buf) {
  g_ct4_stamps = dev_buf;
  return 0;
}
#endif

int conv_tile4_ta_count() { return kNumTiles4T; }
const char* conv_tile4_ta_name(int v) { return v >= 0 && v < kNumTiles4T ? kTiles4T[v].name : ""; }

// col_b = W^T . delta_b for every image b at once: a 1x1 stride-1 "conv"
// whose images are the delta planes (oh x ow, `filters` channels) and whose
// weights are W read k-major; same chains as the TN GEMM (each col element an
// ascending-f fma chain from +0).  Form by measured shape, -1: none applies.
// Measured (scripts/conv_bwd_layers.py, profiles/r03_conv_tile4.json): ahead
// of the TN GEMM on the 13^2 planes only (1x1 layers 0.222 -> 0.155 ms per
// 7 calls, 3x3 1.197 -> 1.180); behind it on the 26^2 .. 104^2 planes, whose
// TN tiles balance better (26^2 3x3 1.48 -> 1.65 with the 128 x 96 form).
// Round 4 (scripts/bwd_sweep.py --what dx, whole backward calls with
// state.delta; profiles/r04_bwd_dx_forms2.json, r04_bwd_dx_forms4.json):
// 3x3 layers on the 13^2 planes take the 64 x 96 form (layer 45 0.440 ->
// 0.397 ms, stride-2 layer 43 0.450 -> 0.407), the stride-2 208^2 -> 104^2
// layer 64 x 64 (0.552 -> 0.501); the 1x1 layers (the product added into
// state.delta in the epilogue) 128 x 48 on the 13^2 planes (0.087 -> 0.080)
// and 64 x 64 on the 26^2 / 52^2 ones (0.079 -> 0.075 at 26^2).
int conv_tile4_dx_pick(int64_t M, int64_t N, int64_t K, int64_t ks) {
#ifndef TNS_CT4_TA_NO_PF
  // the 13^2 planes (N < 4096) on the PF twin of 7: whole pipelined backward
  // 14.80 -> 14.66 ms, joined 17.13 -> 17.11 (scripts/bwd_graph.py, same box,
  // two rounds; profiles/r05_bwd_schedules.json).  The 1x1 layers on those
  // planes are included on purpose (before: form 2, 128 x 48): the A/B was
  // of the whole pass with both kinds switched together
  if (N < 4096 && K % 32 == 0 && M % 64 == 0) return 12;
#endif
  if (ks == 1) {
    if (N >= 4096) return (M % 64 == 0 && K % 32 == 0) ? 7 : -1;
    return (K % 64 == 0 && M % 128 == 0) ? 2 : -1;
  }
  if (K % 32 == 0 && M % 64 == 0) {
    if (N < 4096) return 4;
    if (N >= 50000) return 8;
  }
  return -1;
}

hipError_t launch_conv_tile4_dx(int v, const float* w, const float* delta, float* col,
                                int64_t batch, int64_t C, int64_t ks, int64_t F, int64_t oh,
                                int64_t ow, hipStream_t s, bool add_into) {
  if (v < 0 || v >= kNumTiles4T) return hipErrorInvalidValue;
  if (add_into && ks != 1) return hipErrorInvalidValue;
  const int64_t M = C * ks * ks, hw = oh * ow;
  if (batch * F * hw * 4 > 0x7fffffffLL || batch * hw > 0x7fffffffLL) return hipErrorInvalidValue;
  GemmArgs a{};
  a.M = M; a.N = batch * hw; a.K = F;
  a.alpha = 1.0f; a.beta = 0.0f; a.beta_mode = BETA_ZERO;
  a.A = w; a.lda = M; a.strideA = 0;
  a.B = delta; a.ldb = hw; a.strideB = F * hw;
  a.C = col; a.ldc = hw; a.strideC = M * hw;
  a.batch = 1; a.epi = add_into ? EPI_ADD : EPI_NONE; a.bias = nullptr; a.act = 0;
  a.conv = 2;
  a.conv_H = (int)oh; a.conv_W = (int)ow; a.conv_ow = (int)ow; a.conv_ohw = (int)hw;
  a.conv_sY = 1; a.conv_sX = 1; a.conv_pH = 0; a.conv_pW = 0;
  a.conv_bytes = (int)(4 * batch * F * hw);
  return kTiles4T[v].fn(a, 1, 1, s);
}

int conv_tile4_dx3_count() { return kNumTiles4DX; }
const char* conv_tile4_dx3_name(int v) { return v >= 0 && v < kNumTiles4DX ? kTiles4DX[v].name : ""; }

namespace {
// the launcher's conditions: stride 1, dilation 1, 3x3, pad <= 2, 32-bit
// offsets, F a multiple of the form's k-tile, C of its row tile
bool dx3_fits(int v, int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F, int64_t ks,
              int64_t pad, int64_t oh, int64_t ow) {
  if (v < 0 || v >= kNumTiles4DX || ks != 3 || pad < 0 || pad > ks - 1) return false;
  if (oh != H + 2 * pad - ks + 1 || ow != W + 2 * pad - ks + 1 || oh <= 0 || ow <= 0) return false;
  if (F % kTiles4DX[v].bk || C % kTiles4DX[v].bm || batch <= 0) return false;
  return batch * F * oh * ow * 4 <= 0x7fffffffLL && batch * C * H * W <= 0x7fffffffLL &&
         ks * ks * F * C <= 0x7fffffffLL;
}
}  // namespace

// by plane size.  Measured per YOLOv3 layer (scripts/bwd_sweep.py --what dx,
// whole backward calls at batch 8, profiles/r04_bwd_dx_forms.json): ahead of the
// col = W^T . delta product + col2im on the 104^2 planes (64 x 64 tiles,
// 0.453 -> 0.413 ms a call) and the 52^2 planes (64 x 176: 0.385 -> 0.368 in
// a second sweep, profiles/r04_bwd_dx_forms2.json);
// level on 26^2 (0.339 vs 0.341) and behind on 13^2 (0.44 -> 0.49 and
// worse: too few pixels per filter tap for the per-tap tiles), so not there
int conv_tile4_dx3_pick(int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F, int64_t ks,
                        int64_t pad) {
  const int64_t N = batch * H * W, oh = H + 2 * pad - ks + 1, ow = W + 2 * pad - ks + 1;
  // Round 5: the PF twins (forms 7..10) measured 1-4 % faster a call on
  // the 104^2 / 52^2 / stride-2 208^2 planes (scripts/bwd_sweep.py --what dx,
  // profiles/r05_bwd_dx_sweep.json) but level-to-slower over the pipelined
  // 75-layer pass, where they run beside the pending dW products (14.70 /
  // 14.72 -> 14.82 / 14.80 ms, joined 17.03 / 17.01 -> 16.94 / 16.97;
  // profiles/r05_bwd_schedules.json): not picked
  int v = -1;
  if (C % 64 && N >= 50000)
    v = 6;
  else if (N >= 50000)
    v = 4;
  else if (N >= 16384)
    v = 0;
  return v >= 0 && dx3_fits(v, batch, C, H, W, F, ks, pad, oh, ow) ? v : -1;
}

hipError_t launch_conv_tile4_dx3(int v, const float* wt, const float* delta, float* im,
                                 int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F,
                                 int64_t ks, int64_t pad, int64_t oh, int64_t ow, hipStream_t s) {
  if (!dx3_fits(v, batch, C, H, W, F, ks, pad, oh, ow)) return hipErrorInvalidValue;
  GemmArgs a{};
  a.M = C; a.N = batch * H * W; a.K = ks * ks * F;
  a.alpha = 1.0f; a.beta = 0.0f; a.beta_mode = BETA_ZERO;
  a.A = wt; a.lda = C; a.strideA = 0;
  a.B = delta; a.ldb = oh * ow; a.strideB = F * oh * ow;
  a.C = im; a.ldc = H * W; a.strideC = C * H * W;
  a.batch = 1; a.epi = EPI_NONE; a.bias = nullptr; a.act = 0;
  a.conv = 2;
  // the forward window over the delta planes, padded by ks-1-pad
  a.conv_H = (int)oh; a.conv_W = (int)ow; a.conv_ow = (int)W; a.conv_ohw = (int)(H * W);
  a.conv_sY = 1; a.conv_sX = 1; a.conv_pH = (int)(ks - 1 - pad); a.conv_pW = (int)(ks - 1 - pad);
  a.conv_bytes = (int)(4 * batch * F * oh * ow);
  return kTiles4DX[v].fn(a, 3, 1, s);
}

namespace {
// the taps of output pixel class (py, px) of a stride-2 3x3 layer padded by
// pad, in scol2im's (kr, kc) order: pixel (iy, ix) = (2 qy + py, 2 qx + px)
// takes col entry (kr, kc) at delta pixel ((iy + pad - kr) / 2, (ix + pad -
// kc) / 2) when both differences are even (col2im's stride test) — delta row
// qy + fr - 1 with fr = (py + pad - kr) / 2 + 1 in 0..2: the forward-window
// bit fr*3 + fc of a window over the delta planes padded by 1
int s2_taps(int64_t pad, int py, int px, int* ref, int* fwd) {
  int n = 0;
  for (int kr = 0; kr < 3; ++kr) {
    const int dr = py + (int)pad - kr;
    if (dr & 1) continue;
    for (int kc = 0; kc < 3; ++kc) {
      const int dc = px + (int)pad - kc;
      if (dc & 1) continue;
      ref[n] = kr * 3 + kc;
      fwd[n] = (dr / 2 + 1) * 3 + (dc / 2 + 1);
      ++n;
    }
  }
  return n;
}

bool dx3s2_fits(int v, int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F, int64_t pad,
                int64_t oh, int64_t ow) {
  if (v < 0 || v >= kNumTiles4DX || pad < 0 || pad > 2 || H < 2 || W < 2) return false;
  if (oh != (H + 2 * pad - 3) / 2 + 1 || ow != (W + 2 * pad - 3) / 2 + 1 || oh <= 0 || ow <= 0)
    return false;
  if (F % kTiles4DX[v].bk || C % kTiles4DX[v].bm || batch <= 0) return false;
  return batch * F * oh * ow * 4 <= 0x7fffffffLL && batch * C * H * W <= 0x7fffffffLL &&
         9 * F * C <= 0x7fffffffLL;
}
}  // namespace

unsigned long long conv_tile4_dx3s2_order(int64_t pad) {
  unsigned long long o = 0;
  int sl = 0, ref[9], fwd[9];
  for (int cls = 0; cls < 4; ++cls) {
    const int n = s2_taps(pad, cls >> 1, cls & 1, ref, fwd);
    for (int i = 0; i < n; ++i, ++sl) o |= (unsigned long long)ref[i] << (4 * sl);
  }
  return o;
}

// by the pixel count of a class.  Measured on the YOLOv3 stride-2 layers at
// batch 8 (scripts/bwd_sweep.py --what dx, whole backward calls,
// profiles/r04_bwd_dx_s2.json) against TN + col2im: 416^2 -> 208^2 (32
// channels) 0.840 -> 0.788 ms with the 32 x 176 tile, 208^2 -> 104^2 0.495
// -> 0.456 with 64 x 48; level at 104^2 -> 52^2 (0.384 vs 0.382) and behind
// on the smaller planes (52^2 -> 26^2 0.319 vs >= 0.356), so not there
int conv_tile4_dx3s2_pick(int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F, int64_t ks,
                          int64_t pad) {
  if (ks != 3) return -1;
  const int64_t N = batch * (H / 2) * (W / 2), oh = (H + 2 * pad - 3) / 2 + 1,
                ow = (W + 2 * pad - 3) / 2 + 1;
  int v = -1;
  if (C % 64 && N >= 50000)
    v = 6;
  else if (N >= 50000)
    v = 2;  // (its PF twin 10: see conv_tile4_dx3_pick)
  return v >= 0 && dx3s2_fits(v, batch, C, H, W, F, pad, oh, ow) ? v : -1;
}

hipError_t launch_conv_tile4_dx3s2(int v, const float* wt, const float* delta, float* im,
                                   int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F,
                                   int64_t pad, int64_t oh, int64_t ow, hipStream_t s) {
  if (!dx3s2_fits(v, batch, C, H, W, F, pad, oh, ow)) return hipErrorInvalidValue;
  int sl = 0;
  for (int cls = 0; cls < 4; ++cls) {
    const int py = cls >> 1, px = cls & 1;
    int ref[9], fwd[9];
    const int T = s2_taps(pad, py, px, ref, fwd);
    const int64_t ohc = (H - py + 1) / 2, owc = (W - px + 1) / 2;
    if (T == 0 || ohc <= 0 || owc <= 0) {
      sl += T;
      continue;
    }
    GemmArgs a{};
    a.M = C; a.N = batch * ohc * owc; a.K = T * F;
    a.alpha = 1.0f; a.beta = 0.0f; a.beta_mode = BETA_ZERO;
    a.A = wt + (int64_t)sl * F * C; a.lda = C; a.strideA = 0;
    a.B = delta; a.ldb = oh * ow; a.strideB = F * oh * ow;
    a.C = im; a.ldc = H * W; a.strideC = C * H * W;
    a.batch = 1; a.epi = EPI_NONE; a.bias = nullptr; a.act = 0;
    a.conv = 2;
    // the class's columns over the delta planes: a 3x3 window padded by 1
    a.conv_H = (int)oh; a.conv_W = (int)ow; a.conv_ow = (int)owc; a.conv_ohw = (int)(ohc * owc);
    a.conv_sY = 1; a.conv_sX = 1; a.conv_pH = 1; a.conv_pW = 1;
    a.conv_bytes = (int)(4 * batch * F * oh * ow);
    a.dx_cls = 1 | py << 1 | px << 2;
    a.dx_taps = T << 16;
    for (int i = 0; i < T; ++i) a.dx_taps |= fwd[i] << (4 * i);
    a.dx_imgW = (int)W;
    if (hipError_t e = kTiles4DX[v].fn(a, 3, 1, s); e != hipSuccess) return e;
    sl += T;
  }
  return hipSuccess;
}

hipError_t launch_conv_tile4(int v, const GemmArgs& a, int ks, int dil, hipStream_t s) {
  if (v < 0 || v >= kNumTiles4) return hipErrorInvalidValue;
  return kTiles4[v].fn(a, ks, dil, s);
}

}  // namespace tns
