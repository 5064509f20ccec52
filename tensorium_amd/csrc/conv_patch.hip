// conv_patch.hip — 3x3 stride-1 "same" convolution as an implicit GEMM whose
// B operand is read from a staged INPUT PATCH instead of gathered im2col
// rows (TConvolutionalLayer.forward → Conv2D + forwardBias + activate after
// fuseBatchNorm: nConvolutionLayer.pas:457-569, ntensors.pas:8252-8349; the
// im2col column order of sim2Col, 11415-11532).
//
// Same arithmetic as conv_tile.hip / conv_dma.hip: each output an
// ascending-k fma chain over k = (c, kr, kc) from +0 through the
// v_mfma_f32_16x16x4_f32 lane-quarter order, then bias add and activation,
// each rounded once — bit-identical to sim2Col + the reference GEMM.
//
// A block's columns are R whole output rows of one image (BN >= R*W); a
// 32-deep k-tile touches at most 5 input channels, so its B operand is the
// 5 x (R+2) x (W+2) window of the input around those rows (zero halo) — about
// a quarter of the im2col rows' bytes, copied once by dword LDS-DMA with the
// halo and the rows outside the image landing as 0 through the buffer range
// check.  A B fragment element (k, pixel) is then the patch element at the
// pixel's position plus k's tap offset (a 32-entry per-tile table in LDS,
// broadcast per lane quarter).  A (weights) by 16-byte LDS-DMA into the
// swizzled slot image of conv_dma.hip; a 3-stage ring, tile t+2 issued at
// the top of tile t, one raw barrier per tile after a counted vmcnt.
#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
// Measured and not picked (profiles/): compiled only into the
// diagnostics build (TNS_DIAG=1 python -m tensorium_amd.build); the default
// library reports no forms of this family.
#ifdef TNS_DIAG_KERNELS

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32, NT = 512, NSTAGE = 3, NCH = 5;

template <int BM_, int BN_, int R_, int NIW_>
struct QGeo {
  static constexpr int BM = BM_, BN = BN_, R = R_, NIW = NIW_;
  static constexpr int WM = BM / 16, WN = 8 / WM;
  static constexpr int WTN = BN / WN, J = WTN / 16;
  static constexpr int A_FL = BM * BK;            // A slots (floats)
  static constexpr int TAB = 32;                  // k -> tap offset (ints)
  static constexpr int PFL = NIW * 8 * 64;        // patch floats (DMA granules)
  static constexpr int STAGE = A_FL + TAB + PFL;  // floats
  static constexpr int ADMA = A_FL / 4 / 64 / 8;  // A DMA wave-instructions per wave
  static constexpr int NDMA = ADMA + NIW;
  static_assert(WM * WN == 8 && BN % (16 * WN) == 0 && ADMA >= 1, "geometry");
  static_assert(NSTAGE * STAGE * 4 <= 160 * 1024, "LDS");
};

template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <class G>
__global__ __launch_bounds__(NT, 1) void conv_patch_kernel(GemmArgs p) {
  constexpr int BM = G::BM, BN = G::BN, R = G::R, NIW = G::NIW, WN = G::WN, WTN = G::WTN;
  constexpr int J = G::J, A_FL = G::A_FL, TAB = G::TAB, STAGE = G::STAGE, ADMA = G::ADMA;
  constexpr int NDMA = G::NDMA;
  __shared__ __attribute__((aligned(16))) float smem[NSTAGE * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;
  const int r16 = lane & 15, q = lane >> 4;
  const int H = p.conv_H, W = p.conv_W, HW = H * W, C = (int)(p.K / 9);
  const int PW = W + 2, PCH = (R + 2) * PW;
  const int RG = (H + R - 1) / R;  // row groups per image
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
  const int img = tn / RG, y0 = (tn - img * RG) * R;
  const int rows = min(R, H - y0);
  const int K = (int)p.K;
  const unsigned lds0 =
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)smem;  // byte address

  // ---- patch DMA: instruction i of this wave moves patch floats
  // 64*(wid + 8i) .. +63 = (channel ch, patch row r, patch col x); the
  // source is input (c_lo + ch, y0 + r - 1, x - 1) of this image, or out of
  // range (-> 0) for the halo, rows outside the image and channels >= C
  int prel[NIW], pch[NIW];
  bool pv[NIW];
#pragma unroll
  for (int i = 0; i < NIW; ++i) {
    const int e = 64 * (wid + 8 * i) + lane;
    const int ch = e / PCH, rem = e - ch * PCH;
    const int r = rem / PW, x = rem - r * PW;
    pv[i] = ch < NCH && (unsigned)(y0 + r - 1) < (unsigned)H && (unsigned)(x - 1) < (unsigned)W;
    pch[i] = ch;
    prel[i] = ch * HW + (r - 1) * W + (x - 1);
  }
  const __amdgpu_buffer_rsrc_t brsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.B), 0, p.conv_bytes, 0x00020000);
  const int img_base = img * (int)p.strideB + y0 * W;

  // ---- A DMA sources: slot s of wave-instruction i holds 4 k of one row ---
  const float* a_src[ADMA];
#pragma unroll
  for (int i = 0; i < ADMA; ++i) {
    const int slot = 64 * (ADMA * wid + i) + lane;
    const int row = slot >> 3, kq = (slot & 7) ^ (row & 7);
    a_src[i] = p.A + (m0 + row) * p.lda + 4 * kq;
  }

  // ---- one tile's staging into stage st: DMAs (this wave's share) and the
  // tap-offset table (threads 0..31) -------------------------------------------
  auto issue = [&](int tile, int st) {
    const unsigned sbase = lds0 + (unsigned)(st * STAGE) * 4u;
    const int k0 = tile * BK, c_lo = k0 / 9;
#pragma unroll
    for (int i = 0; i < ADMA; ++i) {
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(a_src[i] + (int64_t)k0), "s"(sbase + (unsigned)((ADMA * wid + i) * 1024))
          : "memory");
    }
    const int base = img_base + c_lo * HW;
#pragma unroll
    for (int i = 0; i < NIW; ++i) {
      const unsigned off =
          (pv[i] && pch[i] < C - c_lo) ? 4u * (unsigned)(base + prel[i]) : 0x80000000u;
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
          "buffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(off), "s"(brsrc),
            "s"(sbase + (unsigned)((A_FL + TAB + 64 * (wid + 8 * i)) * 4))
          : "memory");
    }
    if (tid < 32) {  // tap offset of k = k0 + tid inside the patch
      const int k = k0 + tid, c = k / 9, rem = k - 9 * c;
      const int kr = rem / 3, kc = rem - 3 * kr;
      reinterpret_cast<int*>(smem + st * STAGE + A_FL)[tid] = (c - c_lo) * PCH + kr * PW + kc;
    }
  };

  // ---- pixel of each of this lane's column strips in the patch -----------
  int pbase[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int nl = wc * WTN + 16 * j + r16;
    const int oy = nl / W, ox = nl - oy * W;
    pbase[j] = nl < rows * W ? oy * PW + ox : 0;
  }

  // ---- MFMA: step s consumes k = 4s + q ----------------------------------
  floatx4 acc[J];
#pragma unroll
  for (int j = 0; j < J; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int arow = wr * 16 + r16;
  auto frag = [&](const float* st, int s, float& a, float (&b)[J]) {
    a = st[(arow * 8 + (s ^ (arow & 7))) * 4 + q];
    const int tap = reinterpret_cast<const int*>(st + A_FL)[4 * s + q];
    const float* bp = st + A_FL + TAB + tap;
#pragma unroll
    for (int j = 0; j < J; ++j) b[j] = bp[pbase[j]];
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
      issue(1, 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the tap tables
      wait_vm_barrier<NDMA>();  // tile 0 landed (tile 1 may still be in flight)
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wait_vm_barrier<0>();
    }
  }
  for (int t = 0; t < nt; ++t) {
    const float* cur = smem + (t % NSTAGE) * STAGE;
    const bool ahead = t + 2 < nt;
    // tile t+2 into stage (t+2)%3 = (t-1)%3: every wave left it at the last
    // barrier
    if (ahead) issue(t + 2, (t + 2) % NSTAGE);
    __builtin_amdgcn_sched_barrier(0);
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
    }
    if (t + 1 < nt) {  // tile t+1 landed (own DMAs and table stores), then everyone's
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
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
    const int nl = wc * WTN + 16 * j + r16;
    if (nl >= rows * W) continue;
    const int64_t cofs = (int64_t)img * p.strideC + (int64_t)y0 * W + nl;
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
hipError_t launch_g(const GemmArgs& a, hipStream_t s) {
  const int H = a.conv_H, W = a.conv_W;
  // 3x3, stride 1, "same" padding 1, dilation 1 (the caller checks those);
  // whole rows per tile; the 5-channel patch within the DMA granules
  if (a.M % G::BM || a.K % BK || a.K % 9 || a.K <= 0 || a.lda % 4 ||
      (reinterpret_cast<uintptr_t>(a.A) & 15) || G::R * W > G::BN ||
      NCH * (G::R + 2) * (W + 2) > G::PFL || a.conv_ohw != H * W)
    return hipErrorInvalidValue;
  const int64_t imgs = a.N / ((int64_t)H * W);
  const int64_t tiles = (a.M / G::BM) * imgs * ((H + G::R - 1) / G::R);
  if (tiles > 0x7fffffff || a.K > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL((conv_patch_kernel<G>), dim3((unsigned)tiles), dim3(NT), 0, s, a);
  return hipGetLastError();
}

struct TileInfo {
  hipError_t (*fn)(const GemmArgs&, hipStream_t);
  const char* name;
};
#define TNS_CQ(BMv, BNv, Rv, NIWv) \
  {launch_g<QGeo<BMv, BNv, Rv, NIWv>>, "conv_patch<" #BMv "x" #BNv ",R" #Rv ">"}
const TileInfo kTiles[] = {
    TNS_CQ(128, 208, 4, 4),  // 0: 52^2 (4 rows: 208 px, 8 x 13 x 2 blocks at 256 filters)
    TNS_CQ(128, 112, 4, 2),  // 1: 26^2 (4 rows: 104 px, 8 x 7 x 4 blocks at 512 filters)
    TNS_CQ(64, 96, 7, 2),    // 2: 13^2 (7 rows: 91 px, 8 x 2 x 16 blocks at 1024 filters)
    TNS_CQ(128, 208, 2, 4),  // 3: 104^2 (2 rows: 208 px, 8 x 52 blocks at 128 filters)
    TNS_CQ(128, 176, 13, 3), // 4: 13^2 whole image (169 px)
    TNS_CQ(64, 224, 4, 4),   // 5: 52^2 at 64-row tiles
};
#undef TNS_CQ
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);

}  // namespace

int conv_patch_count() { return kNumTiles; }
const char* conv_patch_name(int v) { return v >= 0 && v < kNumTiles ? kTiles[v].name : ""; }

// not picked by default until measured (TNS_OPT_CONV_VARIANT = 400 + v)
int conv_patch_pick(const GemmArgs& a) {
  (void)a;
  return -1;
}

hipError_t launch_conv_patch(int v, const GemmArgs& a, hipStream_t s) {
  if (v < 0 || v >= kNumTiles) return hipErrorInvalidValue;
  return kTiles[v].fn(a, s);
}

#else
int conv_patch_count() { return 0; }
const char* conv_patch_name(int) { return ""; }
int conv_patch_pick(const GemmArgs&) { return -1; }
hipError_t launch_conv_patch(int, const GemmArgs&, hipStream_t) { return hipErrorInvalidValue; }
#endif  // TNS_DIAG_KERNELS

}  // namespace tns
