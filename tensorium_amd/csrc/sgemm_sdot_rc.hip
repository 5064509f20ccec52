// sgemm_sdot_rc.hip — gemm(NoTrans, Trans) in the reference's sdot order with
// the eight residue chains of an output in ONE wave's registers.
//
// Same product as sgemm_sdot.hip (sdot_avx2, ntensors.pas:1233-1306, under
// s_nt 1957-2005 and cblas_sgemm 2231-2286): lane l of the AVX2 register is
// an ascending fma chain over k = l (mod 8) from +0, then s_l = lane_l +
// lane_{l+4} and dot = (s0 + s1) + (s2 + s3), sum = ALPHA*dot, C += sum.
// sgemm_sdot.hip gives each residue class its own wave and meets the eight
// partial tiles in LDS; here a wave owns a 32 x 32 output tile and keeps all
// eight classes as eight v_mfma_f32_32x32x2_f32 accumulators (128 VGPRs), so
//   * the class fold is eight register adds per output (no LDS epilogue),
//   * a wave's MFMAs run over the whole k of its tile (8 independent chains
//     interleaved: no dependent-issue stall), and
//   * every block does full-k work, so tiles are 32 x 32 per wave, the
//     granularity the YOLOv3 dW shapes need (M x N x images = 9216 wave
//     tiles at 26^2).
//
// k-tiles of 64.  Class r, lane half h and MFMA step s (0..3) consume
// k = r + 8h + 16s, so LDS stores each operand row with k permuted as
// pos(k) = ((k & 7)*2 + ((k >> 3) & 1))*4 + (k >> 4): the four steps of one
// (class, half) are one ds_read_b128.  Rows are 68 floats (8-lane phases of
// the b128 reads and writes hit 8 distinct 16-byte bank groups).  Staging is
// by dword buffer loads (rows need not be 16-byte aligned: K = 169 at 13^2),
// four per (row, k & 15) unit, one b128 LDS write; k >= K and rows past M / N
// read 0 (buffer range check; out-of-range rows are never stored).
// Zero-filled k adds fma(0, 0, x) = x (a chain from +0 never holds -0).
//
// Measured against sgemm_sdot.hip on the YOLOv3 batch-8 dW shapes
// (scripts/dw_forms.py, profiles/r03_dw_forms.json): the 4-class form with
// 3-4 waves per SIMD is 4-7 % faster on the 26^2 / 13^2 layers (k <= 1024
// per image), the 8-class form 2 waves per SIMD and no faster; both sit at
// MFMA busy 0.55 like the one-class-per-wave kernel.  A variant running the
// batch's images inside the block (C updated per image through L2, no
// per-image partials) was slower (13^2: 0.39 vs 0.28 ms) and was dropped.
#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int RC_BK = 64, RC_LD = 68;

__device__ __forceinline__ int rc_pos(int g) { return ((g & 7) * 2 + (g >> 3)) * 4; }

// CS: residue classes per wave.  8: a wave owns its 32 x 32 tile's eight
// chains (128 accumulator VGPRs, 2 waves per SIMD).  4: two waves share a
// tile, classes {0, 1, 4, 5} and {2, 3, 6, 7} (64 accumulator VGPRs, 3-4
// waves per SIMD); each forms its half of the fold, (L0 + L4) + (L1 + L5) or
// (L2 + L6) + (L3 + L7), and the second hands its half over through LDS.
template <int WM, int WN, int CS>
__global__ __launch_bounds__(64 * WM * WN * (8 / CS), (CS == 8 ? 2 : (WM * WN * (8 / CS) >= 8 ? 2 : 3)))
void sdot_rc_kernel(GemmArgs p) {
  constexpr int TW = WM * WN, NW = TW * (8 / CS);
  constexpr int BM = 32 * WM, BN = 32 * WN, NT = 64 * NW, ROWS = BM + BN;
  constexpr int STAGE = ROWS * RC_LD;
  constexpr int RPU = NT / 16;  // rows per staging unit step
  constexpr int UA = BM / RPU, UB = BN / RPU, U = UA + UB;
  static_assert(CS == 8 || CS == 4, "classes per wave");
  static_assert(BM % RPU == 0 && BN % RPU == 0 && U >= 1, "staging split");
  static_assert(CS == 8 || 2 * STAGE >= TW * 16 * 64, "fold hand-over fits the stages");
  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int wt = wid % TW, ch = wid / TW;  // output tile, class set
  const int wm = wt / WN, wn = wt % WN;
  const int tiles_m = (int)((p.M + BM - 1) / BM);
  const int64_t m0 = (int64_t)(blockIdx.x % tiles_m) * BM;
  const int64_t n0 = (int64_t)(blockIdx.x / tiles_m) * BN;
  const int M = (int)p.M, N = (int)p.N, K = (int)p.K;

  // staging unit u: row (tid >> 4) + RPU*u, k & 15 = g; lanes 2i and 2i+1 take
  // g = i and i + 8 (one 8-lane phase: 8 distinct bank groups).  One voffset
  // per operand for the whole launch; the unit's row and the k-tile go in the
  // uniform soffset.  Rows past M / N and k >= K fall outside the buffer
  // ranges and read 0 (never stored / fma(0, 0, x) = x).
  const int l16 = tid & 15;
  const int g = ((l16 & 1) << 3) | (l16 >> 1);
  const int voffA = (int)((m0 + (tid >> 4)) * p.lda + g) * 4;
  const int voffB = (int)((n0 + (tid >> 4)) * p.ldb + g) * 4;
  const int loff = (tid >> 4) * RC_LD + rc_pos(g);
  const int rstepA = RPU * (int)p.lda * 4, rstepB = RPU * (int)p.ldb * 4;
  const unsigned bytesA = (unsigned)(((int64_t)(M - 1) * p.lda + K) * 4);
  const unsigned bytesB = (unsigned)(((int64_t)(N - 1) * p.ldb + K) * 4);

  float st[U][4];
  auto load = [&](__amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int k0, bool mask) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool isa = u < UA;
      const int so = (isa ? u * rstepA : (u - UA) * rstepB) + 4 * k0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        int off = (isa ? voffA : voffB) + 64 * s;
        if (mask) off = k0 + g + 16 * s < K ? off : (int)0x80000000;
        st[u][s] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(isa ? ra : rb, off, so, 0));
      }
    }
  };
  auto store = [&](float* buf) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      *reinterpret_cast<float4*>(buf + loff + u * RPU * RC_LD) =
          make_float4(st[u][0], st[u][1], st[u][2], st[u][3]);
  };

  // acc[i] holds class cls(i): all eight, or (i & 1) + 2*ch + 4*(i >> 1)
  auto cls = [&](int i) { return CS == 8 ? i : (i & 1) + 2 * ch + 4 * (i >> 1); };
  floatx16 acc[CS];
  const int a_rd = (wm * 32 + l31) * RC_LD + 4 * h;
  const int b_rd = (BM + wn * 32 + l31) * RC_LD + 4 * h;
  // classes in groups of CG (4 or 2; 8*CG fragment VGPRs): an accumulator
  // recurs every CG-th MFMA (past the 64-cycle dependency at CG >= 2)
  constexpr int CG = CS == 8 ? 4 : 2;
  auto mma_tile = [&](const float* buf) {
#pragma unroll
    for (int r0 = 0; r0 < CS; r0 += CG) {
      float4 a[CG], b[CG];
#pragma unroll
      for (int r = 0; r < CG; ++r) {
        a[r] = *reinterpret_cast<const float4*>(buf + a_rd + 8 * cls(r0 + r));
        b[r] = *reinterpret_cast<const float4*>(buf + b_rd + 8 * cls(r0 + r));
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int r = 0; r < CG; ++r)
          acc[r0 + r] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[r][s], b[r][s], acc[r0 + r], 0, 0, 0);
      // (no hoisting of the next group's reads: hipcc otherwise reuses the
      // staging registers and issues the next tile's loads mid-tile)
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // one image's product into acc: ascending k-tiles, double-buffered LDS,
  // one barrier per tile; the last, partial tile loads with the k check
  const int nt = (K + RC_BK - 1) / RC_BK;
  const bool ragged = K % RC_BK != 0;
  auto run = [&](const float* A, const float* B) {
    const __amdgpu_buffer_rsrc_t ra =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), 0, bytesA, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B), 0, bytesB, 0x00020000);
#pragma unroll
    for (int r = 0; r < CS; ++r)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[r][e] = 0.0f;
    if (nt == 0) return;  // K = 0: sdot of nothing is +0
    load(ra, rb, 0, ragged && nt == 1);
    store(lds);
    __syncthreads();
    // the loop loads full tiles only; the tile before the last loads the
    // (possibly ragged) last one; the last is peeled (no staging, and no
    // exit inside the body: the accumulators stay in place)
    int t = 0;
    for (; t + 2 < nt; ++t) {
      load(ra, rb, (t + 1) * RC_BK, false);
      __builtin_amdgcn_sched_barrier(0);  // the next tile's loads first
      mma_tile(lds + (t & 1) * STAGE);
      store(lds + ((t + 1) & 1) * STAGE);
      __syncthreads();
    }
    if (t + 1 < nt) {
      load(ra, rb, (t + 1) * RC_BK, ragged);
      __builtin_amdgcn_sched_barrier(0);
      mma_tile(lds + (t & 1) * STAGE);
      store(lds + ((t + 1) & 1) * STAGE);
      __syncthreads();
      ++t;
    }
    mma_tile(lds + (t & 1) * STAGE);
    __syncthreads();  // (the stages are free for the fold hand-over)
  };
  // dot = ((L0 + L4) + (L1 + L5)) + ((L2 + L6) + (L3 + L7)), sum = ALPHA*dot.
  // CS = 4: set 1 leaves (L2 + L6) + (L3 + L7) in LDS for set 0.
  const float alpha = p.alpha;
  float* xch = lds + (wt * 16) * 64 + lane;  // [tile][e][lane]
  auto fold = [&]() {
    if constexpr (CS == 4) {
      if (ch == 1) {
#pragma unroll
        for (int e = 0; e < 16; ++e) xch[64 * e] = (acc[0][e] + acc[2][e]) + (acc[1][e] + acc[3][e]);
      }
      __syncthreads();
    }
  };
  auto sum_at = [&](int e) {
    if constexpr (CS == 8) {
      const float s0 = acc[0][e] + acc[4][e], s1 = acc[1][e] + acc[5][e];
      const float s2 = acc[2][e] + acc[6][e], s3 = acc[3][e] + acc[7][e];
      return alpha * ((s0 + s1) + (s2 + s3));
    } else {  // set 0: acc = L0, L1, L4, L5
      const float s01 = (acc[0][e] + acc[2][e]) + (acc[1][e] + acc[3][e]);
      return alpha * (s01 + xch[64 * e]);
    }
  };
  const bool writer = CS == 8 || ch == 0;
  const int64_t col = n0 + wn * 32 + l31;
  auto row_at = [&](int e) { return m0 + wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h; };
  auto c0_at = [&](const float* cp) {
    if (p.beta_mode == BETA_ZERO) return 0.0f;
    if (p.beta_mode == BETA_SCALE) return p.beta * *cp;  // cblas_sgemm's mulvs pre-scale
    return *cp;
  };

  const int64_t bz = blockIdx.y;
  run(p.A + bz * p.strideA, p.B + bz * p.strideB);
  fold();
  if (!writer) return;
  float* C = p.C + bz * p.strideC;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int64_t row = row_at(e);
    if (row >= M || col >= N) continue;
    float* cp = C + row * p.ldc + col;
    const float sum = sum_at(e);
    *cp = p.beta_mode == BETA_STORE ? sum : c0_at(cp) + sum;  // C[i,j] := C[i,j] + sum
  }
}

template <int WM, int WN, int CS>
hipError_t launch_rc(const GemmArgs& a, hipStream_t s) {
  constexpr int NT = 64 * WM * WN * (8 / CS);
  const int64_t tiles = ((a.M + 32 * WM - 1) / (32 * WM)) * ((a.N + 32 * WN - 1) / (32 * WN));
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  for (int64_t b0 = 0; b0 < a.batch; b0 += 65535) {
    GemmArgs sub = a;
    const int64_t nb = a.batch - b0 < 65535 ? a.batch - b0 : 65535;
    sub.A = a.A + b0 * a.strideA;
    sub.B = a.B + b0 * a.strideB;
    sub.C = a.C + b0 * a.strideC;
    sub.batch = nb;
    hipLaunchKernelGGL((sdot_rc_kernel<WM, WN, CS>), dim3((unsigned)tiles, (unsigned)nb),
                       dim3(NT), 0, s, sub);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

struct RcForm {
  hipError_t (*fn)(const GemmArgs&, hipStream_t);
  const char* name;
};
const RcForm kForms[] = {
    {launch_rc<2, 2, 8>, "rc_64x64_w2x2_c8"},
    {launch_rc<2, 2, 4>, "rc_64x64_w2x2x2_c4"},
    {launch_rc<2, 1, 4>, "rc_64x32_w2x1x2_c4"},
};
constexpr int kNumForms = sizeof(kForms) / sizeof(kForms[0]);

}  // namespace

int sdot_rc_variant_count() { return kNumForms; }
const char* sdot_rc_variant_name(int v) { return v >= 0 && v < kNumForms ? kForms[v].name : ""; }

// every image's operands, and the rows a last tile runs past them,
// byte-addressable in 31 bits (buffer offsets)
bool sdot_rc_applies(const GemmArgs& a) {
  const int64_t ea = (a.M + 128) * a.lda + a.K + RC_BK, eb = (a.N + 128) * a.ldb + a.K + RC_BK;
  return a.M > 0 && a.N > 0 && a.K >= 0 && a.lda >= a.K && a.ldb >= a.K &&
         ea * 4 < 0x7fffffffLL && eb * 4 < 0x7fffffffLL;
}

hipError_t launch_sdot_rc(int v, const GemmArgs& a, hipStream_t s) {
  if (v < 0 || v >= kNumForms) return hipErrorInvalidValue;
  if (a.M <= 0 || a.N <= 0 || a.batch <= 0) return hipSuccess;
  if (!sdot_rc_applies(a)) return hipErrorInvalidValue;
  return kForms[v].fn(a, s);
}

}  // namespace tns
