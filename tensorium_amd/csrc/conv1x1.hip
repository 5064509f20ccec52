// conv1x1.hip — the 1x1 / stride-1 conv layers whose planes hold a multiple
// of 4 pixels (YOLOv3: 26^2 .. 208^2) as an NN GEMM straight from the input
// planes: out[b][m][p] = act(bias[m] + sum_k W[m][k] X[b][k][p]), the batch
// folded into N (TConvolutionalLayer.forward -> Conv2D, which skips im2col
// for 1x1/s1, ntensors.pas:8286-8312, + forwardBias + activate after
// fuseBatchNorm, nConvolutionLayer.pas:457-569).
//
// Arithmetic: every output an ascending-k fma chain from +0
// (v_mfma_f32_16x16x4_f32, step s consumes k = 4s + q for lane quarter q),
// then bias add and activation, each rounded once — bit-identical to
// conv_tile4 / the reference GEMM.
//
// Operands:
//   * B (the input planes, [k][pixel] rows) streams global -> LDS by
//     LDS-DMA (global_load_lds_dwordx4) into a row-major [BK][BN] image; each
//     lane's 16 bytes are 4 pixels of one image row (the plane's pixel count a
//     multiple of 4, so a chunk never straddles two images) and its source
//     address is its own (a tile's columns may span images);
//   * interleaved columns: fragment j of a wave's 64-column group takes
//     columns 4c + j (c = lane & 15), so one ds_read_b128 of a k-row gives a
//     lane its four fragments' values of one MFMA step, and the 16-lane groups
//     of that read fall on distinct bank quads (row stride 64 floats);
//   * A (weights, k-contiguous rows) through registers into k-permuted slots
//     (conv_tile4's layout: one ds_read_b128 per 4 steps);
//   * epilogue: a lane's four fragments' values of one row are 4 consecutive
//     pixels of one image: 16-byte stores.
// Small blocks (BM = 32: two waves) so that every CU holds several: the
// 1x1 layers' k is short (64 .. 1024), and a block's first-tile latency hides
// under the other blocks' MFMAs.
#include <algorithm>
#include <type_traits>

#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void c1_dma16(const float* sbase, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

struct C1Args {
  const float* A;  // weights [M][K]
  const float* X;  // input planes [batch][K][P]
  float* C;        // [batch][M][P]
  const float* bias;
  int M, N, K, P, tiles_m, act;
  bool fuse;
  bool add;  // C := C + product (the conv backward's 1x1 col2im: one add a pixel)
};

// BM x BN block, BK-deep k-tiles, WM x WN waves: a wave = 16 rows x 64
// columns (4 interleaved 16-wide fragments)
template <int BM_, int BK_, int WM_, int WN_>
struct C1G {
  static constexpr int BM = BM_, BK = BK_, WM = WM_, WN = WN_;
  static constexpr int BN = 64 * WN, NW = WM * WN, NT = 64 * NW, NG = BK / 16;
  static constexpr int A_TILE = BK * BM, B_TILE = BK * BN, STAGE = A_TILE + B_TILE;  // floats
  static constexpr int AU = BM * BK / 4 / NT;       // float4 A units per thread and tile
  static constexpr int RPI = 256 / BN;              // B k-rows per DMA instruction
  static constexpr int BDMA = BK / RPI;             // B DMA instructions per tile
  static constexpr int DPW = (BDMA + NW - 1) / NW;  // ... per wave (padded)
  static_assert(BM == 16 * WM && BK % 16 == 0 && 256 % BN == 0 && BK % RPI == 0, "geometry");
  static_assert(AU >= 1 && BM * BK / 4 % NT == 0, "A units");
  static_assert(2 * STAGE * 4 <= 65536, "LDS: several blocks per CU");
  static_assert(NG % 2 == 0, "groups: f0 holds group 0 at every tile start");
};

template <int N>
__device__ __forceinline__ void c1_wait(bool keep_n) {
  if (keep_n)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <class G>
__global__ __launch_bounds__(G::NT) void conv1x1_kernel(C1Args p) {
  constexpr int BM = G::BM, BN = G::BN, BK = G::BK, NG = G::NG;
  constexpr int A_TILE = G::A_TILE, STAGE = G::STAGE, AU = G::AU, DPW = G::DPW;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), wm = w % G::WM, wn = w / G::WM;
  const int r16 = lane & 15, q = lane >> 4;
  // XCD-contiguous order, row tiles inner: an XCD's blocks share column
  // ranges of the planes in its L2
  int tm, tn;
  {
    const int nb = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, qq = nb >> 3, rr = nb & 7;
    const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    tm = wg % p.tiles_m;
    tn = wg / p.tiles_m;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int N = p.N, K = p.K, P = p.P, nt = K / BK;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)smem;
  // B DMA lane offset: k-row L / (BN/4) of an instruction's RPI rows, 4
  // pixels from column 4 (L % (BN/4)) (past N: the last chunk, never stored)
  unsigned b_off;
  {
    int n = n0 + 4 * (lane % (BN / 4));
    if (n > N - 4) n = N - 4;
    const int img = n / P, pix = n - img * P;
    b_off = 4u * (unsigned)(img * K * P + (lane / (BN / 4)) * P + pix);
  }
  auto dma_b = [&](int t, int st, int v) {
    int u = w + G::NW * v;
    if (G::BDMA % G::NW != 0 && u >= G::BDMA) u -= G::NW;
    c1_dma16(p.X + (int64_t)(t * BK + u * G::RPI) * P, b_off,
             lds0 + 4u * (unsigned)(st * STAGE + A_TILE) + 1024u * (unsigned)u);
  };
  auto dma_all = [&](int t, int st) {
#pragma unroll
    for (int v = 0; v < DPW; ++v) dma_b(t, st, v);
  };
  // A staging: unit = k-quad kq4 of row m; values to slot rows 4(kq4>>2)+0..3,
  // component kq4 & 3 (rows past M read row M-1: computed, never stored)
  unsigned a_off[AU];
  int a_dst[AU];
#pragma unroll
  for (int u = 0; u < AU; ++u) {
    const int idx = tid + G::NT * u;
    const int lo = idx & 7, rest = idx >> 3;
    const int m = rest % BM, kq4 = lo + 8 * (rest / BM);
    const int mr = m0 + m < p.M ? m : p.M - 1 - m0;
    a_off[u] = 4u * (unsigned)(mr * K + 4 * kq4);
    a_dst[u] = (4 * (kq4 >> 2)) * BM * 4 + m * 4 + (kq4 & 3);
  }
  const float* a_row0 = p.A + (int64_t)m0 * K;
  floatx4 ra[AU];
  auto load_a = [&](int t) {
    const float* sb = a_row0 + t * BK;
#pragma unroll
    for (int u = 0; u < AU; ++u)
      asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(ra[u]) : "v"(a_off[u]), "s"(sb) : "memory");
  };
  auto store_a = [&](int st) {
    float* as = smem + st * STAGE;
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      asm volatile("" : "+v"(ra[u]));
      as[a_dst[u]] = ra[u][0];
      as[a_dst[u] + BM * 4] = ra[u][1];
      as[a_dst[u] + 2 * BM * 4] = ra[u][2];
      as[a_dst[u] + 3 * BM * 4] = ra[u][3];
    }
  };

  floatx4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  struct Frag {
    floatx4 a, b[4];
  };
  // group g: the A slot (k = 16g + 4i + q, i = 0..3) and the four steps' B
  // rows (k = 16g + 4i + q: columns 4 r16 .. 4 r16 + 3 of the wave's group)
  auto frag = [&](int st, int g, Frag& f) {
    const float* ap = smem + st * STAGE + ((4 * g + q) * BM + wm * 16 + r16) * 4;
    f.a = *reinterpret_cast<const floatx4*>(ap);
    const float* bp = smem + st * STAGE + A_TILE + (16 * g + q) * BN + wn * 64 + 4 * r16;
#pragma unroll
    for (int i = 0; i < 4; ++i) f.b[i] = *reinterpret_cast<const floatx4*>(bp + 4 * i * BN);
  };
  auto mma = [&](const Frag& f) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[i], f.b[i][j], acc[j], 0, 0, 0);
  };
  auto mma_dma = [&](const Frag& f, int tb, int st) {
    constexpr int NM = 16, STEP = NM / DPW > 0 ? NM / DPW : 1;
#pragma unroll
    for (int x = 0; x < NM; ++x) {
      const int i = x / 4, j = x % 4;
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[i], f.b[i][j], acc[j], 0, 0, 0);
      if (x % STEP == 0 && x / STEP < DPW) dma_b(tb, st, x / STEP);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (NM / STEP < DPW) {
#pragma unroll
      for (int v = NM / STEP; v < DPW; ++v) dma_b(tb, st, v);
    }
  };

  Frag f0, f1;
  // prologue: tile 0 in stage 0; tile 1's A loads and B DMA in flight
  load_a(0);
  dma_all(0, 0);
  c1_wait<0>(false);
  store_a(0);
  if (nt > 1) {
    load_a(1);
    dma_all(1, 1);
  }
  __syncthreads();
  frag(0, 0, f0);
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1, nxt = cur ^ 1;
#pragma unroll
    for (int g = 0; g + 1 < NG; ++g) {
      Frag& fc = (g & 1) ? f1 : f0;
      Frag& fn = (g & 1) ? f0 : f1;
      frag(cur, g + 1, fn);
      __builtin_amdgcn_sched_barrier(0);
      mma(fc);
      __builtin_amdgcn_sched_barrier(0);
    }
    Frag& fl = f1;  // the last group's fragments (NG even)
    Frag& ff = f0;  // the next tile's first
    if (t + 1 < nt) {
      // tile t+1: its A loads and B DMA (a tile old) complete, then every
      // wave's; tile t+2's go out after the barrier into tile t's stage
      c1_wait<0>(false);
      store_a(nxt);
      __syncthreads();
      frag(nxt, 0, ff);
      if (t + 2 < nt) {
        load_a(t + 2);
        __builtin_amdgcn_sched_barrier(0);
        mma_dma(fl, t + 2, cur);
      } else {
        __builtin_amdgcn_sched_barrier(0);
        mma(fl);
      }
    } else {
      mma(fl);
    }
  }

  // epilogue: row m0 + wm*16 + 4q + e, columns n .. n+3 of one image
  const int n = n0 + wn * 64 + 4 * r16;
  if (n >= N) return;
  const int img = n / P, pix = n - img * P;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int m = m0 + wm * 16 + 4 * q + e;
    if (m >= p.M) continue;
    const float bi = p.fuse ? p.bias[m] : 0.0f;
    floatx4 v = {acc[0][e], acc[1][e], acc[2][e], acc[3][e]};
    if (p.fuse) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = act_apply_cheap(v[j] + bi, p.act);
    }
    floatx4* cp = reinterpret_cast<floatx4*>(p.C + ((int64_t)img * p.M + m) * P + pix);
    if (p.add) {
      const floatx4 o = *cp;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = o[j] + v[j];
    }
    *cp = v;
  }
}

struct C1Form {
  int bm, bn, bk;
  hipError_t (*fn)(const C1Args&, hipStream_t);
  const char* name;
};

template <class G>
hipError_t launch_c1(const C1Args& a, hipStream_t s) {
  const int64_t blocks = (int64_t)a.tiles_m * ((a.N + G::BN - 1) / G::BN);
  hipLaunchKernelGGL((conv1x1_kernel<G>), dim3((unsigned)blocks), dim3(G::NT), 0, s, a);
  return hipGetLastError();
}

#define TNS_C1(BMv, BKv, WMv, WNv) \
  {BMv, 64 * WNv, BKv, launch_c1<C1G<BMv, BKv, WMv, WNv>>, "conv1x1<" #BMv "x" #WNv "x64x" #BKv ">"}
const C1Form kC1[] = {
    TNS_C1(32, 32, 2, 1),   // 0: 32 x 64
    TNS_C1(64, 32, 4, 1),   // 1: 64 x 64
    TNS_C1(32, 64, 2, 1),   // 2: 32 x 64, 64-deep k-tiles
    TNS_C1(32, 32, 2, 2),   // 3: 32 x 128 — picked (planes of >= 52^2)
    TNS_C1(16, 32, 1, 2),   // 4: 16 x 128
};
#undef TNS_C1
constexpr int kNumC1 = sizeof(kC1) / sizeof(kC1[0]);

}  // namespace

int conv1x1_count() { return kNumC1; }
const char* conv1x1_name(int v) { return v >= 0 && v < kNumC1 ? kC1[v].name : ""; }

// the form for a layer, -1: the other 1x1 paths stay.  Measured at batch 8,
// warm clock (scripts/fwd_sweep.sh, profiles/r06_conv1x1.json): 32 x 128 on
// the planes of >= 52^2 pixels (208^2 0.0426 -> 0.0298 ms, 104^2 0.0222 ->
// 0.0213, 52^2 0.0211 -> 0.0185, the 255-filter 52^2 head 0.0411 -> 0.0316);
// behind conv_tile4's 64 x 32 PF form on the 26^2 planes (0.0193 -> 0.0229)
int conv1x1_pick(int64_t M, int64_t N, int64_t K, int64_t P) {
  (void)M; (void)N;
  if (P % 4 || P < 2704 || K % 32) return -1;
  return 3;
}

// out[c][r] = in[r][c] (rows x cols, 32 x 32 tiles through LDS): the
// backward's transposed weights
__global__ __launch_bounds__(256) void c1_transpose_kernel(const float* __restrict__ in,
                                                           float* __restrict__ out, int rows,
                                                           int cols) {
  __shared__ float t[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    t[y][tx] = r < rows && c < cols ? in[(int64_t)r * cols + c] : 0.0f;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (c < cols && r < rows) out[(int64_t)c * rows + r] = t[tx][y];
  }
}

hipError_t launch_transpose(const float* in, float* out, int64_t rows, int64_t cols,
                            hipStream_t s) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  if (rows > (1 << 26) || cols > (1 << 26)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(c1_transpose_kernel,
                     dim3((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32)), dim3(256), 0,
                     s, in, out, (int)rows, (int)cols);
  return hipGetLastError();
}

hipError_t launch_conv1x1(int v, const float* weights, const float* x, const float* bias,
                          float* out, int64_t batch, int64_t M, int64_t K, int64_t P, int act,
                          hipStream_t s, bool add) {
  if (v < 0 || v >= kNumC1) return hipErrorInvalidValue;
  const C1Form& f = kC1[v];
  const int64_t N = batch * P;
  if (P % 4 || K % f.bk || M < 1 || N < 4 || batch * K * P * 4 > 0x7fffffffLL ||
      M * K * 4 > 0x7fffffffLL || (reinterpret_cast<uintptr_t>(weights) & 15) ||
      (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(out) & 15))
    return hipErrorInvalidValue;
  C1Args a{};
  a.A = weights; a.X = x; a.C = out; a.bias = bias;
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.P = (int)P;
  a.tiles_m = (int)((M + f.bm - 1) / f.bm); a.act = act; a.fuse = bias != nullptr; a.add = add;
  if ((int64_t)a.tiles_m * ((N + f.bn - 1) / f.bn) > 0x7fffffffLL) return hipErrorInvalidValue;
  return f.fn(a, s);
}

}  // namespace tns
