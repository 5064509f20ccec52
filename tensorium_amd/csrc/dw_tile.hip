// dw_tile.hip — the conv backward's weight gradient in the reference's sdot
// order with the im2col matrix generated inside the staging (no col
// workspace, no im2col pass).
//
// TConvolutionalLayer.backward (nConvolutionLayer.pas:571-671) runs, per image
// b, state.input.im2Col (640) then weight_updates += delta_b . col_b^T
// (gemm(NoTrans, Trans), beta = 1, 636-640), whose every element is
// sdot_avx2 (ntensors.pas:1233-1306) over k = pixel: 8 fma lanes, lane l an
// ascending chain over k = l (mod 8) from +0 (the masked tail is that
// chain's last element), then s_l = lane_l + lane_{l+4} and (s0 + s1) +
// (s2 + s3), then ALPHA * sdot, each rounded.  This kernel computes that sum
// for every image at once (grid.y = image) and stores it (BETA_STORE); the
// host adds the images to weight_updates in image order (add_in_order) — the
// roundings of the reference's per-image beta = 1 loop.
//
//   * Each wave owns a 16-row strip x JW 16-column fragments of the block
//     tile and all 8 residue chains of it: acc[r][j], r = k mod 8, one
//     v_mfma_f32_16x16x4_f32 chain per (r, j) (lane quarter q = the q-th of
//     four consecutive chain elements, measured as an ascending fmaf chain,
//     profiles/r01_mfma_order_probe.txt), so the fold is in registers;
//   * a 64-pixel k-tile gives every chain 8 elements = 2 MFMA steps; LDS
//     slots hold a lane's two elements (k = r + 8q + 32s, s = 0, 1) and are
//     read by ds_read_b64, k-permuted images [r][q][row][s];
//   * A = delta rows (float4 loads down the pixels, ds_write_b64 of pixel
//     pairs 32 apart); B[n][k] = the input at tap n = (c, kr, kc) of output
//     pixel k, gathered by dword buffer loads with the window bounds checked
//     through a per-pixel 9-bit tap mask (out-of-window and k >= oH*oW read
//     0: fma(0, 0, x) = x, so zero-filled k adds nothing);
//   * wave columns may carry unequal fragment counts (144 = 5 + 4: waves w
//     and w + 4 share a SIMD, 9 fragments per SIMD either way), so the 52^2
//     YOLOv3 layers (M = 256, N = 1152) make 4 x 8 x 8 images = 256 blocks.
#include <type_traits>

#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int DW_BK = 64;  // pixels per k-tile (8 per residue chain)

template <int BM_, int BN_, int WM_, int WN_, int JA_, int NA_, int SP_ = 2>
struct DGeo {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr int SP = SP_;  // the next tile is stored after residue pair SP (0, 2, 4, 6)
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int J = BN / 16;
  static constexpr int JA = JA_ > 0 ? JA_ : J / WN, NA = JA_ > 0 ? NA_ : WN;
  static constexpr int JB = NA < WN ? (J - NA * JA) / (WN - NA) : 0;
  static constexpr int A_TILE = BM * DW_BK, STAGE = (BM + BN) * DW_BK;  // floats
  static constexpr int UA = BM * 8 / NT;         // A units (row, float4 pair) per thread
  static constexpr int TPK = NT / 32;            // threads per pixel pair of the B gather
  static constexpr int UB = BN / TPK;            // B taps per thread
  static_assert(BM == 16 * WM && BN % 16 == 0 && NW == 8, "geometry");
  static_assert(UA >= 1 && BM * 8 % NT == 0 && BN % TPK == 0, "staging split");
  static_assert(NA * JA + (WN - NA) * JB == J && NA >= 1 && NA <= WN, "wave column split");
  static_assert(2 * STAGE * 4 <= 163840, "LDS");
};

template <class G, int KS>
__global__ __launch_bounds__(G::NT) void dw_tile_kernel(DwArgs p) {
  constexpr int BM = G::BM, BN = G::BN, A_TILE = G::A_TILE, STAGE = G::STAGE;
  constexpr int UA = G::UA, UB = G::UB, TPK = G::TPK;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w % G::WM, wn = w / G::WM;
  const int r16 = lane & 15, q = lane >> 4;
  const int tiles_m = p.M / BM;
  const int tm = blockIdx.x % tiles_m, tn = blockIdx.x / tiles_m, img = blockIdx.y;
  const int m0 = tm * BM, n0 = tn * BN;
  const int HW = p.HW, H = p.H, W = p.W;
  const float* __restrict__ dl = p.delta + (int64_t)img * p.strideA;
  float* __restrict__ part = p.part + (int64_t)img * p.strideP;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.x + (int64_t)img * p.strideX), 0, 4 * p.C * H * W, 0x00020000);

  // ---- A (delta rows): unit = (row m, float4 column c4 < 8) loads pixels
  // 4c4..4c4+3 and 32 later; element e goes to slot (r = 4(c4&1)+e,
  // q' = (c4>>1)&3, m), components s = 0, 1 ----------------------------------
  int a_m[UA], a_c4[UA];
#pragma unroll
  for (int u = 0; u < UA; ++u) {
    const int idx = tid + G::NT * u;
    a_m[u] = idx % BM;  // lanes along rows: conflict-free ds_write_b64
    a_c4[u] = idx / BM;
  }
  float4 ra0[UA], ra1[UA];
  auto load_a = [&](int k0) {
#pragma unroll
    for (int u = 0; u < UA; ++u) {
      const float* row = dl + (int64_t)(m0 + a_m[u]) * HW;
      const int k = k0 + 4 * a_c4[u];
      if (p.va) {  // HW % 4 == 0: a float4 is wholly inside or outside
        ra0[u] = k < HW ? *reinterpret_cast<const float4*>(row + k) : make_float4(0, 0, 0, 0);
        ra1[u] = k + 32 < HW ? *reinterpret_cast<const float4*>(row + k + 32)
                             : make_float4(0, 0, 0, 0);
      } else {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = k + e < HW ? row[k + e] : 0.0f;
          v[4 + e] = k + 32 + e < HW ? row[k + 32 + e] : 0.0f;
        }
        ra0[u] = make_float4(v[0], v[1], v[2], v[3]);
        ra1[u] = make_float4(v[4], v[5], v[6], v[7]);
      }
    }
  };
  auto store_a = [&](float* as) {
#pragma unroll
    for (int u = 0; u < UA; ++u) {
      const int c4 = a_c4[u];
      float* d = as + ((4 * (c4 & 1) * 4 + ((c4 >> 1) & 3)) * BM + a_m[u]) * 2;
      constexpr int RS = 4 * BM * 2;  // next residue
      *reinterpret_cast<float2*>(d) = make_float2(ra0[u].x, ra1[u].x);
      *reinterpret_cast<float2*>(d + RS) = make_float2(ra0[u].y, ra1[u].y);
      *reinterpret_cast<float2*>(d + 2 * RS) = make_float2(ra0[u].z, ra1[u].z);
      *reinterpret_cast<float2*>(d + 3 * RS) = make_float2(ra0[u].w, ra1[u].w);
    }
  };

  // ---- B (im2col generated): thread = pixel pair (kk, kk + 32) x taps
  // n = n0 + tn16 + 16u (lanes along the pixels: 128 contiguous bytes per tap
  // and wave-instruction); tap constants fixed for the launch.  Slot columns
  // are XOR-swizzled by (r + 8q') & 15 within 16-column groups, so the 16
  // pixels of a store group hit 16 different slots of one row group -------
  static_assert(TPK == 16, "16 tap groups");
  const int kk = tid & 31, tn16 = tid >> 5;
  // per tap: element offset c*H*W + kr*d*W + kc*d (< 2^27, checked by the
  // host) in bits 0..27, the tap index kr*KS + kc in bits 28..31
  unsigned b_tap[UB];
#pragma unroll
  for (int u = 0; u < UB; ++u) {
    const int n = n0 + tn16 + TPK * u;
    const int c = n / (KS * KS), t = n - c * KS * KS;
    const int kr = t / KS, kc = t - kr * KS;
    b_tap[u] = (unsigned)(c * H * W + kr * p.dil * W + kc * p.dil) | (unsigned)t << 28;
  }
  // pixel state of the two pixels (advanced by DW_BK per tile)
  int py[2], px[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = kk + 32 * h;
    py[h] = k / p.oW;
    px[h] = k - py[h] * p.oW;
  }
  const int dq = DW_BK / p.oW, dr = DW_BK - dq * p.oW;
  auto advance = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      px[h] += dr;
      py[h] += dq;
      if (px[h] >= p.oW) { px[h] -= p.oW; ++py[h]; }
    }
  };
  float rb[2][UB];
  auto gather_b = [&](int k0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int iy0 = py[h] * p.stride - p.pad, ix0 = px[h] * p.stride - p.pad;
      unsigned mask = 0;
#pragma unroll
      for (int kr = 0; kr < KS; ++kr)
#pragma unroll
        for (int kc = 0; kc < KS; ++kc)
          mask |= (unsigned)(((unsigned)(iy0 + kr * p.dil) < (unsigned)H) &
                             ((unsigned)(ix0 + kc * p.dil) < (unsigned)W))
                  << (kr * KS + kc);
      if (k0 + kk + 32 * h >= HW) mask = 0;
      const unsigned base = (unsigned)(iy0 * W + ix0);
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const bool ok = __builtin_amdgcn_ubfe(mask, b_tap[u] >> 28, 1) != 0;
        const unsigned off = ok ? 4u * (base + (b_tap[u] & 0x0fffffffu)) : 0x80000000u;
        rb[h][u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, off, 0, 0));
      }
    }
  };
  // slot (r = kk & 7, q' = (kk >> 3) & 3, n ^ (kk & 15)), components s = 0, 1
  // (kk, kk + 32)
  const int b_dst = (((kk & 7) * 4 + ((kk >> 3) & 3)) * BN + (tn16 ^ (kk & 15))) * 2;
  auto store_b = [&](float* bs) {
#pragma unroll
    for (int u = 0; u < UB; ++u)
      *reinterpret_cast<float2*>(bs + b_dst + 2 * TPK * u) = make_float2(rb[0][u], rb[1][u]);
  };

  const int nt = (HW + DW_BK - 1) / DW_BK;

  // ---- the main loop and epilogue for a wave of JW fragments from column
  // fragment coff ----------------------------------------------------------
  auto run = [&](auto JWC, const int coff) {
    constexpr int JW = decltype(JWC)::value;
    floatx4 acc[8][JW];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int j = 0; j < JW; ++j) acc[r][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // fragments of residue r: the A slot and JW B slots, two steps each
    struct Fr {
      float2 a, b[JW];
    };
    auto frag = [&](const float* st, int r, Fr& f) {
      f.a = *reinterpret_cast<const float2*>(st + ((r * 4 + q) * BM + wm * 16 + r16) * 2);
      const float* bp = st + A_TILE + ((r * 4 + q) * BN + coff * 16 + (r16 ^ ((r + 8 * q) & 15))) * 2;
#pragma unroll
      for (int j = 0; j < JW; ++j) f.b[j] = *reinterpret_cast<const float2*>(bp + 32 * j);
    };
    auto mma = [&](int r, const Fr& f) {
#pragma unroll
      for (int j = 0; j < JW; ++j)
        acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a.x, f.b[j].x, acc[r][j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < JW; ++j)
        acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a.y, f.b[j].y, acc[r][j], 0, 0, 0);
    };
    if (nt > 0) {
      load_a(0);
      gather_b(0);
      store_a(smem);
      store_b(smem + A_TILE);
      __syncthreads();
    }
    for (int t = 0; t < nt; ++t) {
      const float* cur = smem + (t & 1) * STAGE;
      float* nxt = smem + ((t + 1) & 1) * STAGE;
      const bool more = t + 1 < nt;
      if (more) {
        advance();
        load_a((t + 1) * DW_BK);
        gather_b((t + 1) * DW_BK);
      }
      Fr f0, f1;
      frag(cur, 0, f0);
#pragma unroll
      for (int r = 0; r < 8; r += 2) {
        frag(cur, r + 1, f1);
        __builtin_amdgcn_sched_barrier(0);
        mma(r, f0);
        if (r + 2 < 8) frag(cur, r + 2, f0);
        __builtin_amdgcn_sched_barrier(0);
        mma(r + 1, f1);
        if (r == G::SP && more) {  // the next tile's stores
          __builtin_amdgcn_sched_barrier(0);
          store_a(nxt);
          store_b(nxt + A_TILE);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __syncthreads();
    }
    // ---- epilogue: s_l = lane_l + lane_{l+4}, (s0 + s1) + (s2 + s3), alpha
    const float alpha = p.alpha;
#pragma unroll
    for (int j = 0; j < JW; ++j) {
      const int n = n0 + (coff + j) * 16 + r16;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * 16 + 4 * q + e;
        const float s0 = acc[0][j][e] + acc[4][j][e], s1 = acc[1][j][e] + acc[5][j][e];
        const float s2 = acc[2][j][e] + acc[6][j][e], s3 = acc[3][j][e] + acc[7][j][e];
        const float dot = (s0 + s1) + (s2 + s3);
        part[(int64_t)m * p.N + n] = alpha * dot;
      }
    }
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

template <class G>
hipError_t launch_dw(const DwArgs& a, int ks, hipStream_t s) {
  if (a.M % G::BM || a.N % G::BN || a.M <= 0 || a.N <= 0 || a.HW <= 0) return hipErrorInvalidValue;
  const int64_t tiles = (int64_t)(a.M / G::BM) * (a.N / G::BN);
  if (tiles > 0x7fffffff || a.batch > 65535) return hipErrorInvalidValue;
  if (ks == 3)
    hipLaunchKernelGGL((dw_tile_kernel<G, 3>), dim3((unsigned)tiles, (unsigned)a.batch), dim3(G::NT),
                       0, s, a);
  else if (ks == 1)
    hipLaunchKernelGGL((dw_tile_kernel<G, 1>), dim3((unsigned)tiles, (unsigned)a.batch), dim3(G::NT),
                       0, s, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

struct DwInfo {
  int bm, bn;
  hipError_t (*fn)(const DwArgs&, int, hipStream_t);
  const char* name;
};
#define TNS_DW(BMv, BNv, WMv, WNv, JAv, NAv, SPv)                                       \
  {BMv, BNv, launch_dw<DGeo<BMv, BNv, WMv, WNv, JAv, NAv, SPv>>,                        \
   "dw_tile<" #BMv "x" #BNv ",w" #WMv "x" #WNv ",j" #JAv "x" #NAv ",s" #SPv ">"}
const DwInfo kDw[] = {
    TNS_DW(64, 144, 4, 2, 5, 1, 2),  // 0: 52^2 (4 x 8 blocks per image)
    TNS_DW(64, 128, 4, 2, 0, 0, 2),  // 1
    TNS_DW(64, 64, 4, 2, 0, 0, 2),   // 2
    TNS_DW(128, 64, 8, 1, 0, 0, 2),  // 3
    TNS_DW(64, 144, 4, 2, 5, 1, 6),  // 4: stores after the last-but-one residue pair
    TNS_DW(64, 128, 4, 2, 0, 0, 6),  // 5
    TNS_DW(64, 64, 4, 2, 0, 0, 6),   // 6
    TNS_DW(64, 144, 4, 2, 5, 1, 4),  // 7
};
#undef TNS_DW
constexpr int kNumDw = sizeof(kDw) / sizeof(kDw[0]);

}  // namespace

int dw_tile_count() { return kNumDw; }
const char* dw_tile_name(int v) { return v >= 0 && v < kNumDw ? kDw[v].name : ""; }

// Measured per YOLOv3 layer (scripts/conv_bwd_layers.py --dw-tile, whole
// backward call at batch 8, profiles/r03_dw_tile.json): the 64 x 144 form on
// the 3x3 layers with 256 filters over 128 channels (52^2 outputs: exactly
// 256 blocks at batch 8) — 11 layers 3.94 -> 3.84 ms, the im2col pass gone
// and the product about as fast as im2col + the sdot kernels; on the 26^2 /
// 13^2 layers the product itself runs slower than the sdot kernels by about
// the im2col time it saves (3.69 -> 3.81, 3.15 -> 3.14 ms), so they, the
// 104^2+ planes (few tall tiles over a long k) and the 1x1 layers keep
// im2col + sdot.
int dw_tile_pick(const DwArgs& a, int ks) {
  if (ks != 3 || a.M != 256 || a.N != 1152) return -1;
  const int64_t blocks = (int64_t)(a.M / 64) * (a.N / 144) * a.batch;
  return blocks >= 256 ? 0 : -1;
}

hipError_t launch_dw_tile(int v, const DwArgs& a, int ks, hipStream_t s) {
  if (v < 0 || v >= kNumDw) return hipErrorInvalidValue;
  return kDw[v].fn(a, ks, s);
}

}  // namespace tns
