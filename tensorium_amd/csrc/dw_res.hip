// dw_res.hip — the conv backward's weight gradient in the reference's sdot
// order, as residue chains run one after another over residue-major operands.
//
// TConvolutionalLayer.backward (nConvolutionLayer.pas:571-671) adds, image by
// image, weight_updates += delta_b . col_b^T (gemm(NoTrans, Trans), beta = 1,
// 636-640) whose every element is sdot_avx2 over k = output pixel
// (ntensors.pas:1233-1306, 1957-2005): 8 fma lanes, lane l an ascending chain
// over k = l (mod 8) from +0 (the masked tail is that chain's last element),
// then s_l = lane_l + lane_{l+4}, dot = (s0 + s1) + (s2 + s3), sum = ALPHA *
// dot, C = C + sum — each rounded.
//
// The kernels elsewhere keep a tile's eight residue chains side by side (8
// waves, or 8 accumulator sets per wave), which holds the output tile to 32 x
// 64 (sgemm_sdot.hip) or 16 x 80 per wave (dw_tile.hip).  Here the operands
// are first rearranged residue-major, X'[row][r][i] = X[row][r + 8 i] (zero
// for r + 8 i >= K, rows padded to K4 = 32-aligned K1 = ceil(K / 8)), so the
// chain of residue r is a plain ascending-k product over a contiguous slice:
//
//   * a block owns a BM x BN output tile (2 x 2 waves, 32x32x2 MFMA tiles,
//     each an ascending fmaf chain, profiles/r01_mfma_order_probe.txt) and
//     runs R of the 8 residue chains in sequence, in sdot's pairing order
//     (r, r + 4, ...); a finished chain is folded into registers at once
//     (s_l = lane_l + lane_{l+4}, then s0 + s1 ...), so only a few
//     accumulator sets are live and the tile is as large as a plain GEMM's;
//   * grid.y = residue group (8 / R groups, each its own partial plane),
//     grid.z = image; a second kernel forms dot from the group planes in
//     sdot's order and adds ALPHA * dot to weight_updates image by image;
//   * both operands stream global -> LDS by 16-byte LDS-DMA into row images
//     [row][32 k] with the 16-byte k-chunks XOR-swizzled by row (as
//     sgemm_nn_w4.hip's A), two stages, one barrier per k-tile; the last
//     k-tile of a chain runs only the steps its (zero-padded) k covers.
//
// The rearranged delta (rows = filters) and col (rows = (c, kr, kc), or the
// input planes themselves for a 1x1 / stride-1 layer) are written by one pass
// each over their sources (reads coalesced, 32-byte write sectors).
#include <cstdlib>
#include <algorithm>

#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int RBK = 32;  // k per tile

__device__ __forceinline__ void dma16(const float* sbase, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

struct ResArgs {
  const float* A;  // [batch][M][8][K4] (delta')
  const float* B;  // [batch][N][8][K4] (col')
  float* P;        // [batch][G][M][N]
  int M, N, K1, K4, G;
  int64_t strideA, strideB, strideP;
  // (IF) every image in one block: weight_updates [M][N] += ALPHA * dot_b
  float* W;
  float alpha;
  int batch;
};

// R residues per block: the residue of position rho in group g, in sdot's
// pairing order ((r, r + 4) pairs, pairs ascending)
template <int R>
__device__ __forceinline__ int residue_of(int g, int rho) {
  if constexpr (R == 1) return g;
  return (R / 2) * g + (rho >> 1) + 4 * (rho & 1);
}

// IF: the block runs every image in turn (grid.z = 1, R = 8) and adds
// ALPHA * dot of each to the weight_updates tile it holds in registers, in
// image order — no partial planes and no second pass (the 13^2 planes, whose
// 1024 x 4608 partials per image cost more to write and re-read than the
// product)
template <int BM, int BN, int R, bool IF = false>
__global__ __launch_bounds__(256, 2) void dw_res_kernel(
    ResArgs p) {
  static_assert(!IF || R == 8, "image folding needs the whole dot in the block");
  constexpr int TI = BM / 64, TJ = BN / 64;  // 32x32 tiles of a wave (2 x 2 waves)
  constexpr int A_T = BM * RBK, STAGE = (BM + BN) * RBK;  // floats
  constexpr int GA = BM / 8, GT = (BM + BN) / 8, GPW = GT / 4;  // DMA row groups
  static_assert(TI >= 1 && TJ >= 1 && GT % 4 == 0, "geometry");
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1, l31 = lane & 31, h = lane >> 5;
  const int tiles_m = p.M / BM;
  // XCD-contiguous tiles (blocks go to the 8 XCDs round-robin): each XCD
  // takes one contiguous run of the m-fastest tile list — a few column tiles
  // with every row tile — so its L2 holds those col' rows while delta'
  // streams past, instead of every XCD streaming all of col'
  int tile;
  {
    const int nb = (int)gridDim.x, bid = (int)blockIdx.x;
    const int xcd = bid & 7, q = nb >> 3, r = nb & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int m0 = (tile % tiles_m) * BM, n0 = (tile / tiles_m) * BN;
  const int g = blockIdx.y;
  const int64_t img = IF ? 0 : blockIdx.z;
  const int64_t ld = 8LL * p.K4;  // row stride, floats
  const float* A = p.A + img * p.strideA + (int64_t)m0 * ld;
  const float* B = p.B + img * p.strideB + (int64_t)n0 * ld;

  // DMA: row group q (8 rows x 128 B) -> LDS bytes q * 1024; lane -> row
  // 8q + (lane >> 3), slot lane & 7 <- k-chunk (lane & 7) ^ ((row >> 1) & 7)
  // (q even: (arow >> 1) & 7, q odd: that ^ 4)
  const int arow = lane >> 3;
  const unsigned voff0 = (unsigned)(arow * ld * 4) + 16u * (unsigned)((lane & 7) ^ ((arow >> 1) & 7));
  const unsigned voff1 =
      (unsigned)(arow * ld * 4) + 16u * (unsigned)((lane & 7) ^ (((arow >> 1) & 7) ^ 4));
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)smem;
  auto issue = [&](int residue, int kt, int st, int b) {
    const int64_t koff = (int64_t)residue * p.K4 + (int64_t)kt * RBK;
    const float* Ab = IF ? A + b * p.strideA : A;
    const float* Bb = IF ? B + b * p.strideB : B;
    const unsigned sb = lds0 + (unsigned)(st * STAGE * 4);
#pragma unroll
    for (int u = 0; u < GPW; ++u) {
      const int q = wid * GPW + u;
      if (q < GA)
        dma16(Ab + (int64_t)(8 * q) * ld + koff, (q & 1) ? voff1 : voff0, sb + (unsigned)(q * 1024));
      else
        dma16(Bb + (int64_t)(8 * (q - GA)) * ld + koff, ((q - GA) & 1) ? voff1 : voff0,
              sb + (unsigned)(A_T * 4 + (q - GA) * 1024));
    }
  };

  // fragments of step group q (steps 4q .. 4q+3, k = 8q + h + 2j): the
  // rearranged rows hold each 32-k block as [h][q][j] (kperm), so a lane's
  // four steps are one 16-byte chunk, 4h + q, at slot (4h + q) ^ ((R >> 1) &
  // 7); the wave's rows start at multiples of 32, so (R >> 1) & 7 =
  // (l31 >> 1) & 7
  const int swz = (l31 >> 1) & 7;
  const int a_row = (wm * (BM / 2) + l31) * RBK;
  const int b_row = A_T + (wn * (BN / 2) + l31) * RBK;
  struct Frag {
    floatx4 a[TI], b[TJ];
  };
  auto frag = [&](const float* st, int q, Frag& f) {
    const int ka = 4 * ((4 * h + q) ^ swz);
#pragma unroll
    for (int i = 0; i < TI; ++i)
      f.a[i] = *reinterpret_cast<const floatx4*>(st + a_row + 32 * RBK * i + ka);
#pragma unroll
    for (int j = 0; j < TJ; ++j)
      f.b[j] = *reinterpret_cast<const floatx4*>(st + b_row + 32 * RBK * j + ka);
  };
  floatx16 acc[TI][TJ];
  auto zero = [&](floatx16 (&x)[TI][TJ]) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) x[i][j][e] = 0.0f;
  };
  zero(acc);
  auto mma = [&](const Frag& f) {
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[i][st], f.b[j][st], acc[i][j], 0,
                                                           0, 0);
  };
  // step groups 0 .. groups-2 of a k-tile (4 groups, or `groups`, 1 .. 4,
  // for a chain's last tile: the rest is zero padding) from fragments f0 =
  // group 0; leaves the last group's fragments in f1 (its MFMAs are issued
  // by the caller, after the barrier)
  Frag f0, f1;
  auto compute = [&](const float* st, int groups) {
#pragma unroll
    for (int q = 0; q < RBK / 8; q += 2) {
      if (q + 1 < groups) {  // (wave-uniform)
        frag(st, q + 1, f1);
        mma(f0);
        if (q + 2 < groups) {
          frag(st, q + 2, f0);
          mma(f1);
        }
      } else if (q + 1 == groups) {
        f1 = f0;  // (an odd count: group q is the last)
      }
    }
  };
  // finished chains folded in sdot's order: even positions wait in P, odd
  // ones give s = P + acc; R = 4: X = s0 (+ s1); R = 8: X = s0 + s1, Y = s2 + s3
  floatx16 P[TI][TJ], X[TI][TJ], Y[TI][TJ];
  auto fold = [&](int rho) {
    if constexpr (R == 1) return;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        if ((rho & 1) == 0) {
          P[i][j] = acc[i][j];
        } else {
          const floatx16 s = P[i][j] + acc[i][j];
          if constexpr (R == 2) {
            P[i][j] = s;
          } else if constexpr (R == 4) {
            X[i][j] = rho == 1 ? s : X[i][j] + s;
          } else {
            if (rho == 1) X[i][j] = s;
            else if (rho == 3) X[i][j] = X[i][j] + s;
            else if (rho == 5) Y[i][j] = s;
            else Y[i][j] = Y[i][j] + s;
          }
        }
      }
    zero(acc);
  };

  const int nt = (p.K1 + RBK - 1) / RBK;
  // the last tile's step groups: its k rounded up to 8 (K4 is a multiple of
  // 32, so the rest of the tile is zero; the chain's masked tail element,
  // i = K1 - 1, is always run: sdot's one fma(0, 0, lane) on the residues
  // past K, and the further zero steps of the group leave the lane as it is)
  const int last_groups = (p.K1 - (nt - 1) * RBK + 7) / 8;
  const int TI1 = R * nt;                // tiles of one image
  const int T = IF ? p.batch * TI1 : TI1;
  // the barrier that publishes tile t+1 sits before tile t's last step: tile
  // t+1's first fragments are read under that step's MFMAs, and the DMA of
  // tile t+2 (into tile t's stage, every read of which completed before the
  // barrier) goes out a whole tile ahead of its use
  auto tile_of = [&](int t, int& res, int& kt, int& b) {
    b = IF ? t / TI1 : 0;
    const int u = t - b * TI1;
    res = residue_of<R>(g, u / nt);
    kt = u - (u / nt) * nt;
  };
  // (IF) the weight_updates tile, accumulated image by image
  floatx16 Wt[IF ? TI : 1][IF ? TJ : 1];
  auto w_at = [&](int i, int j, int e, int& row, int& col) {
    col = n0 + wn * (BN / 2) + 32 * j + l31;
    row = m0 + wm * (BM / 2) + 32 * i + 8 * (e >> 2) + 4 * h + (e & 3);
  };
  if constexpr (IF) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          int row, col;
          w_at(i, j, e, row, col);
          Wt[i][j][e] = col < p.N ? p.W[(int64_t)row * p.N + col] : 0.0f;
        }
  }
  {
    int r0, k0, b0;
    tile_of(0, r0, k0, b0);
    issue(r0, k0, 0, b0);
    if (T > 1) {
      tile_of(1, r0, k0, b0);
      issue(r0, k0, 1, b0);
      // (this wave's DMA of tile 0 landed: the newer GPW may stay in flight)
      if constexpr (GPW == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if constexpr (GPW == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if constexpr (GPW == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    frag(smem, 0, f0);
  }
  for (int t = 0; t < T; ++t) {
    int rt, kt, bt;
    tile_of(t, rt, kt, bt);
    const int u = t - bt * TI1;  // tile within its image
    compute(smem + (t & 1) * STAGE, kt == nt - 1 ? last_groups : RBK / 8);
    if (t + 1 < T) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile t+1
      __syncthreads();  // every wave's; every read of tile t complete
      if (t + 2 < T) {
        int r2, k2, b2;
        tile_of(t + 2, r2, k2, b2);
        issue(r2, k2, t & 1, b2);
      }
      frag(smem + ((t + 1) & 1) * STAGE, 0, f0);
    }
    mma(f1);  // the tile's last step
    if (kt == nt - 1) fold(u / nt);
    if constexpr (IF) {
      if (u == TI1 - 1) {  // image bt done: C := C + ALPHA * dot, (s0+s1)+(s2+s3)
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            const floatx16 dot = X[i][j] + Y[i][j];
            Wt[i][j] = Wt[i][j] + p.alpha * dot;
          }
      }
    }
  }
  if constexpr (IF) {
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          int row, col;
          w_at(i, j, e, row, col);
          if (col < p.N) p.W[(int64_t)row * p.N + col] = Wt[i][j][e];
        }
    return;
  }

  // ---- the group's partial plane -------------------------------------------
  float* out = p.P + img * p.strideP + (int64_t)g * p.M * p.N;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      floatx16 v;
      if constexpr (R == 1) v = acc[i][j];
      else if constexpr (R == 2) v = P[i][j];
      else if constexpr (R == 4) v = X[i][j];
      else v = X[i][j] + Y[i][j];  // (s0 + s1) + (s2 + s3)
      const int col = n0 + wn * (BN / 2) + 32 * j + l31;
      if (col >= p.N) continue;  // (padded col rows)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wm * (BM / 2) + 32 * i + 8 * (e >> 2) + 4 * h + (e & 3);
        out[(int64_t)row * p.N + col] = v[e];
      }
    }
}

// dot from the G group planes of each image in sdot's order, then
// C := C + ALPHA * dot image by image (the reference's beta = 1 loop)
__global__ __launch_bounds__(256) void dw_res_accumulate_kernel(float* __restrict__ C,
                                                                const float* __restrict__ P,
                                                                int64_t mn, int G, int64_t strideP,
                                                                int batch, float alpha) {
  for (int64_t o = blockIdx.x * 256LL + threadIdx.x; o < mn; o += (int64_t)gridDim.x * 256) {
    float c = C[o];
    for (int b = 0; b < batch; ++b) {
      const float* q = P + b * strideP + o;
      float dot;
      if (G == 1)
        dot = q[0];
      else if (G == 2)
        dot = q[0] + q[mn];
      else if (G == 4)
        dot = (q[0] + q[mn]) + (q[2 * mn] + q[3 * mn]);
      else
        dot = ((q[0] + q[4 * mn]) + (q[mn] + q[5 * mn])) +
              ((q[2 * mn] + q[6 * mn]) + (q[3 * mn] + q[7 * mn]));
      c = c + alpha * dot;
    }
    C[o] = c;
  }
}

// float4 form of the same (mn % 4 == 0, 16-byte aligned planes), per element
// the same operations in the same order; the G group planes of 8 / G images
// are loaded before the adds so eight 16-byte reads a lane are in flight
// (the scalar form holds one 4-byte read a lane: latency-bound near 1.5 TB/s)
template <int G>
__global__ __launch_bounds__(256) void dw_res_accumulate4_kernel(float4* __restrict__ C,
                                                                 const float4* __restrict__ P,
                                                                 int64_t mn4, int64_t strideP4,
                                                                 int batch, float alpha) {
  constexpr int U = 8 / G;  // images per load group
  for (int64_t o = blockIdx.x * 256LL + threadIdx.x; o < mn4; o += (int64_t)gridDim.x * 256) {
    float4 c = C[o];
    for (int b0 = 0; b0 < batch; b0 += U) {
      float4 v[U][G];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (b0 + u < batch) {
#pragma unroll
          for (int g = 0; g < G; ++g) v[u][g] = P[(b0 + u) * strideP4 + g * mn4 + o];
        }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (b0 + u < batch) {
          const float4* q = v[u];
          float4 dot;
#define TNS_ACC_DOT(f)                                                                           \
  if constexpr (G == 1)                                                                          \
    dot.f = q[0].f;                                                                              \
  else if constexpr (G == 2)                                                                     \
    dot.f = q[0].f + q[1].f;                                                                     \
  else if constexpr (G == 4)                                                                     \
    dot.f = (q[0].f + q[1].f) + (q[2].f + q[3].f);                                               \
  else                                                                                           \
    dot.f = ((q[0].f + q[4].f) + (q[1].f + q[5].f)) + ((q[2].f + q[6].f) + (q[3].f + q[7].f)); \
  c.f = c.f + alpha * dot.f;
          TNS_ACC_DOT(x)
          TNS_ACC_DOT(y)
          TNS_ACC_DOT(z)
          TNS_ACC_DOT(w)
#undef TNS_ACC_DOT
        }
    }
    C[o] = c;
  }
}

// Residue-major rearrangement: dst[row][r][i] = v(row, r + 8 i) for i < K4,
// v(row, p) = 0 for p >= K.  A block takes CH consecutive p of one row (CH =
// 256 .. 2048 by row length; grid.y = row from row0, grid.x = chunk): all of
// a thread's reads issued together, coalesced, into LDS, then each residue's
// CH/8 consecutive i written as one run (LDS row stride 264: both phases
// conflict-free).
constexpr int RCH = 2048, RLD = 264;
// im2col_res_lds_kernel's input stage (dynamic LDS), beside its 16.9 KB
// transpose buffers: two blocks a CU
constexpr int64_t kResStageBytes = 44 * 1024;

// position of chain element i in its row: each 32-element block stored as
// [h][q][j] for element 32 b + 8 q + h + 2 j (the kernel's step groups)
__device__ __forceinline__ int kperm(int i) {
  const int k = i & 31;
  return (i & ~31) | ((k & 1) << 4) | ((k >> 3) << 2) | ((k >> 1) & 3);
}

template <int CH, class Src>
__device__ __forceinline__ void res_chunk(Src&& src, float* __restrict__ drow, int K4) {
  __shared__ float t[8 * RLD];
  const int tid = threadIdx.x, base = (int)blockIdx.x * CH;
  float v[CH / 256];  // all of a thread's loads in flight before the stores
#pragma unroll
  for (int j = 0; j < CH / 256; ++j) v[j] = src(base + tid + 256 * j, j);
#pragma unroll
  for (int j = 0; j < CH / 256; ++j) {
    const int pl = tid + 256 * j;
    t[(pl & 7) * RLD + (pl >> 3)] = v[j];
  }
  __syncthreads();
  // written as 16-byte pieces: piece a of a 32-element block holds elements
  // e = (a >> 2) + 8 (a & 3) + 2 b, b = 0..3 (kperm); a residue's CH/8
  // elements are CH/32 consecutive pieces
  constexpr int PIECES = CH / 32;  // per residue
  const int i0 = (int)blockIdx.x * (CH / 8);
#pragma unroll
  for (int u = 0; u < (8 * PIECES + 255) / 256; ++u) {
    const int idx = tid + 256 * u;
    if (8 * PIECES % 256 == 0 || idx < 8 * PIECES) {
      const int r = idx / PIECES, pc = idx - r * PIECES, kb = pc >> 3, a = pc & 7;
      if (i0 + 32 * kb < K4) {
        const int e = 32 * kb + (a >> 2) + 8 * (a & 3);
        const float* tr = t + r * RLD + e;
        *reinterpret_cast<float4*>(drow + (int64_t)r * K4 + i0 + 4 * pc) =
            make_float4(tr[0], tr[2], tr[4], tr[6]);
      }
    }
  }
}

template <int CH>
__global__ __launch_bounds__(256) void res_permute_kernel(const float* __restrict__ src,
                                                          int64_t srcImg, float* __restrict__ dst,
                                                          int64_t dstImg, int rows, int K, int K4,
                                                          int row0) {
  const int ra = row0 + (int)blockIdx.y;
  const int b = ra / rows, row = ra - b * rows;
  const float* s = src + b * srcImg + (int64_t)row * K;
  res_chunk<CH>([&](int pp, int) { return pp < K ? s[pp] : 0.0f; },
                dst + b * dstImg + (int64_t)row * 8 * K4, K4);
}

// the im2col matrix (rows n = (c, kr, kc), columns = output pixels; the
// reference's sim2Col, ntensors.pas:11415-11532) written residue-major; a
// thread's pixels p0 + 256 j walk the output plane by a fixed (rows,
// columns) step, one division per thread
template <int CH>
__global__ __launch_bounds__(256) void im2col_res_kernel(const float* __restrict__ x, int64_t xImg,
                                                         float* __restrict__ dst, int64_t dstImg,
                                                         int H, int W, int kH, int kW, int sY,
                                                         int sX, int pH, int pW, int dY, int dX,
                                                         int oW, int HWo, int rows, int K4,
                                                         int row0) {
  const int ra = row0 + (int)blockIdx.y;
  const int b = ra / rows, n = ra - b * rows;
  const int taps = kH * kW, c = n / taps, t = n - c * taps, kr = t / kW, kc = t - kr * kW;
  const float* xc = x + b * xImg + (int64_t)c * H * W;
  const int p0 = (int)blockIdx.x * CH + (int)threadIdx.x;
  const int dy = 256 / oW, dx = 256 - dy * oW;
  int oy = p0 / oW, ox = p0 - oy * oW;
  res_chunk<CH>(
      [&](int pp, int j) {
        if (j > 0) {  // pp = p0 + 256 j: advance the pixel by 256
          ox += dx;
          oy += dy;
          if (ox >= oW) {
            ox -= oW;
            ++oy;
          }
        }
        if (pp >= HWo) return 0.0f;
        const int iy = oy * sY - pH + kr * dY, ix = ox * sX - pW + kc * dX;
        return ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) ? xc[iy * W + ix] : 0.0f;
      },
      dst + b * dstImg + (int64_t)n * 8 * K4, K4);
}

// The same rows from one block per (image, channel, chunk of output pixels):
// the input rows the chunk's windows cover are staged in LDS ONCE (one
// contiguous span of the plane, coalesced), and the block writes the chunk of
// all kH * kW rows n = (c, kr, kc) from there, tap after tap — each input
// element is fetched once instead of once per tap (the per-row kernel above
// reads a plane kH * kW times, from different blocks on different XCDs).
// Per tap: the values go through a residue-transpose buffer (double-buffered,
// one barrier a tap) and leave as res_chunk's 16-byte pieces.
template <int CH>
__global__ __launch_bounds__(256) void im2col_res_lds_kernel(
    const float* __restrict__ x, int64_t xImg, float* __restrict__ dst, int64_t dstImg, int C,
    int H, int W, int kH, int kW, int sY, int sX, int pH, int pW, int dY, int dX, int oW, int HWo,
    int rows, int K4, int plane0) {
  extern __shared__ float stage[];
  __shared__ float tb[2][8 * RLD];
  const int pa = plane0 + (int)blockIdx.y;  // (image, channel)
  const int b = pa / C, c = pa - b * C;
  const int tid = threadIdx.x, base = (int)blockIdx.x * CH;
  const float* xc = x + b * xImg + (int64_t)c * H * W;
  // the input rows of the chunk's output rows (none past the plane's end)
  const int oy_lo = base / oW, oy_hi = min((base + CH - 1) / oW, (HWo - 1) / oW);
  const int r_lo = max(oy_lo * sY - pH, 0), r_hi = min(oy_hi * sY - pH + (kH - 1) * dY, H - 1);
  const int span = base < HWo && r_hi >= r_lo ? (r_hi - r_lo + 1) * W : 0;
  {
    const float* src = xc + (int64_t)r_lo * W;
    int e = tid;
    for (; e + 768 < span; e += 1024) {  // (four loads in flight)
      const float v0 = src[e], v1 = src[e + 256], v2 = src[e + 512], v3 = src[e + 768];
      stage[e] = v0;
      stage[e + 256] = v1;
      stage[e + 512] = v2;
      stage[e + 768] = v3;
    }
    for (; e < span; e += 256) stage[e] = src[e];
  }
  // a thread's pixels base + tid + 256 j: window origin in the plane, and the
  // origin's offset in the stage (oy0 = -1 << 20 marks a pixel past HWo)
  constexpr int NJ = CH / 256;
  int iy0[NJ], ix0[NJ];
  {
    const int p0 = base + tid, dy = 256 / oW, dx = 256 - dy * oW;
    int oy = p0 / oW, ox = p0 - oy * oW;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if (j > 0) {
        ox += dx;
        oy += dy;
        if (ox >= oW) {
          ox -= oW;
          ++oy;
        }
      }
      const bool in = p0 + 256 * j < HWo;
      iy0[j] = in ? oy * sY - pH : -(1 << 20);
      ix0[j] = ox * sX - pW;
    }
  }
  __syncthreads();
  constexpr int PIECES = CH / 32;  // 16-byte pieces per residue and tap
  const int i0 = (int)blockIdx.x * (CH / 8);
  const int taps = kH * kW;
  float* drow0 = dst + b * dstImg + (int64_t)c * taps * 8 * K4;
  for (int t = 0, kr = 0, kc = 0; t < taps; ++t) {
    float* tt = tb[t & 1];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int pl = tid + 256 * j;
      const int iy = iy0[j] + kr * dY, ix = ix0[j] + kc * dX;
      const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      tt[(pl & 7) * RLD + (pl >> 3)] = ok ? stage[(iy - r_lo) * W + ix] : 0.0f;
    }
    __syncthreads();
    float* drow = drow0 + (int64_t)t * 8 * K4;
#pragma unroll
    for (int u = 0; u < (8 * PIECES + 255) / 256; ++u) {
      const int idx = tid + 256 * u;
      if (8 * PIECES % 256 == 0 || idx < 8 * PIECES) {
        const int r = idx / PIECES, pc = idx - r * PIECES, kb = pc >> 3, a = pc & 7;
        if (i0 + 32 * kb < K4) {
          const int e = 32 * kb + (a >> 2) + 8 * (a & 3);
          const float* tr = tt + r * RLD + e;
          *reinterpret_cast<float4*>(drow + (int64_t)r * K4 + i0 + 4 * pc) =
              make_float4(tr[0], tr[2], tr[4], tr[6]);
        }
      }
    }
    if (++kc == kW) {
      kc = 0;
      ++kr;
    }
  }
  (void)rows;
}

// Rows of up to 1024 elements (K4 = 32 NB, NB <= 4; launched for the 13^2
// planes' NB = 1): eight rows a block, each row's 64 NB 16-byte pieces written
// straight to their rearranged place — piece a of kperm block kb of residue r
// holds elements i = 32 kb + (a >> 2) + 8 (a & 3) + 2 e, e = 0..3; a thread
// 2 NB pieces, each four loads and one 16-byte store (a block writes its rows
// whole, so the lines complete in L2 without the LDS transpose)
struct Piece {
  int j, r, i0, off;  // row in the block, residue, first element, float offset in the row
};
template <int NB>
__device__ __forceinline__ Piece piece_of(int idx) {
  constexpr int PR = 64 * NB;  // pieces per row
  const int j = idx / PR, rem = idx - j * PR, r = rem / (8 * NB), pc = rem - r * (8 * NB);
  const int kb = pc >> 3, a = pc & 7;
  return Piece{j, r, 32 * kb + (a >> 2) + 8 * (a & 3), r * 32 * NB + 32 * kb + 4 * a};
}

template <int NB>
__global__ __launch_bounds__(256) void res_permute_short_kernel(
    const float* __restrict__ src, int64_t srcImg, float* __restrict__ dst, int64_t dstImg,
    int rows, int K, int K4, int row0, int total) {
#pragma unroll
  for (int u = 0; u < 2 * NB; ++u) {
    const Piece q = piece_of<NB>((int)threadIdx.x + 256 * u);
    const int ra = row0 + 8 * (int)blockIdx.y + q.j;
    if (ra >= total) continue;
    const int b = ra / rows, row = ra - b * rows;
    const float* s = src + b * srcImg + (int64_t)row * K;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int pp = q.r + 8 * (q.i0 + 2 * e);
      v[e] = pp < K ? s[pp] : 0.0f;
    }
    *reinterpret_cast<float4*>(dst + b * dstImg + (int64_t)row * 8 * K4 + q.off) =
        make_float4(v[0], v[1], v[2], v[3]);
  }
}

template <int NB>
__global__ __launch_bounds__(256) void im2col_res_short_kernel(
    const float* __restrict__ x, int64_t xImg, float* __restrict__ dst, int64_t dstImg, int H,
    int W, int kH, int kW, int sY, int sX, int pH, int pW, int dY, int dX, int oW, int HWo,
    int rows, int K4, int row0, int total) {
  const int taps = kH * kW;
#pragma unroll
  for (int u = 0; u < 2 * NB; ++u) {
    const Piece q = piece_of<NB>((int)threadIdx.x + 256 * u);
    const int ra = row0 + 8 * (int)blockIdx.y + q.j;
    if (ra >= total) continue;
    const int b = ra / rows, n = ra - b * rows;
    const int c = n / taps, t = n - c * taps, kr = t / kW, kc = t - kr * kW;
    const float* xc = x + b * xImg + (int64_t)c * H * W;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int pp = q.r + 8 * (q.i0 + 2 * e);
      const int oy = pp / oW, ox = pp - oy * oW;
      const int iy = oy * sY - pH + kr * dY, ix = ox * sX - pW + kc * dX;
      v[e] = (pp < HWo && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
                 ? xc[iy * W + ix]
                 : 0.0f;
    }
    *reinterpret_cast<float4*>(dst + b * dstImg + (int64_t)n * 8 * K4 + q.off) =
        make_float4(v[0], v[1], v[2], v[3]);
  }
}

template <int BM, int BN, int R, bool IF = false>
hipError_t launch_res(const ResArgs& a, int64_t batch, hipStream_t s) {
  if (a.M % BM) return hipErrorInvalidValue;
  const int64_t tiles = (int64_t)(a.M / BM) * ((a.N + BN - 1) / BN);
  hipLaunchKernelGGL((dw_res_kernel<BM, BN, R, IF>),
                     dim3((unsigned)tiles, 8 / R, IF ? 1u : (unsigned)batch), dim3(256), 0, s, a);
  return hipGetLastError();
}

struct ResForm {
  int bm, bn, r;
  hipError_t (*fn)(const ResArgs&, int64_t, hipStream_t);
  const char* name;
  bool fold_images;  // (IF) weight_updates accumulated in the block
};
#define TNS_RES(BMv, BNv, Rv) \
  {BMv, BNv, Rv, launch_res<BMv, BNv, Rv>, "dw_res<" #BMv "x" #BNv ",r" #Rv ">", false}
#define TNS_RESI(BMv, BNv) \
  {BMv, BNv, 8, launch_res<BMv, BNv, 8, true>, "dw_res<" #BMv "x" #BNv ",r8,images>", true}
// (R = 8 on the 128-wide tiles: four live accumulator sets spill)
const ResForm kResForms[] = {
    TNS_RES(128, 128, 2), TNS_RES(128, 128, 4), TNS_RES(64, 128, 2),
    TNS_RES(64, 128, 4),  TNS_RES(64, 64, 4),   TNS_RES(64, 64, 8),
    // one residue a block (8 group planes): the long-k layers with few outputs
    TNS_RES(64, 64, 1),   TNS_RES(128, 64, 1),  TNS_RES(128, 128, 1),
    // every image in one block (no partial planes)
    TNS_RESI(64, 64),
};
#undef TNS_RES
#undef TNS_RESI
constexpr int kNumResForms = sizeof(kResForms) / sizeof(kResForms[0]);

int blocks_for(int64_t n) { return (int)std::min<int64_t>((n + 255) / 256, 16384); }

}  // namespace

int dw_res_count() { return kNumResForms; }
const char* dw_res_name(int v) { return v >= 0 && v < kNumResForms ? kResForms[v].name : ""; }

int64_t dw_res_k4(int64_t K) { return ((K + 7) / 8 + 31) / 32 * 32; }

// Measured per YOLOv3 layer (scripts/dw_res_prof.py under a kernel trace,
// whole backward calls without state.delta at batch 8; profiles/
// r04_dw_res_forms4*), against the kernels before (dw_tile at 52^2, the
// residue-register kernel at 26^2 / 13^2, im2col + the sdot kernel on the
// long-k planes):
//   k <= 1024 (26^2, 13^2 planes): all 8 residues in one 64 x 64 block, one
//     partial plane (26^2 0.221 -> 0.191 ms, 13^2 0.309 -> 0.275; the
//     image-folded form, no partial planes, runs the 13^2 layers in 0.289
//     against 0.269, profiles/r04_dw_res_forms6); the
//     one-residue forms make 8 planes of these large outputs to add, and the
//     26^2 product runs 0.26-0.27 with them;
//   k <= 4096 (52^2): one residue a block, 128 x 64 (0.213 -> 0.194);
//   longer k (104^2, 208^2 planes): one residue a block, 64 x 64 (104^2
//   0.379 -> 0.267, 208^2 0.560 -> 0.434).
// -1: none applies (filters not a multiple of 64, k < 64).
int dw_res_pick(int64_t M, int64_t N, int64_t K, int64_t batch) {
  (void)N;
  if (M % 64 || batch < 1 || K < 64) return -1;
  if (K <= 1024) return 5;
  if (K <= 4096) return M % 128 == 0 ? 7 : 6;
  return 6;
}

int64_t dw_res_b_rows(int v, int64_t N) {
  if (v < 0 || v >= kNumResForms) return N;
  const int64_t bn = kResForms[v].bn;
  return (N + bn - 1) / bn * bn;
}

int64_t dw_res_groups(int v) {
  return v >= 0 && v < kNumResForms && !kResForms[v].fold_images ? 8 / kResForms[v].r : 0;
}

hipError_t launch_dw_res(int v, const DwResArgs& d, hipStream_t s) {
  if (v < 0 || v >= kNumResForms) return hipErrorInvalidValue;
  const ResForm& f = kResForms[v];
  if (d.M % f.bm || d.N <= 0 || d.K <= 0 || d.batch <= 0 || d.batch > 65535)
    return hipErrorInvalidValue;
  const int64_t K4 = dw_res_k4(d.K), rowlen = 8 * K4;
  const int64_t npad = dw_res_b_rows(v, d.N);  // col' rows per image (tile multiple)
  if (rowlen * 4 * 8 > 0x7fffffffLL || d.M * d.N > 0x7fffffffLL || d.batch * d.N > 0x7fffffffLL ||
      d.batch * d.M > 0x7fffffffLL)
    return hipErrorInvalidValue;
  // delta' and col' (or the input planes' rearrangement): one block row per
  // operand row, 65535 rows a launch
  // chunk of a block: 2048, or the row rounded up to 256 when shorter (a
  // block's loads are its latency: small chunks measured slower even where
  // the 2048-chunk leaves a partial last block; 52^2 rows: 83 us with 256,
  // 46 us with 2048)
  const int chs = rowlen >= RCH ? RCH : rowlen > 512 ? 1024 : rowlen > 256 ? 512 : 256;
  const unsigned gx = (unsigned)((rowlen + chs - 1) / chs);
  auto rows_launch = [&](int64_t nrows, auto&& launch) -> hipError_t {
    for (int64_t r0 = 0; r0 < nrows; r0 += 65535) {
      launch(dim3(gx, (unsigned)std::min<int64_t>(nrows - r0, 65535)), (int)r0);
      if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  auto by_chunk = [&](auto&& f) {
    switch (chs) {
      case 256: f(std::integral_constant<int, 256>{}); break;
      case 512: f(std::integral_constant<int, 512>{}); break;
      case 1024: f(std::integral_constant<int, 1024>{}); break;
      default: f(std::integral_constant<int, 2048>{}); break;
    }
  };
  // the im2col rearrangement from LDS-staged input rows (im2col_res_lds_kernel):
  // the chunk's input rows must fit the stage budget
  const ConvGeom& gg = d.g;
  const int chl = rowlen <= 256 ? 256 : chs;
  const int64_t lds_rows = ((chl - 1) / gg.ow + 1) * gg.sY + (gg.kH - 1) * gg.dY + 1;
  const int64_t lds_bytes = std::min<int64_t>(lds_rows, gg.H) * gg.W * 4;
#ifdef TNS_RES_LDS_OFF  // (A/B side builds: the per-row kernels)
  const bool lds_im2col = false;
#else
  const bool lds_im2col = !d.direct && lds_bytes <= kResStageBytes;
#endif
  auto lds_launch = [&]() -> hipError_t {
    const int64_t planes = d.batch * gg.C;
    const unsigned gxl = (unsigned)((rowlen + chl - 1) / chl);
    for (int64_t p0 = 0; p0 < planes; p0 += 65535) {
      const dim3 gr(gxl, (unsigned)std::min<int64_t>(planes - p0, 65535));
      auto go = [&](auto cc) {
        constexpr int CHv = decltype(cc)::value;
        hipLaunchKernelGGL((im2col_res_lds_kernel<CHv>), gr, dim3(256), (size_t)lds_bytes, s, d.x,
                           d.xStride, d.dB, npad * rowlen, (int)gg.C, (int)gg.H, (int)gg.W,
                           (int)gg.kH, (int)gg.kW, (int)gg.sY, (int)gg.sX, (int)gg.padH,
                           (int)gg.padW, (int)gg.dY, (int)gg.dX, (int)gg.ow, (int)d.K, (int)d.N,
                           (int)K4, (int)p0);
      };
      switch (chl) {
        case 256: go(std::integral_constant<int, 256>{}); break;
        case 512: go(std::integral_constant<int, 512>{}); break;
        case 1024: go(std::integral_constant<int, 1024>{}); break;
        default: go(std::integral_constant<int, 2048>{}); break;
      }
      if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  auto delta_rows = [&]() {
    return rows_launch(d.batch * d.M, [&](dim3 gr, int r0) {
      by_chunk([&](auto c) {
        hipLaunchKernelGGL((res_permute_kernel<decltype(c)::value>), gr, dim3(256), 0, s, d.delta,
                           d.M * d.K, d.dA, d.M * rowlen, (int)d.M, (int)d.K, (int)K4, r0);
      });
    });
  };
  // (direct short rows only for K4 = 32: at K4 = 96, the 26^2 planes, the
  // LDS row chunks measured faster, 25.6 vs 28.0 us, profiles/r04_dw_res_forms12)
  if (rowlen <= 256) {
    const int nb = (int)(K4 / 32);
    auto by_nb = [&](auto&& f) {
      switch (nb) {
        case 1: f(std::integral_constant<int, 1>{}); break;
        case 2: f(std::integral_constant<int, 2>{}); break;
        case 3: f(std::integral_constant<int, 3>{}); break;
        default: f(std::integral_constant<int, 4>{}); break;
      }
    };
    auto short_launch = [&](int64_t nrows, auto&& launch) -> hipError_t {
      const int64_t groups = (nrows + 7) / 8;
      for (int64_t g0 = 0; g0 < groups; g0 += 65535) {
        launch(dim3(1, (unsigned)std::min<int64_t>(groups - g0, 65535)), (int)(8 * g0), (int)nrows);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
      }
      return hipSuccess;
    };
    if (hipError_t e = short_launch(d.batch * d.M, [&](dim3 gr, int r0, int tot) {
          by_nb([&](auto c) {
            hipLaunchKernelGGL((res_permute_short_kernel<decltype(c)::value>), gr, dim3(256), 0, s,
                               d.delta, d.M * d.K, d.dA, d.M * rowlen, (int)d.M, (int)d.K, (int)K4,
                               r0, tot);
          });
        });
        e != hipSuccess)
      return e;
    if (lds_im2col) {
      if (hipError_t e = lds_launch(); e != hipSuccess) return e;
    } else if (hipError_t e = short_launch(d.batch * d.N, [&](dim3 gr, int r0, int tot) {
          by_nb([&](auto c) {
            constexpr int NB = decltype(c)::value;
            if (d.direct) {
              hipLaunchKernelGGL((res_permute_short_kernel<NB>), gr, dim3(256), 0, s, d.x,
                                 d.xStride, d.dB, npad * rowlen, (int)d.N, (int)d.K, (int)K4, r0,
                                 tot);
            } else {
              const ConvGeom& g = d.g;
              hipLaunchKernelGGL((im2col_res_short_kernel<NB>), gr, dim3(256), 0, s, d.x,
                                 d.xStride, d.dB, npad * rowlen, (int)g.H, (int)g.W, (int)g.kH,
                                 (int)g.kW, (int)g.sY, (int)g.sX, (int)g.padH, (int)g.padW,
                                 (int)g.dY, (int)g.dX, (int)g.ow, (int)d.K, (int)d.N, (int)K4,
                                 r0, tot);
            }
          });
        });
        e != hipSuccess)
      return e;
  } else {
    if (hipError_t e = delta_rows(); e != hipSuccess) return e;
    if (lds_im2col) {
      if (hipError_t e = lds_launch(); e != hipSuccess) return e;
    } else if (hipError_t e = rows_launch(d.batch * d.N, [&](dim3 gr, int r0) {
          by_chunk([&](auto c) {
            constexpr int C = decltype(c)::value;
            if (d.direct) {
              hipLaunchKernelGGL((res_permute_kernel<C>), gr, dim3(256), 0, s, d.x, d.xStride, d.dB,
                                 npad * rowlen, (int)d.N, (int)d.K, (int)K4, r0);
            } else {
              const ConvGeom& g = d.g;
              hipLaunchKernelGGL((im2col_res_kernel<C>), gr, dim3(256), 0, s, d.x, d.xStride, d.dB,
                                 npad * rowlen, (int)g.H, (int)g.W, (int)g.kH, (int)g.kW, (int)g.sY,
                                 (int)g.sX, (int)g.padH, (int)g.padW, (int)g.dY, (int)g.dX,
                                 (int)g.ow, (int)d.K, (int)d.N, (int)K4, r0);
            }
          });
        });
        e != hipSuccess)
      return e;
  }
  ResArgs a{};
  a.A = d.dA;
  a.B = d.dB;
  a.P = d.part;
  a.M = (int)d.M;
  a.N = (int)d.N;
  a.K1 = (int)((d.K + 7) / 8);
  a.K4 = (int)K4;
  a.G = 8 / f.r;
  a.strideA = d.M * rowlen;
  a.strideB = npad * rowlen;
  a.strideP = (int64_t)a.G * d.M * d.N;
  a.W = d.weight_updates;
  a.alpha = d.alpha;
  a.batch = (int)d.batch;
  if (hipError_t e = f.fn(a, d.batch, s); e != hipSuccess) return e;
  if (f.fold_images) return hipSuccess;  // (weight_updates written by the product)
  const int64_t mn = d.M * d.N;
  // (TNS_ACC4=0: the scalar form, for A/B runs)
  static const bool acc4 = !(getenv("TNS_ACC4") && getenv("TNS_ACC4")[0] == '0');
  if (acc4 && mn % 4 == 0 && !(reinterpret_cast<uintptr_t>(d.weight_updates) & 15) &&
      !(reinterpret_cast<uintptr_t>(d.part) & 15)) {
    const int64_t mn4 = mn / 4;
    auto go = [&](auto gc) {
      constexpr int Gv = decltype(gc)::value;
      hipLaunchKernelGGL((dw_res_accumulate4_kernel<Gv>), dim3(blocks_for(mn4)), dim3(256), 0, s,
                         reinterpret_cast<float4*>(d.weight_updates),
                         reinterpret_cast<const float4*>(d.part), mn4, a.strideP / 4,
                         (int)d.batch, d.alpha);
    };
    switch (a.G) {
      case 1: go(std::integral_constant<int, 1>{}); break;
      case 2: go(std::integral_constant<int, 2>{}); break;
      case 4: go(std::integral_constant<int, 4>{}); break;
      default: go(std::integral_constant<int, 8>{}); break;
    }
    return hipGetLastError();
  }
  hipLaunchKernelGGL(dw_res_accumulate_kernel, dim3(blocks_for(mn)), dim3(256), 0, s,
                     d.weight_updates, d.part, mn, a.G, a.strideP, (int)d.batch, d.alpha);
  return hipGetLastError();
}

}  // namespace tns
