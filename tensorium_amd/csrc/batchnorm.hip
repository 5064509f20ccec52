// batchnorm.hip — batch-norm, softmax / cross-entropy and reductions for the
// connected-layer train step (BASELINE config 5), gfx950.
//
// Device twins of TNNCuda.meansAndVars / normalize / forwardScale(Add) /
// meansAndVarsDelta / normalizeDelta / addDots / softmaxBatch /
// crossEntropySoftmax (nncuda.pas:1056-1510), with the CPU semantics of
// ntensors.pas:7687-7830, 8693-8718, 8821-8951, 9102-9177 and
// nsoftmaxlayer.pas:83-137 (see oracle/tns_oracle_train.c).
//
// Reductions over one channel follow the reference's order exactly: ONE
// thread per channel when it has <= kSeqMax elements (the FC layers:
// blockSize 1, groups = batch); larger channels (conv BN) give each block's
// 8 AVX2 lanes to 8 GPU lanes and add the block results in order.  Transcendentals (exp, ln, pow) are evaluated in
// double and rounded once, as the oracle does.
#include <cstdlib>

#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
namespace {

constexpr int TPB = 256;
constexpr int64_t kSeqMax = 8192;
__device__ constexpr float SEPS = 0.000001f;  // sEPSILON, ntensors.pas:95

inline unsigned nblk(int64_t n) {
  int64_t g = (n + TPB - 1) / TPB;
  return (unsigned)(g < 1 ? 1 : (g > 65535 * 4 ? 65535 * 4 : g));
}

// ---- MeansAndVars --------------------------------------------------------
// MeansAndVars (ntensors.pas:9102-9177) per channel: m := m + sumv(block)
// over the groups in order, m / S; v := v + rssv(block, m), v / S2.  With
// stride-1 blocks on an AVX2 host sumv is vssum_avx2 (3592-3620) and rssv is
// srss (1493-1523): 8 lanes, then (for srss, when a tail exists) lanes l and
// l+4 folded and the tail added to lane 0, then ((x0+x1)+(x2+x3)).  srss
// without a tail drops lanes 4..7 in the reference; reproduced only under
// TNS_OPT_SRSS_QUIRK (quirk != 0), otherwise folded as with a tail.
__device__ __forceinline__ float vssum8(const float* a, int64_t n);  // below

__device__ __forceinline__ float srss_fold(const float (&acc)[8], bool notail_quirk) {
  float x0, x1, x2, x3;
  if (notail_quirk) {
    x0 = acc[0]; x1 = acc[1]; x2 = acc[2]; x3 = acc[3];
  } else {
    x0 = acc[0] + acc[4]; x1 = acc[1] + acc[5]; x2 = acc[2] + acc[6]; x3 = acc[3] + acc[7];
  }
  return (x0 + x1) + (x2 + x3);
}

__device__ __forceinline__ float srss8(const float* a, int64_t n, float mean, int quirk) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t blocks = n >> 3;
  for (int64_t t = 0; t < blocks; ++t)
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      const float d = mean - a[8 * t + l];
      acc[l] = acc[l] + d * d;
    }
  if ((n & 7) == 0) return srss_fold(acc, quirk != 0);
  float x0 = acc[0] + acc[4];
  for (int64_t i = blocks * 8; i < n; ++i) {
    const float d = mean - a[i];
    x0 = x0 + d * d;
  }
  return (x0 + (acc[1] + acc[5])) + ((acc[2] + acc[6]) + (acc[3] + acc[7]));
}

// one thread per channel (FC layers: blockSize 1, groups = batch).  what:
// MV_MEAN and / or MV_VAR; the variance alone (TNNCuda.variances) reads the
// caller's means
enum { MV_MEAN = 1, MV_VAR = 2 };
__global__ void means_vars_seq(const float* __restrict__ x, int64_t groups, int64_t N, int64_t bs,
                               float* __restrict__ means, float* __restrict__ vars, int quirk,
                               int what) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= N) return;
  const float S = (float)(groups * bs), S2 = (float)(groups * bs - 1);
  float m;
  if (what & MV_MEAN) {
    m = 0.0f;
    for (int64_t b = 0; b < groups; ++b) m = m + vssum8(x + (i + b * N) * bs, bs);
    m = m / S;
    means[i] = m;
  } else {
    m = means[i];
  }
  if (!(what & MV_VAR)) return;
  float v = 0.0f;
  for (int64_t b = 0; b < groups; ++b) v = v + srss8(x + (i + b * N) * bs, bs, m, quirk);
  vars[i] = v / S2;
}

// ---- normalize / scale / bias ----------------------------------------------
__global__ void normalize_k(float* __restrict__ x, int64_t total, int64_t N, int64_t bs,
                            const float* __restrict__ means, int64_t mstride,
                            const float* __restrict__ vars, int64_t vstride) {
  for (int64_t e = (int64_t)blockIdx.x * TPB + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * TPB) {
    const int64_t i = (e / bs) % N;
    const float m = means[i * mstride], v = vars[i * vstride];
    float sd;
    if (bs == 1) {
      sd = sqrtf(v > SEPS ? v : SEPS);  // _snormvv
    } else {
      sd = sqrtf(v);                     // _snormblkvv -> snormvss
      sd = sd > SEPS ? sd : SEPS;
    }
    x[e] = (x[e] - m) / sd;
  }
}

__global__ void scale_add_k(float* __restrict__ x, int64_t total, int64_t N, int64_t bs,
                            const float* __restrict__ scales, const float* __restrict__ biases,
                            int64_t incb) {
  for (int64_t e = (int64_t)blockIdx.x * TPB + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * TPB) {
    const int64_t i = (e / bs) % N;
    float v = x[e] * scales[i * incb];            // forwardScale (vsMulB)
    if (biases) v = v + biases[i * incb];         // forwardBias  (vsAddB)
    x[e] = v;
  }
}

// ---- addDots / addSums -------------------------------------------------------
__global__ void add_dots_seq(float* __restrict__ dst, const float* __restrict__ a,
                             const float* __restrict__ b, int64_t groups, int64_t N, int64_t bs) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= N) return;
  if (bs == 1) {  // strided cblas_sdot: scalar mul then add
    float r = 0.0f;
    for (int64_t g = 0; g < groups; ++g) r = r + a[i + g * N] * b[i + g * N];
    dst[i] = dst[i] + r;
  } else {        // per block sdot_avx2 (8 FMA lanes), blocks summed
    float sum = 0.0f;
    for (int64_t g = 0; g < groups; ++g) {
      const float* pa = a + (i + g * N) * bs;
      const float* pb = b + (i + g * N) * bs;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      const int64_t blocks = bs >> 3;
      for (int64_t t = 0; t < blocks; ++t)
#pragma unroll
        for (int l = 0; l < 8; ++l) acc[l] = fmaf(pa[8 * t + l], pb[8 * t + l], acc[l]);
      const int64_t rem = bs & 7;
      if (rem) {
#pragma unroll
        for (int l = 0; l < 8; ++l) {
          const float xa = l < rem ? pa[8 * blocks + l] : 0.0f;
          const float xb = l < rem ? pb[8 * blocks + l] : 0.0f;
          acc[l] = fmaf(xa, xb, acc[l]);
        }
      }
      const float s0 = acc[0] + acc[4], s1 = acc[1] + acc[5], s2 = acc[2] + acc[6],
                  s3 = acc[3] + acc[7];
      sum = sum + ((s0 + s1) + (s2 + s3));
    }
    dst[i] = dst[i] + sum;
  }
}

__global__ void add_sums_seq(float* __restrict__ dst, const float* __restrict__ src,
                             int64_t groups, int64_t N) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= N) return;
  float r = 0.0f;  // strided vsSumI: scalar running sum
  for (int64_t g = 0; g < groups; ++g) r = r + src[i + g * N];
  dst[i] = dst[i] + r;
}

// ---- MeanAndVarianceDelta / NormalizeDelta ---------------------------------
__device__ __forceinline__ float vssum8(const float* a, int64_t n) {  // vssum_avx2 order
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t blocks = n >> 3;
  int64_t t = 0;
  for (; t + 4 <= blocks; t += 4) {  // 32 loads ahead of the lane adds
    float w[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) w[u] = a[8 * t + u];
#pragma unroll
    for (int u = 0; u < 32; ++u) acc[u & 7] = acc[u & 7] + w[u];
  }
  for (; t < blocks; ++t)
#pragma unroll
    for (int l = 0; l < 8; ++l) acc[l] = acc[l] + a[8 * t + l];
  const float s0 = acc[0] + acc[4], s1 = acc[1] + acc[5], s2 = acc[2] + acc[6],
              s3 = acc[3] + acc[7];
  float r = (s0 + s1) + (s2 + s3);
  for (int64_t i = blocks * 8; i < n; ++i) r = r + a[i];
  return r;
}

// sVarinceDelta_avx (ntensors.pas:8721-8757): 8 lanes of (x - mean) * delta
// (sub, mul, add each rounded) over the full 8-blocks; with a tail, lanes
// l+4 folded into l and the tail added to lane 0; then (x0+x1)+(x2+x3).  A
// tail-less block skips the fold in the reference (lanes 4..7 dropped):
// reproduced when quirk != 0, folded otherwise.
__device__ __forceinline__ float var_delta8(const float* dd, const float* xx, int64_t n, float mu,
                                            int quirk) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t blocks = n >> 3;
  for (int64_t t = 0; t < blocks; ++t)
#pragma unroll
    for (int l = 0; l < 8; ++l) acc[l] = acc[l] + (xx[8 * t + l] - mu) * dd[8 * t + l];
  float x0, x1, x2, x3;
  if ((n & 7) == 0 && quirk) {
    x0 = acc[0]; x1 = acc[1]; x2 = acc[2]; x3 = acc[3];
  } else {
    x0 = acc[0] + acc[4]; x1 = acc[1] + acc[5]; x2 = acc[2] + acc[6]; x3 = acc[3] + acc[7];
    for (int64_t k = blocks * 8; k < n; ++k) x0 = x0 + (xx[k] - mu) * dd[k];
  }
  return (x0 + x1) + (x2 + x3);
}

__global__ void mean_var_delta_seq(const float* __restrict__ delta, const float* __restrict__ x,
                                   const float* __restrict__ mean, const float* __restrict__ var,
                                   int64_t groups, int64_t N, int64_t bs,
                                   float* __restrict__ mean_delta, float* __restrict__ var_delta,
                                   int quirk) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= N) return;
  float m = 0.0f, v = 0.0f;
  const float mu = mean[i];
  for (int64_t j = 0; j < groups; ++j) {
    const float* dd = delta + (i + j * N) * bs;
    const float* xx = x + (i + j * N) * bs;
    m = m + vssum8(dd, bs);
    v = v + var_delta8(dd, xx, bs, mu, quirk);
  }
  const float ve = var[i] > SEPS ? var[i] : SEPS;
  const float inv = -1.0f / sqrtf(ve);
  mean_delta[i] = m * inv;
  var_delta[i] = (float)((double)v * -0.5 * pow((double)ve, -1.5));
}

__global__ void normalize_delta_k(const float* __restrict__ x, const float* __restrict__ mean,
                                  const float* __restrict__ var,
                                  const float* __restrict__ mean_delta,
                                  const float* __restrict__ var_delta, float* __restrict__ delta,
                                  int64_t total, int64_t N, int64_t bs, float B,
                                  const float* __restrict__ scales,
                                  const float* __restrict__ out, int act) {
  for (int64_t e = (int64_t)blockIdx.x * TPB + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * TPB) {
    const int64_t i = (e / bs) % N;
    const float md = mean_delta[i] / B;
    const float vd = 2.0f * var_delta[i] / B;
    const float ve = var[i] > SEPS ? var[i] : SEPS;
    const float sd = sqrtf(ve);
    float d = delta[e];
    if (out) d = d * grad_apply(out[e], act);  // (Derivative folded in)
    const float a = (scales ? d * scales[i] : d) / sd;
    const float t = (x[e] - mean[i]) * vd + md;  // sNormalizeDelta_avx order
    delta[e] = a + t;
  }
}

// ---- softmax / cross-entropy ------------------------------------------------
// one thread per (batch, group): TSoftmaxLayer.softmaxBatch / softmax
__global__ void softmax_batch_k(int64_t n, const float* __restrict__ in, int64_t batch,
                                int64_t batch_size, int64_t groups, int64_t group_size,
                                int64_t stride, float temp, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (t >= batch * groups || n == 0) return;
  const int64_t b = t / groups, g = t - b * groups;
  const float* ip = in + b * batch_size + g * group_size;
  float* op = out + b * batch_size + g * group_size;
  float largest = ip[0];
  for (int64_t i = 1; i < n; ++i)
    if (ip[i * stride] > largest) largest = ip[i * stride];
  float sum = 0.0f;
  for (int64_t i = 0; i < n; ++i) {
    const float e = (float)exp((double)((ip[i * stride] - largest) / temp));
    sum = sum + e;
    op[i * stride] = e;
  }
  for (int64_t i = 0; i < n; ++i) op[i * stride] = op[i * stride] / sum;
}

__global__ void xent_softmax_k(int64_t n, const float* __restrict__ pred,
                               const float* __restrict__ truth, float* __restrict__ delta,
                               float* __restrict__ error) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * TPB) {
    const float t = truth[i], p = pred[i];
    error[i] = t != 0.0f ? (float)(-log((double)(p > SEPS ? p : SEPS))) : 0.0f;
    delta[i] = t - p;
  }
}

// vssum_avx2-ordered sum of a vector into *out (one thread; cost vector is
// batch*classes elements)
__global__ void vssum_k(int64_t n, const float* __restrict__ a, float* __restrict__ out) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *out = vssum8(a, n);
}


// ---- conv-sized blocks: lane chains over one (group, channel) block ---------
// The reference reduces every contiguous block with an AVX2 routine whose 8
// lanes are strictly sequential chains (vssum_avx2, srss, sVarinceDelta_avx,
// sdot_avx2), then adds the block results over the groups in order.  Only
// groups x channels x 8 chains exist (2048 for YOLOv3's first layer at batch
// 8, each 21632 long), so the chains cannot be the unit of memory traffic:
// one workgroup per block streams it through LDS in coalesced tiles
// (double-buffered, the next tile's loads in flight while the chains run),
// the elementwise part (mean - x)^2 or (x - mean) * delta is formed by all
// threads while staging (one rounding each, as vsubps / vmulps), and the
// first 8 (or 16) lanes of wave 0 run the lane chains out of LDS.  The block
// results go to part[block] (block = g*N + i, memory order) and a per-channel
// pass adds them in group order.
// CH_DSUM: CH_SUM over delta * f'(output) — the conv backward's Derivative
// fused into its bias sums: a = delta (each derived term also written back
// through wa), b = output, act = the activation; the same product as
// derive4_kernel, the same chains as CH_SUM
// CH_DDOT: CH_DOT (addDots) over delta * f'(output) and x_norm — the BN
// conv backward's Derivative fused into its addDots: a = delta (each derived
// term written back through wa), b = x_norm, c3 = output.
// sc (CH_VDELTA): the per-channel scales of forwardScale applied to each delta
// term as it is staged (one rounding, as the separate pass would store it) —
// the BN conv backward's forwardScale folded into MeansAndVarsDelta (and
// normalizeDelta), the scaled delta never written
// CH_BNB: the BN conv backward's three reductions in one pass over delta,
// output, x_norm and x (a, c3, b, xx): d = delta * f'(output) (Derivative),
// ds = d * scale (forwardScale); lanes 0-7 the addDots chains of d . x_norm
// (sdot), lanes 8-15 the MeansAndVarsDelta mean chains of ds (vssum), lanes
// 16-23 its variance chains of (x - mean) * ds (sVarinceDelta); nothing is
// written back (normalizeDelta recomputes d and ds) — one pass and one
// finish instead of three passes and two finishes.  All three chain groups
// run fma(term, w, acc) so the wave executes one instruction stream: w =
// x_norm for the dot, 1.0 (an LDS row of ones) for the sums — fma(t, 1, acc)
// rounds t + acc exactly as the add does
enum ChainMode {
  CH_SUM = 0, CH_SRSS = 1, CH_VDELTA = 2, CH_DOT = 3, CH_DSUM = 4, CH_DDOT = 5, CH_BNB = 6
};

template <int MODE, int NT, int E>
__global__ __launch_bounds__(NT) void block_chains(const float* __restrict__ a,
                                                   const float* __restrict__ b,
                                                   const float* __restrict__ mu_arr,
                                                   int64_t nblocks, int64_t N, int64_t bs,
                                                   int quirk, float* __restrict__ part0,
                                                   float* __restrict__ part1, int act,
                                                   float* wa, const float* __restrict__ c3,
                                                   const float* __restrict__ sc_arr,
                                                   const float* __restrict__ xx,
                                                   float* __restrict__ part2) {
  // chain waves first at the SIMD issue arbiter: their dependent adds are the
  // critical path, the MFMA waves of a concurrent dW product have slack
  __builtin_amdgcn_s_setprio(3);
  constexpr int TILE = NT * E;
  constexpr bool BNB = MODE == CH_BNB;
  constexpr bool DOTF = MODE == CH_DOT || MODE == CH_DDOT || BNB;  // the fma chains
  constexpr bool TWO = MODE == CH_VDELTA || DOTF;             // two LDS streams
  constexpr bool LB = TWO || MODE == CH_DSUM;                 // b loaded
  constexpr bool LC = MODE == CH_DDOT || BNB;                 // c3 loaded
  // tiles stored lane-major: element e of the tile at (e & 7) * LDT + e / 8,
  // so a chain lane's consecutive terms are contiguous (ds_read_b128 reads
  // four); rows padded by 8 floats (conflict-free staging stores)
  constexpr int LDT = TILE / 8 + 8;
  __shared__ __attribute__((aligned(16))) float U[2][8 * LDT];
  __shared__ __attribute__((aligned(16))) float V[TWO ? 2 : 1][TWO ? 8 * LDT : 1];
  // (BNB) the mean and variance terms, and the row of ones the sum chains
  // multiply by
  __shared__ __attribute__((aligned(16))) float Mt[BNB ? 2 : 1][BNB ? 8 * LDT : 1];
  __shared__ __attribute__((aligned(16))) float Qt[BNB ? 2 : 1][BNB ? 8 * LDT : 1];
  __shared__ __attribute__((aligned(16))) float ONES[BNB ? LDT : 1];
  const int tid = threadIdx.x;
  const int l = tid & 7, grp = tid >> 3;  // chain lane, chain set (wave 0)
  const bool chain = grp == 0 || (MODE == CH_VDELTA && grp == 1) || (BNB && grp <= 2);
  if constexpr (BNB)
    for (int q = tid; q < LDT; q += NT) ONES[q] = 1.0f;  // (published by the first barrier)
  const int64_t nb8 = (bs >> 3) << 3;  // elements in full 8-blocks
  const int ntile = (int)((nb8 + TILE - 1) / TILE);
  const int tail = (int)(bs & 7);
  for (int64_t blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
    const int64_t i = blk % N;
    const float* pa = a + blk * bs;
    const float* pb = LB ? b + blk * bs : nullptr;
    const float* pc = LC ? c3 + blk * bs : nullptr;
    const float* px = BNB ? xx + blk * bs : nullptr;
    float* pw = (MODE == CH_DSUM || MODE == CH_DDOT) ? wa + blk * bs : nullptr;
    const float mu = (MODE == CH_SRSS || MODE == CH_VDELTA || BNB) ? mu_arr[i] : 0.0f;
    const bool scaled = (MODE == CH_VDELTA && sc_arr != nullptr) || BNB;
    const float scl = scaled ? sc_arr[i] : 1.0f;
    float ra[E], rb[LB ? E : 1], rc[LC ? E : 1], rx[BNB ? E : 1];
    auto load = [&](int t) {
      const int64_t base = (int64_t)t * TILE + tid;
#pragma unroll
      for (int u = 0; u < E; ++u) {
        const int64_t k = base + NT * u;
        ra[u] = k < nb8 ? pa[k] : 0.0f;
        if constexpr (LB) rb[u] = k < nb8 ? pb[k] : 0.0f;
        if constexpr (LC) rc[u] = k < nb8 ? pc[k] : 0.0f;
        if constexpr (BNB) rx[u] = k < nb8 ? px[k] : 0.0f;
      }
    };
    auto store = [&](int buf, int t) {
#pragma unroll
      for (int u = 0; u < E; ++u) {
        const int e = ((tid + NT * u) & 7) * LDT + ((tid + NT * u) >> 3);
        if constexpr (MODE == CH_DSUM) {
          const float d = ra[u] * grad_apply(rb[u], act);
          U[buf][e] = d;
          const int64_t k = (int64_t)t * TILE + tid + NT * u;
          if (k < nb8) pw[k] = d;
        } else if constexpr (MODE == CH_DDOT) {
          const float d = ra[u] * grad_apply(rc[u], act);
          U[buf][e] = d;
          V[buf][e] = rb[u];
          const int64_t k = (int64_t)t * TILE + tid + NT * u;
          if (k < nb8) pw[k] = d;
        } else if constexpr (BNB) {
          const float d = ra[u] * grad_apply(rc[u], act);  // Derivative
          const float ds = d * scl;                          // forwardScale
          U[buf][e] = d;
          V[buf][e] = rb[u];
          Mt[buf][e] = ds;
          Qt[buf][e] = (rx[u] - mu) * ds;
        } else if constexpr (MODE == CH_SUM) {
          U[buf][e] = ra[u];
        } else if constexpr (MODE == CH_SRSS) {  // srss: vsubps (mean - a), vmulps
          const float d = mu - ra[u];
          U[buf][e] = d * d;
        } else if constexpr (MODE == CH_VDELTA) {  // a = delta, b = x
          const float d = scaled ? ra[u] * scl : ra[u];
          U[buf][e] = d;
          V[buf][e] = (rb[u] - mu) * d;
        } else {
          U[buf][e] = ra[u];
          V[buf][e] = rb[u];
        }
      }
    };
    float acc = 0.0f;
    if (ntile > 0) {
      load(0);
      store(0, 0);
    }
    __syncthreads();
    for (int t = 0; t < ntile; ++t) {
      if (t + 1 < ntile) load(t + 1);
      if (tid < 64 && chain) {
        const int64_t rem = nb8 - (int64_t)t * TILE;
        const int cnt = (int)((rem < TILE ? rem : TILE) >> 3);
        const float* row =
            ((MODE == CH_VDELTA && grp == 1) ? &V[t & 1][0] : &U[t & 1][0]) + l * LDT;
        const float* rowb = TWO ? &V[t & 1][0] + l * LDT : row;
        if constexpr (BNB) {
          if (grp == 1) row = &Mt[t & 1][0] + l * LDT;
          if (grp == 2) row = &Qt[t & 1][0] + l * LDT;
          if (grp >= 1) rowb = ONES;
        }
        int q = 0;
        for (; q + 16 <= cnt; q += 16) {
          float v[16], w[16];
#pragma unroll
          for (int z = 0; z < 16; z += 4) {
            const float4 x4 = *reinterpret_cast<const float4*>(row + q + z);
            v[z] = x4.x; v[z + 1] = x4.y; v[z + 2] = x4.z; v[z + 3] = x4.w;
            if constexpr (DOTF) {
              const float4 y4 = *reinterpret_cast<const float4*>(rowb + q + z);
              w[z] = y4.x; w[z + 1] = y4.y; w[z + 2] = y4.z; w[z + 3] = y4.w;
            }
          }
#pragma unroll
          for (int z = 0; z < 16; ++z) {
            if constexpr (DOTF) acc = fmaf(v[z], w[z], acc);
            else acc = acc + v[z];
          }
        }
        for (; q < cnt; ++q) {
          if constexpr (DOTF) acc = fmaf(row[q], rowb[q], acc);
          else acc = acc + row[q];
        }
      }
      if (t + 1 < ntile) store((t + 1) & 1, t + 1);
      __syncthreads();
    }
    if (tid < 64) {  // lane-order epilogues (8-lane groups of wave 0)
      // vssum_avx2: fold, hadd, hadd, then the tail in order
      // srss / sVarinceDelta_avx: fold (unless quirk and no tail), tail into
      //   lane 0, hadd, hadd
      // sdot_avx2: masked-FMA tail into lanes 0..tail-1, fold, hadd, hadd
      const bool lanes_form =
          MODE == CH_SRSS || (MODE == CH_VDELTA && grp == 1) || (BNB && grp == 2);
      // (BNB) tail element k's derived, scaled terms
      auto bnb_d = [&](int k) { return pa[nb8 + k] * grad_apply(pc[nb8 + k], act); };
      if constexpr (DOTF) {
        if (tail && grp == 0) {
          float xa = l < tail ? pa[nb8 + l] : 0.0f;
          const float xb = l < tail ? pb[nb8 + l] : 0.0f;
          if constexpr (MODE == CH_DDOT) {
            if (l < tail) {
              xa = xa * grad_apply(pc[nb8 + l], act);
              pw[nb8 + l] = xa;
            }
          }
          if constexpr (BNB)
            if (l < tail) xa = bnb_d(l);
          acc = fmaf(xa, xb, acc);
        }
      }
      const float up = __shfl_down(acc, 4, 8);
      float x0 = (lanes_form && tail == 0 && quirk) ? acc : acc + up;
      if (lanes_form && l == 0)
        for (int k = 0; k < tail; ++k) {
          if (MODE == CH_SRSS) {
            const float d = mu - pa[nb8 + k];
            x0 = x0 + d * d;
          } else if (BNB) {
            x0 = x0 + (px[nb8 + k] - mu) * (bnb_d(k) * scl);
          } else {
            const float d = scaled ? pa[nb8 + k] * scl : pa[nb8 + k];
            x0 = x0 + (pb[nb8 + k] - mu) * d;
          }
        }
      const float h = x0 + __shfl_down(x0, 1, 8);
      float r = h + __shfl_down(h, 2, 8);
      if (l == 0 && chain) {
        if constexpr (MODE == CH_DSUM) {
          for (int k = 0; k < tail; ++k) {
            const float d = pa[nb8 + k] * grad_apply(pb[nb8 + k], act);
            pw[nb8 + k] = d;
            r = r + d;
          }
        } else if constexpr (BNB) {
          if (grp == 1)
            for (int k = 0; k < tail; ++k) r = r + bnb_d(k) * scl;
        } else if (!lanes_form && !DOTF) {
          for (int k = 0; k < tail; ++k) r = r + (scaled ? pa[nb8 + k] * scl : pa[nb8 + k]);
        }
        if (grp == 0) part0[blk] = r;
        else if (grp == 1) part1[blk] = r;
        else if constexpr (BNB) part2[blk] = r;
      }
    }
    __syncthreads();
  }
}

// The same lane chains with the waves specialised (blocks of >= 16384
// elements, the YOLOv3 conv planes at 104^2 and above): wave 0 runs only the
// chains, waves 1..3 only stage.  A chain's 8-16 terms per LDS row are read
// a 16-term group ahead of the adds that consume them (the lock-step kernel
// above waited on each group's reads before its adds: ~12 cycles per
// dependent add), and the staging waves keep one tile of loads in flight in
// registers while the chain wave works, three LDS buffers deep (a tile is
// loaded at the top of tile t, written after the barrier that ends t, read
// in tile t+2).  The loop bodies of the two roles are separate, so no staging
// register is carried around a loop edge (hipcc copies such registers right
// after their loads and waits there).  Same terms, same order: bit-identical.
template <int MODE>
__global__ __launch_bounds__(256) void block_chains_ws(const float* __restrict__ a,
                                                       const float* __restrict__ b,
                                                       const float* __restrict__ mu_arr,
                                                       int64_t nblocks, int64_t N, int64_t bs,
                                                       int quirk, float* __restrict__ part0,
                                                       float* __restrict__ part1, int act,
                                                       float* wa, const float* __restrict__ c3,
                                                       const float* __restrict__ sc_arr,
                                                       const float* __restrict__ xx,
                                                       float* __restrict__ part2) {
  // chain waves first at the SIMD issue arbiter: their dependent adds are the
  // critical path, the MFMA waves of a concurrent dW product have slack
  __builtin_amdgcn_s_setprio(3);
  static_assert(MODE != CH_DDOT && MODE != CH_BNB, "the specialised-wave form stages two load streams");
  (void)c3;
  (void)xx;
  (void)part2;
  constexpr int SNT = 192, E = 32, TILE = SNT * E, NBUF = 3;
  constexpr bool TWO = MODE == CH_VDELTA || MODE == CH_DOT;
  constexpr bool LB = TWO || MODE == CH_DSUM;
  // lane-major rows (a chain's terms contiguous), LDT = 8 mod 32 for
  // conflict-free staging stores, and 72 floats of slack past a row's last
  // term: the chain loop reads up to 47 terms past its last full group
  // without a bound test
  constexpr int LDT = TILE / 8 + 72;
  __shared__ __attribute__((aligned(16))) float U[NBUF][8 * LDT];
  __shared__ __attribute__((aligned(16))) float V[TWO ? NBUF : 1][TWO ? 8 * LDT : 1];
  const int tid = threadIdx.x;
  const bool chainwave = __builtin_amdgcn_readfirstlane(tid >> 6) == 0;
  const int st = tid - 64;  // staging thread index (waves 1..3)
  const int l = tid & 7, grp = tid >> 3;
  const bool chain = grp == 0 || (MODE == CH_VDELTA && grp == 1);
  const int64_t nb8 = (bs >> 3) << 3;
  const int ntile = (int)((nb8 + TILE - 1) / TILE);
  const int tail = (int)(bs & 7);
  for (int64_t blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
    const int64_t i = blk % N;
    const float* pa = a + blk * bs;
    const float* pb = LB ? b + blk * bs : nullptr;
    float* pw = MODE == CH_DSUM ? wa + blk * bs : nullptr;
    const float mu = (MODE == CH_SRSS || MODE == CH_VDELTA) ? mu_arr[i] : 0.0f;
    const bool scaled = MODE == CH_VDELTA && sc_arr != nullptr;
    const float scl = scaled ? sc_arr[i] : 1.0f;
    float acc = 0.0f;
    if (!chainwave) {
      // float4 staging where the block is 16-byte aligned (nb8 % 8 == 0: a
      // float4 is wholly inside or outside the full 8-blocks)
      const bool v4 = ((reinterpret_cast<uintptr_t>(pa) | (LB ? reinterpret_cast<uintptr_t>(pb) : 0)) & 15) == 0;
      float ra[E], rb[LB ? E : 1];
      auto load = [&](int t) {
        const int64_t t0 = (int64_t)t * TILE;
        if (v4) {
#pragma unroll
          for (int u = 0; u < E / 4; ++u) {
            const int64_t k = t0 + 4 * (st + SNT * u);
            const bool in = k < nb8;
            const float4 x = in ? *reinterpret_cast<const float4*>(pa + k) : float4{0, 0, 0, 0};
            ra[4 * u] = x.x; ra[4 * u + 1] = x.y; ra[4 * u + 2] = x.z; ra[4 * u + 3] = x.w;
            if constexpr (LB) {
              const float4 y = in ? *reinterpret_cast<const float4*>(pb + k) : float4{0, 0, 0, 0};
              rb[4 * u] = y.x; rb[4 * u + 1] = y.y; rb[4 * u + 2] = y.z; rb[4 * u + 3] = y.w;
            }
          }
        } else {
#pragma unroll
          for (int u = 0; u < E / 4; ++u)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const int64_t k = t0 + 4 * (st + SNT * u) + c;
              ra[4 * u + c] = k < nb8 ? pa[k] : 0.0f;
              if constexpr (LB) rb[4 * u + c] = k < nb8 ? pb[k] : 0.0f;
            }
        }
      };
      auto store = [&](int buf, int t) {
#pragma unroll
        for (int u = 0; u < E / 4; ++u)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int ee = 4 * (st + SNT * u) + c;
            const int e = (ee & 7) * LDT + (ee >> 3);
            const float va = ra[4 * u + c];
            if constexpr (MODE == CH_DSUM) {
              const float d = va * grad_apply(rb[4 * u + c], act);
              U[buf][e] = d;
              const int64_t k = (int64_t)t * TILE + ee;
              if (k < nb8) pw[k] = d;
            } else if constexpr (MODE == CH_SUM) {
              U[buf][e] = va;
            } else if constexpr (MODE == CH_SRSS) {  // srss: vsubps (mean - a), vmulps
              const float d = mu - va;
              U[buf][e] = d * d;
            } else if constexpr (MODE == CH_VDELTA) {  // a = delta, b = x
              const float d = scaled ? va * scl : va;
              U[buf][e] = d;
              V[buf][e] = (rb[4 * u + c] - mu) * d;
            } else {
              U[buf][e] = va;
              V[buf][e] = rb[4 * u + c];
            }
          }
      };
      for (int t = 0; t < 2 && t < ntile; ++t) {
        load(t);
        store(t, t);
      }
      __syncthreads();
      for (int t = 0; t < ntile; ++t) {
        const bool more = t + 2 < ntile;
        if (more) load(t + 2);
        __syncthreads();
        if (more) store((t + 2) % NBUF, t + 2);
      }
    } else {
      __syncthreads();
      for (int t = 0; t < ntile; ++t) {
        if (chain) {
          const int64_t rem = nb8 - (int64_t)t * TILE;
          const int cnt = (int)((rem < TILE ? rem : TILE) >> 3);
          const int buf = t % NBUF;
          const float* row =
              ((MODE == CH_VDELTA && grp == 1) ? &V[buf][0] : &U[buf][0]) + l * LDT;
          const float* rowb = TWO ? &V[buf][0] + l * LDT : row;
          // groups of 16 terms read by ds_read_b128 issued as inline asm
          // with explicit counted waits: hipcc's own waits at the loop
          // header assumed only the newest reads pending and drained the
          // whole ring there (lgkmcnt 3..0 before the first group's adds),
          // exposing the LDS latency once per loop trip.  One stream: a
          // ring of three register sets, a group's reads issued right after
          // the group two ahead of it is consumed (lgkmcnt(8) = the two
          // newer sets in flight); two streams (CH_DOT): two sets of 8 reads
          // (lgkmcnt(8) = the newer set).  The waits take the sets as
          // operands, so no add moves above them and no register of a set
          // in flight is reused.  Rows have 72 floats of slack: the ring may
          // read up to 47 terms past cnt.
          typedef float f4 __attribute__((ext_vector_type(4)));
          const unsigned ra_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const float*)row;
          const unsigned rb_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const float*)rowb;
          auto rd = [&](int q, f4 (&v)[4], f4 (&w)[4]) {
            const unsigned a = ra_lds + 4u * (unsigned)q;
            asm volatile("ds_read_b128 %0, %1" : "=v"(v[0]) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(v[1]) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:32" : "=v"(v[2]) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:48" : "=v"(v[3]) : "v"(a));
            if constexpr (MODE == CH_DOT) {
              const unsigned b = rb_lds + 4u * (unsigned)q;
              asm volatile("ds_read_b128 %0, %1" : "=v"(w[0]) : "v"(b));
              asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(w[1]) : "v"(b));
              asm volatile("ds_read_b128 %0, %1 offset:32" : "=v"(w[2]) : "v"(b));
              asm volatile("ds_read_b128 %0, %1 offset:48" : "=v"(w[3]) : "v"(b));
            }
          };
          // wait until at most 8 reads are pending, with the set as operand
          auto wait8 = [&](f4 (&v)[4], f4 (&w)[4]) {
            if constexpr (MODE == CH_DOT)
              asm volatile("s_waitcnt lgkmcnt(8)"
                           : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(w[0]),
                             "+v"(w[1]), "+v"(w[2]), "+v"(w[3]));
            else
              asm volatile("s_waitcnt lgkmcnt(8)"
                           : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
          };
          auto add16 = [&](const f4 (&v)[4], const f4 (&w)[4]) {
#pragma unroll
            for (int z = 0; z < 16; ++z) {
              if constexpr (MODE == CH_DOT) acc = fmaf(v[z >> 2][z & 3], w[z >> 2][z & 3], acc);
              else acc = acc + v[z >> 2][z & 3];
            }
          };
          f4 va[4], wa[4], vb[4], wb[4], vc[4], wc[4];
          int full;
          if constexpr (MODE == CH_DOT) {
            full = cnt - cnt % 32;
            rd(0, va, wa);
            rd(16, vb, wb);
            for (int q = 0; q < full; q += 32) {
              wait8(va, wa);
              add16(va, wa);
              rd(q + 32, va, wa);
              wait8(vb, wb);
              add16(vb, wb);
              rd(q + 48, vb, wb);
            }
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(va[0]), "+v"(va[1]), "+v"(va[2]), "+v"(va[3]), "+v"(wa[0]),
                           "+v"(wa[1]), "+v"(wa[2]), "+v"(wa[3]), "+v"(vb[0]), "+v"(vb[1]),
                           "+v"(vb[2]), "+v"(vb[3]), "+v"(wb[0]), "+v"(wb[1]), "+v"(wb[2]),
                           "+v"(wb[3]));
          } else {
            full = cnt - cnt % 48;
            rd(0, va, wa);
            rd(16, vb, wb);
            rd(32, vc, wc);
            for (int q = 0; q < full; q += 48) {
              wait8(va, wa);
              add16(va, wa);
              rd(q + 48, va, wa);
              wait8(vb, wb);
              add16(vb, wb);
              rd(q + 64, vb, wb);
              wait8(vc, wc);
              add16(vc, wc);
              rd(q + 80, vc, wc);
            }
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(va[0]), "+v"(va[1]), "+v"(va[2]), "+v"(va[3]), "+v"(vb[0]),
                           "+v"(vb[1]), "+v"(vb[2]), "+v"(vb[3]), "+v"(vc[0]), "+v"(vc[1]),
                           "+v"(vc[2]), "+v"(vc[3]));
          }
          for (int q = full; q < cnt; ++q) {
            if constexpr (MODE == CH_DOT) acc = fmaf(row[q], rowb[q], acc);
            else acc = acc + row[q];
          }
        }
        __syncthreads();
      }
    }
    if (tid < 64) {  // lane-order epilogues (as block_chains)
      const bool lanes_form = MODE == CH_SRSS || (MODE == CH_VDELTA && grp == 1);
      if constexpr (MODE == CH_DOT) {
        if (tail && grp == 0) {
          const float xa = l < tail ? pa[nb8 + l] : 0.0f;
          const float xb = l < tail ? pb[nb8 + l] : 0.0f;
          acc = fmaf(xa, xb, acc);
        }
      }
      const float up = __shfl_down(acc, 4, 8);
      float x0 = (lanes_form && tail == 0 && quirk) ? acc : acc + up;
      if (lanes_form && l == 0)
        for (int k = 0; k < tail; ++k) {
          if (MODE == CH_SRSS) {
            const float d = mu - pa[nb8 + k];
            x0 = x0 + d * d;
          } else {
            const float d = scaled ? pa[nb8 + k] * scl : pa[nb8 + k];
            x0 = x0 + (pb[nb8 + k] - mu) * d;
          }
        }
      const float h = x0 + __shfl_down(x0, 1, 8);
      float r = h + __shfl_down(h, 2, 8);
      if (l == 0 && chain) {
        if constexpr (MODE == CH_DSUM) {
          for (int k = 0; k < tail; ++k) {
            const float d = pa[nb8 + k] * grad_apply(pb[nb8 + k], act);
            pw[nb8 + k] = d;
            r = r + d;
          }
        } else if (!lanes_form && MODE != CH_DOT) {
          for (int k = 0; k < tail; ++k) r = r + (scaled ? pa[nb8 + k] * scl : pa[nb8 + k]);
        }
        if (grp == 0) part0[blk] = r;
        else part1[blk] = r;
      }
    }
    __syncthreads();
  }
}

// per-channel passes: block results added over the groups in order
enum FinMode { FIN_MEAN = 0, FIN_VAR = 1, FIN_VDELTA = 2, FIN_ADD = 3 };
template <int MODE>
__global__ void chains_finish(const float* __restrict__ part0, const float* __restrict__ part1,
                              int64_t groups, int64_t N, int64_t bs, const float* __restrict__ var,
                              float* __restrict__ out0, float* __restrict__ out1) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= N) return;
  float m = 0.0f, v = 0.0f;
  for (int64_t g = 0; g < groups; ++g) {
    m = m + part0[g * N + i];
    if (MODE == FIN_VDELTA) v = v + part1[g * N + i];
  }
  if (MODE == FIN_MEAN) {
    out0[i] = m / (float)(groups * bs);
  } else if (MODE == FIN_VAR) {
    out0[i] = m / (float)(groups * bs - 1);
  } else if (MODE == FIN_VDELTA) {
    const float ve = var[i] > SEPS ? var[i] : SEPS;
    const float inv = -1.0f / sqrtf(ve);
    out0[i] = m * inv;
    out1[i] = (float)((double)v * -0.5 * pow((double)ve, -1.5));
  } else {
    out0[i] = out0[i] + m;
  }
}

// (BNB) per channel, over the groups in order: scale_updates += the dot
// sums; mean_delta / var_delta as FIN_VDELTA
__global__ void bnb_finish(const float* __restrict__ part0, const float* __restrict__ part1,
                           const float* __restrict__ part2, int64_t groups, int64_t N,
                           const float* __restrict__ var, float* __restrict__ dot_out,
                           float* __restrict__ mean_delta, float* __restrict__ var_delta) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= N) return;
  float d = 0.0f, m = 0.0f, v = 0.0f;
  for (int64_t g = 0; g < groups; ++g) {
    d = d + part0[g * N + i];
    m = m + part1[g * N + i];
    v = v + part2[g * N + i];
  }
  dot_out[i] = dot_out[i] + d;
  const float ve = var[i] > SEPS ? var[i] : SEPS;
  const float inv = -1.0f / sqrtf(ve);
  mean_delta[i] = m * inv;
  var_delta[i] = (float)((double)v * -0.5 * pow((double)ve, -1.5));
}

template <int MODE>
hipError_t run_chains(const float* a, const float* b, const float* mu, int64_t groups, int64_t N,
                      int64_t bs, int quirk, float* part0, float* part1, hipStream_t s,
                      int act = 0, float* wa = nullptr, const float* c3 = nullptr,
                      const float* sc = nullptr, const float* xx = nullptr,
                      float* part2 = nullptr) {
  const int64_t nblocks = groups * N;
  const unsigned grid = (unsigned)(nblocks < (1 << 20) ? nblocks : (1 << 20));
  if constexpr (MODE != CH_DDOT && MODE != CH_BNB) {
    if (bs >= 16384) {
      hipLaunchKernelGGL((block_chains_ws<MODE>), dim3(grid), dim3(256), 0, s, a, b, mu, nblocks,
                         N, bs, quirk, part0, part1, act, wa, c3, sc, xx, part2);
      return hipGetLastError();
    }
  }
  if (bs >= 4096)
    hipLaunchKernelGGL((block_chains<MODE, 256, 16>), dim3(grid), dim3(256), 0, s, a, b, mu,
                       nblocks, N, bs, quirk, part0, part1, act, wa, c3, sc, xx, part2);
  else
    hipLaunchKernelGGL((block_chains<MODE, 64, 8>), dim3(grid), dim3(64), 0, s, a, b, mu, nblocks,
                       N, bs, quirk, part0, part1, act, wa, c3, sc, xx, part2);
  return hipGetLastError();
}

template <int MODE>
hipError_t run_finish(const float* part0, const float* part1, int64_t groups, int64_t N,
                      int64_t bs, const float* var, float* out0, float* out1, hipStream_t s) {
  hipLaunchKernelGGL(chains_finish<MODE>, dim3(nblk(N)), dim3(TPB), 0, s, part0, part1, groups,
                     N, bs, var, out0, out1);
  return hipGetLastError();
}

// blocks long enough for the chain kernels (shorter ones: one thread per
// channel, which is also the only form for blockSize 1)
bool use_chains(int64_t bs, const float* part) { return part != nullptr && bs >= 64; }
}  // namespace
bool bn_folds_scale(int64_t bs) { return use_chains(bs, reinterpret_cast<const float*>(1)); }
namespace {

// ---- conv layer batch norm, forward (TBaseLayer.batchNorm + activate) -----
// One pass instead of the reference's six (CopyTo(x), blockNormalize,
// copyTo(x_norm), forwardScale, forwardBias, activate; nbaselayer.pas:351-
// 365, nConvolutionLayer.pas:530-545) with the same per-element roundings:
// x := y; xn := (y - m) / sd; out := act(xn*scale + bias), sd as
// blockNormalize (bs == 1: sqrt(max(v, eps)); bs > 1: max(sqrt(v), eps)).
template <int V>
__global__ __launch_bounds__(TPB) void bn_apply_k(const float* y,  // may alias out
                                                  float* __restrict__ x, float* __restrict__ xn,
                                                  float* out, int64_t total_v,
                                                  int64_t N, int64_t bs,
                                                  const float* __restrict__ means,
                                                  const float* __restrict__ vars,
                                                  const float* __restrict__ scales,
                                                  const float* __restrict__ biases, int act) {
  for (int64_t e = (int64_t)blockIdx.x * TPB + threadIdx.x; e < total_v;
       e += (int64_t)gridDim.x * TPB) {
    float v[V], a[V], o[V];
    if constexpr (V == 4) {
      const float4 t = reinterpret_cast<const float4*>(y)[e];
      v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
      v[0] = y[e];
    }
    const int64_t i = ((e * V) / bs) % N;  // bs % V == 0: one channel per vector
    const float m = means[i], var = vars[i], sc = scales[i], bi = biases[i];
    float sd;
    if (bs == 1) {
      sd = sqrtf(var > SEPS ? var : SEPS);
    } else {
      sd = sqrtf(var);
      sd = sd > SEPS ? sd : SEPS;
    }
#pragma unroll
    for (int j = 0; j < V; ++j) {
      a[j] = (v[j] - m) / sd;
      float t = a[j] * sc;
      t = t + bi;
      o[j] = act_apply(t, act);
    }
    if constexpr (V == 4) {
      if (x) reinterpret_cast<float4*>(x)[e] = make_float4(v[0], v[1], v[2], v[3]);
      if (xn) reinterpret_cast<float4*>(xn)[e] = make_float4(a[0], a[1], a[2], a[3]);
      reinterpret_cast<float4*>(out)[e] = make_float4(o[0], o[1], o[2], o[3]);
    } else {
      if (x) x[e] = v[0];
      if (xn) xn[e] = a[0];
      out[e] = o[0];
    }
  }
}

// ---- row form of the per-channel elementwise passes ------------------------
// A workgroup owns a segment of one (group, channel) row of bs contiguous
// elements, so the channel's constants are read once per workgroup and no
// element pays the 64-bit (e / bs) % N of the grid-stride forms — that integer
// division, not HBM, bounded them on the conv shapes (normalizeDelta 3.6 TB/s
// at 8 x 32 x 173056).  Same per-element arithmetic, same order.  V = 4 on
// 16-byte aligned rows with bs % 4 == 0.
constexpr int RU = 4;  // vectors per thread

__device__ __forceinline__ void row_of(int bpr, int64_t N, int64_t& row, int64_t& ch, int& seg) {
  row = (int64_t)(blockIdx.x / (unsigned)bpr);
  seg = (int)(blockIdx.x - (unsigned)row * (unsigned)bpr);
  ch = row % N;
}

template <int V>
__device__ __forceinline__ void ld(const float* p, float (&v)[V]) {
  if constexpr (V == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
    v[0] = *p;
  }
}
template <int V>
__device__ __forceinline__ void st(float* p, const float (&v)[V]) {
  if constexpr (V == 4)
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  else
    *p = v[0];
}

// (FIN: the CH_BNB finish folded in — each block sums its channel's group
// partials in order (bnb_finish's arithmetic) for its mean / variance
// deltas, and the channel's first block stores them and adds the dot sums
// to scale_updates: one launch less per layer)
struct BnbFin {
  const float *p0, *p1, *p2;
  int64_t groups;
  float *dot_out, *md_out, *vd_out;
};
template <int V, bool FIN = false>
__global__ __launch_bounds__(TPB) void normalize_delta_rows(
    const float* __restrict__ x, const float* __restrict__ mean, const float* __restrict__ var,
    const float* __restrict__ mean_delta, const float* __restrict__ var_delta,
    float* __restrict__ delta, int64_t N, int64_t bs, int bpr, float B,
    const float* __restrict__ scales, const float* __restrict__ out, int act, BnbFin fin) {
  int64_t row, i;
  int seg;
  row_of(bpr, N, row, i, seg);
  // (out: Derivative folded in first, delta * f'(out); scales: forwardScale)
  const bool scaled = scales != nullptr;
  const float scl = scaled ? scales[i] : 1.0f;
  float mdi, vdi;
  if constexpr (FIN) {
    __shared__ float sh[2];
    if (threadIdx.x == 0) {
      float d = 0.0f, m = 0.0f, v = 0.0f;
      for (int64_t g = 0; g < fin.groups; ++g) {
        d = d + fin.p0[g * N + i];
        m = m + fin.p1[g * N + i];
        v = v + fin.p2[g * N + i];
      }
      const float ve = var[i] > SEPS ? var[i] : SEPS;
      const float inv = -1.0f / sqrtf(ve);
      const float mdv = m * inv;
      const float vdv = (float)((double)v * -0.5 * pow((double)ve, -1.5));
      if (row < N && seg == 0) {  // (group 0's first block of the channel)
        fin.dot_out[i] = fin.dot_out[i] + d;
        fin.md_out[i] = mdv;
        fin.vd_out[i] = vdv;
      }
      sh[0] = mdv;
      sh[1] = vdv;
    }
    __syncthreads();
    mdi = sh[0];
    vdi = sh[1];
  } else {
    mdi = mean_delta[i];
    vdi = var_delta[i];
  }
  const float md = mdi / B;
  const float vd = 2.0f * vdi / B;
  const float ve = var[i] > SEPS ? var[i] : SEPS;
  const float sd = sqrtf(ve);
  const float m = mean[i];
  const int64_t base = row * bs;
#pragma unroll
  for (int u = 0; u < RU; ++u) {
    const int64_t j = ((int64_t)seg * RU * TPB + u * TPB + threadIdx.x) * V;
    if (j >= bs) break;
    float d[V], xv[V], ov[V];
    ld<V>(delta + base + j, d);
    ld<V>(x + base + j, xv);
    if (out) ld<V>(out + base + j, ov);
#pragma unroll
    for (int c = 0; c < V; ++c) {
      if (out) d[c] = d[c] * grad_apply(ov[c], act);
      const float dv = scaled ? d[c] * scl : d[c];
      const float a = dv / sd;
      const float t = (xv[c] - m) * vd + md;  // sNormalizeDelta_avx order
      d[c] = a + t;
    }
    st<V>(delta + base + j, d);
  }
}

template <int V>
__global__ __launch_bounds__(TPB) void scale_add_rows(float* __restrict__ x, int64_t N, int64_t bs,
                                                      int bpr, const float* __restrict__ scales,
                                                      const float* __restrict__ biases,
                                                      int64_t incb) {
  int64_t row, i;
  int seg;
  row_of(bpr, N, row, i, seg);
  const float sc = scales[i * incb];
  const float bi = biases ? biases[i * incb] : 0.0f;
  const int64_t base = row * bs;
#pragma unroll
  for (int u = 0; u < RU; ++u) {
    const int64_t j = ((int64_t)seg * RU * TPB + u * TPB + threadIdx.x) * V;
    if (j >= bs) break;
    float v[V];
    ld<V>(x + base + j, v);
#pragma unroll
    for (int c = 0; c < V; ++c) {
      v[c] = v[c] * sc;                // forwardScale (vsMulB)
      if (biases) v[c] = v[c] + bi;    // forwardBias  (vsAddB)
    }
    st<V>(x + base + j, v);
  }
}

template <int V>
__global__ __launch_bounds__(TPB) void normalize_rows(float* __restrict__ x, int64_t N, int64_t bs,
                                                      int bpr, const float* __restrict__ means,
                                                      int64_t mstride,
                                                      const float* __restrict__ vars,
                                                      int64_t vstride) {
  int64_t row, i;
  int seg;
  row_of(bpr, N, row, i, seg);
  const float m = means[i * mstride];
  float sd = sqrtf(vars[i * vstride]);  // (bs > 1) _snormblkvv -> snormvss
  sd = sd > SEPS ? sd : SEPS;
  const int64_t base = row * bs;
#pragma unroll
  for (int u = 0; u < RU; ++u) {
    const int64_t j = ((int64_t)seg * RU * TPB + u * TPB + threadIdx.x) * V;
    if (j >= bs) break;
    float v[V];
    ld<V>(x + base + j, v);
#pragma unroll
    for (int c = 0; c < V; ++c) v[c] = (v[c] - m) / sd;
    st<V>(x + base + j, v);
  }
}

template <int V>
__global__ __launch_bounds__(TPB) void bn_apply_rows(const float* y,  // may alias out
                                                     float* __restrict__ x,
                                                     float* __restrict__ xn, float* out,
                                                     int64_t N, int64_t bs, int bpr,
                                                     const float* __restrict__ means,
                                                     const float* __restrict__ vars,
                                                     const float* __restrict__ scales,
                                                     const float* __restrict__ biases, int act) {
  int64_t row, i;
  int seg;
  row_of(bpr, N, row, i, seg);
  const float m = means[i], sc = scales[i], bi = biases[i];
  float sd = sqrtf(vars[i]);
  sd = sd > SEPS ? sd : SEPS;
  const int64_t base = row * bs;
#pragma unroll
  for (int u = 0; u < RU; ++u) {
    const int64_t j = ((int64_t)seg * RU * TPB + u * TPB + threadIdx.x) * V;
    if (j >= bs) break;
    float v[V], a[V], o[V];
    ld<V>(y + base + j, v);
#pragma unroll
    for (int c = 0; c < V; ++c) {
      a[c] = (v[c] - m) / sd;
      float t = a[c] * sc;
      t = t + bi;
      o[c] = act_apply(t, act);
    }
    if (x) st<V>(x + base + j, v);
    if (xn) st<V>(xn + base + j, a);
    st<V>(out + base + j, o);
  }
}

// rolling_mean.Multiply(1 - m); rolling_mean.axpy(m, mean) and the same for
// the variance (nbaselayer.pas:353-356): one multiply, then one FMA
__global__ void rolling_update_k(int64_t n, float* __restrict__ rm, float* __restrict__ rv,
                                 const float* __restrict__ mean, const float* __restrict__ var,
                                 float keep, float mom) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  rm[i] = fmaf(mom, mean[i], rm[i] * keep);
  rv[i] = fmaf(mom, var[i], rv[i] * keep);
}

}  // namespace

// row form for blocks of >= 256 elements (the conv shapes); returns the
// workgroups per row, 0 when the grid-stride form is used instead
static int row_bpr(int64_t rows, int64_t bs, int V) {
  if (bs < 256) return 0;
  const int64_t span = (int64_t)TPB * RU * V;
  const int64_t bpr = (bs + span - 1) / span;
  return rows * bpr <= 0x7fffffffLL ? (int)bpr : 0;
}
static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

hipError_t launch_bn_apply(const float* y, float* x, float* xn, float* out, int64_t groups,
                           int64_t N, int64_t bs, const float* means, const float* vars,
                           const float* scales, const float* biases, int act, hipStream_t s) {
  const int64_t total = groups * N * bs;
  if (total <= 0) return hipSuccess;
  const auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const bool v4 = bs % 4 == 0 && al(y) && al(out) && (!x || al(x)) && (!xn || al(xn));
  if (const int bpr = row_bpr(groups * N, bs, v4 ? 4 : 1)) {
    if (v4)
      hipLaunchKernelGGL(bn_apply_rows<4>, dim3((unsigned)(groups * N * bpr)), dim3(TPB), 0, s, y,
                         x, xn, out, N, bs, bpr, means, vars, scales, biases, act);
    else
      hipLaunchKernelGGL(bn_apply_rows<1>, dim3((unsigned)(groups * N * bpr)), dim3(TPB), 0, s, y,
                         x, xn, out, N, bs, bpr, means, vars, scales, biases, act);
    return hipGetLastError();
  }
  if (v4)
    hipLaunchKernelGGL(bn_apply_k<4>, dim3(nblk(total / 4)), dim3(TPB), 0, s, y, x, xn, out,
                       total / 4, N, bs, means, vars, scales, biases, act);
  else
    hipLaunchKernelGGL(bn_apply_k<1>, dim3(nblk(total)), dim3(TPB), 0, s, y, x, xn, out, total,
                       N, bs, means, vars, scales, biases, act);
  return hipGetLastError();
}

hipError_t launch_rolling_update(int64_t n, float* rm, float* rv, const float* mean,
                                 const float* var, float momentum, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const float keep = 1.0f - momentum;
  hipLaunchKernelGGL(rolling_update_k, dim3(nblk(n)), dim3(TPB), 0, s, n, rm, rv, mean, var, keep,
                     momentum);
  return hipGetLastError();
}

namespace {
}  // namespace

hipError_t launch_means_vars(const float* x, int64_t groups, int64_t N, int64_t bs, float* means,
                             float* vars, int quirk, float* part, hipStream_t s, int what) {
  if (N <= 0) return hipSuccess;
  // one thread per channel for FC shapes (blockSize 1) and short blocks;
  // longer blocks: the lane chains per block, then the group-order sums
  // (the variance pass needs the finished means)
  if (!use_chains(bs, part)) {
    hipLaunchKernelGGL(means_vars_seq, dim3(nblk(N)), dim3(TPB), 0, s, x, groups, N, bs, means,
                       vars, quirk, what);
    return hipGetLastError();
  }
  hipError_t e;
  if (what & MV_MEAN)
    if ((e = run_chains<CH_SUM>(x, nullptr, nullptr, groups, N, bs, 0, part, nullptr, s)) ||
        (e = run_finish<FIN_MEAN>(part, nullptr, groups, N, bs, nullptr, means, nullptr, s)))
      return e;
  if (!(what & MV_VAR)) return hipSuccess;
  if ((e = run_chains<CH_SRSS>(x, nullptr, means, groups, N, bs, quirk, part, nullptr, s)))
    return e;
  return run_finish<FIN_VAR>(part, nullptr, groups, N, bs, nullptr, vars, nullptr, s);
}

hipError_t launch_normalize(float* x, int64_t groups, int64_t N, int64_t bs, const float* means,
                            int64_t mstride, const float* vars, int64_t vstride, hipStream_t s) {
  const int64_t total = groups * N * bs;
  if (total <= 0) return hipSuccess;
  const bool v4 = bs % 4 == 0 && al16(x);
  if (const int bpr = row_bpr(groups * N, bs, v4 ? 4 : 1)) {
    if (v4)
      hipLaunchKernelGGL(normalize_rows<4>, dim3((unsigned)(groups * N * bpr)), dim3(TPB), 0, s, x,
                         N, bs, bpr, means, mstride, vars, vstride);
    else
      hipLaunchKernelGGL(normalize_rows<1>, dim3((unsigned)(groups * N * bpr)), dim3(TPB), 0, s, x,
                         N, bs, bpr, means, mstride, vars, vstride);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(normalize_k, dim3(nblk(total)), dim3(TPB), 0, s, x, total, N, bs, means,
                     mstride, vars, vstride);
  return hipGetLastError();
}

hipError_t launch_scale_add(float* x, int64_t groups, int64_t N, int64_t bs, const float* scales,
                            const float* biases, int64_t incb, hipStream_t s) {
  const int64_t total = groups * N * bs;
  if (total <= 0) return hipSuccess;
  const bool v4 = bs % 4 == 0 && al16(x);
  if (const int bpr = row_bpr(groups * N, bs, v4 ? 4 : 1)) {
    if (v4)
      hipLaunchKernelGGL(scale_add_rows<4>, dim3((unsigned)(groups * N * bpr)), dim3(TPB), 0, s, x,
                         N, bs, bpr, scales, biases, incb);
    else
      hipLaunchKernelGGL(scale_add_rows<1>, dim3((unsigned)(groups * N * bpr)), dim3(TPB), 0, s, x,
                         N, bs, bpr, scales, biases, incb);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(scale_add_k, dim3(nblk(total)), dim3(TPB), 0, s, x, total, N, bs, scales,
                     biases, incb);
  return hipGetLastError();
}

hipError_t launch_add_dots(float* dst, const float* a, const float* b, int64_t groups, int64_t N,
                           int64_t bs, float* part, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  if (!use_chains(bs, part)) {
    hipLaunchKernelGGL(add_dots_seq, dim3(nblk(N)), dim3(TPB), 0, s, dst, a, b, groups, N, bs);
    return hipGetLastError();
  }
  if (hipError_t e = run_chains<CH_DOT>(a, b, nullptr, groups, N, bs, 0, part, nullptr, s))
    return e;
  return run_finish<FIN_ADD>(part, nullptr, groups, N, bs, nullptr, dst, nullptr, s);
}

hipError_t launch_add_sums(float* dst, const float* src, int64_t groups, int64_t N, int64_t bs,
                           float* part, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  if (bs == 1 && N == 1)  // stride 1: sumv is vssum_avx2 over the groups
    return launch_backward_bias(dst, 1, src, groups, 1, 1, s);
  if (bs == 1) {
    hipLaunchKernelGGL(add_sums_seq, dim3(nblk(N)), dim3(TPB), 0, s, dst, src, groups, N);
    return hipGetLastError();
  }
  if (!use_chains(bs, part)) return launch_backward_bias(dst, N, src, bs, groups, 1, s);
  if (hipError_t e = run_chains<CH_SUM>(src, nullptr, nullptr, groups, N, bs, 0, part, nullptr, s))
    return e;
  return run_finish<FIN_ADD>(part, nullptr, groups, N, bs, nullptr, dst, nullptr, s);
}

// Derivative() then addSums(delta) of the conv backward (nConvolutionLayer.pas:
// 583-598) in one pass: each term delta * f'(output) written back and summed
// in the chains of launch_add_sums — the same values and sums as the two
// launches (which remain the path where the chains do not apply)
hipError_t launch_derive_add_sums(float* dst, float* delta, const float* output, int act,
                                  int64_t groups, int64_t N, int64_t bs, float* part,
                                  hipStream_t s) {
  if (N <= 0 || groups <= 0 || bs <= 0) return hipSuccess;
  // (the planes of >= 16384 pixels, whose chain kernel is one block per
  // plane with three staging waves, keep the separate derivative pass: the
  // extra read and write stream there outlasts the chains, YOLOv3 layer 0
  // 0.57 -> 0.68 ms a call)
  if (act == TNS_acLINEAR || bs == 1 || bs >= 16384 || !use_chains(bs, part)) {
    if (hipError_t e = launch_derive(output, groups * N * bs, act, delta, s)) return e;
    return launch_add_sums(dst, delta, groups, N, bs, part, s);
  }
  if (hipError_t e = run_chains<CH_DSUM>(delta, output, nullptr, groups, N, bs, 0, part, nullptr, s,
                                         act, delta))
    return e;
  return run_finish<FIN_ADD>(part, nullptr, groups, N, bs, nullptr, dst, nullptr, s);
}

// the BN conv backward's Derivative and addDots in one pass (CH_DDOT): delta
// *= f'(output) written back, dst += sum x_norm * delta in the sdot order;
// the planes of >= 16384 pixels (the specialised-wave chain form stages two
// streams) and the short blocks keep the two passes
hipError_t launch_add_dots_derive(float* dst, const float* x_norm, float* delta,
                                  const float* output, int act, int64_t groups, int64_t N,
                                  int64_t bs, float* part, hipStream_t s) {
  if (N <= 0 || groups <= 0 || bs <= 0) return hipSuccess;
  if (act == TNS_acLINEAR || bs >= 16384 || !use_chains(bs, part)) {
    if (hipError_t e = launch_derive(output, groups * N * bs, act, delta, s)) return e;
    return launch_add_dots(dst, x_norm, delta, groups, N, bs, part, s);
  }
  if (hipError_t e = run_chains<CH_DDOT>(delta, x_norm, nullptr, groups, N, bs, 0, part, nullptr,
                                         s, act, delta, output))
    return e;
  return run_finish<FIN_ADD>(part, nullptr, groups, N, bs, nullptr, dst, nullptr, s);
}
hipError_t launch_mean_var_delta(const float* delta, const float* x, const float* mean,
                                 const float* var, int64_t groups, int64_t N, int64_t bs,
                                 float* mean_delta, float* var_delta, int quirk, float* part,
                                 hipStream_t s, const float* scales) {
  if (N <= 0) return hipSuccess;
  // (the one-thread-per-channel form has no folded scale: the caller runs
  // forwardScale first there — bn_folds_scale says which)
  if (scales && !use_chains(bs, part)) return hipErrorInvalidValue;
  if (!use_chains(bs, part)) {
    hipLaunchKernelGGL(mean_var_delta_seq, dim3(nblk(N)), dim3(TPB), 0, s, delta, x, mean, var,
                       groups, N, bs, mean_delta, var_delta, quirk);
    return hipGetLastError();
  }
  float* part1 = part + groups * N;
  if (hipError_t e = run_chains<CH_VDELTA>(delta, x, mean, groups, N, bs, quirk, part, part1, s,
                                           0, nullptr, nullptr, scales))
    return e;
  return run_finish<FIN_VDELTA>(part, part1, groups, N, bs, var, mean_delta, var_delta, s);
}

hipError_t launch_normalize_delta(const float* x, const float* mean, const float* var,
                                  const float* mean_delta, const float* var_delta, float* delta,
                                  int64_t groups, int64_t N, int64_t bs, hipStream_t s,
                                  const float* scales) {
  const int64_t total = groups * N * bs;
  if (total <= 0) return hipSuccess;
  const bool v4 = bs % 4 == 0 && al16(x) && al16(delta);
  if (const int bpr = row_bpr(groups * N, bs, v4 ? 4 : 1)) {
    if (v4)
      hipLaunchKernelGGL(normalize_delta_rows<4>, dim3((unsigned)(groups * N * bpr)), dim3(TPB), 0,
                         s, x, mean, var, mean_delta, var_delta, delta, N, bs, bpr,
                         (float)(groups * bs), scales, nullptr, 0, BnbFin{});
    else
      hipLaunchKernelGGL(normalize_delta_rows<1>, dim3((unsigned)(groups * N * bpr)), dim3(TPB), 0,
                         s, x, mean, var, mean_delta, var_delta, delta, N, bs, bpr,
                         (float)(groups * bs), scales, nullptr, 0, BnbFin{});
    return hipGetLastError();
  }
  hipLaunchKernelGGL(normalize_delta_k, dim3(nblk(total)), dim3(TPB), 0, s, x, mean, var,
                     mean_delta, var_delta, delta, total, N, bs, (float)(groups * bs), scales,
                     nullptr, 0);
  return hipGetLastError();
}

// the BN conv backward (Derivative, addDots, forwardScale, MeansAndVarsDelta,
// normalizeDelta) as one CH_BNB chain pass + its finish + normalizeDelta with
// the Derivative and the scale applied to each loaded term; hipErrorNotSupported
// where it does not apply (short blocks, planes that the row form of
// normalizeDelta does not cover): the caller runs the separate passes.  part: 3 * groups * N floats
hipError_t launch_bn_backward_fused(float* scale_updates, const float* x_norm, float* delta,
                                    const float* output, int act, const float* x,
                                    const float* mean, const float* var, const float* scales,
                                    float* mean_delta, float* var_delta, int64_t groups,
                                    int64_t N, int64_t bs, int quirk, float* part, hipStream_t s) {
  if (N <= 0 || groups <= 0 || bs <= 0) return hipSuccess;
  // (the >= 16384-pixel planes keep the separate passes: a specialised-wave
  // form of this pass with four LDS streams was bit-exact and no faster —
  // YOLOv3 training backward 17.22 ms without it, 17.27 with it,
  // profiles/r06_bn_fused_ws.json)
  if (bs >= 16384 || !use_chains(bs, part)) return hipErrorNotSupported;
  const bool v4 = bs % 4 == 0 && al16(x) && al16(delta) && al16(output);
  const int bpr = row_bpr(groups * N, bs, v4 ? 4 : 1);
  float* part1 = part + groups * N;
  float* part2 = part + 2 * groups * N;
  if (hipError_t e = run_chains<CH_BNB>(delta, x_norm, mean, groups, N, bs, quirk, part, part1, s,
                                        act, nullptr, output, scales, x, part2))
    return e;
  if (!bpr) {  // (short planes: the finish, then the element form of normalizeDelta)
    hipLaunchKernelGGL(bnb_finish, dim3(nblk(N)), dim3(TPB), 0, s, part, part1, part2, groups, N,
                       var, scale_updates, mean_delta, var_delta);
    if (hipError_t e = hipGetLastError()) return e;
    const int64_t total = groups * N * bs;
    hipLaunchKernelGGL(normalize_delta_k, dim3(nblk(total)), dim3(TPB), 0, s, x, mean, var,
                       mean_delta, var_delta, delta, total, N, bs, (float)(groups * bs), scales,
                       output, act);
    return hipGetLastError();
  }
  const BnbFin fin{part, part1, part2, groups, scale_updates, mean_delta, var_delta};
  if (v4)
    hipLaunchKernelGGL((normalize_delta_rows<4, true>), dim3((unsigned)(groups * N * bpr)), dim3(TPB),
                       0, s, x, mean, var, mean_delta, var_delta, delta, N, bs, bpr,
                       (float)(groups * bs), scales, output, act, fin);
  else
    hipLaunchKernelGGL((normalize_delta_rows<1, true>), dim3((unsigned)(groups * N * bpr)), dim3(TPB),
                       0, s, x, mean, var, mean_delta, var_delta, delta, N, bs, bpr,
                       (float)(groups * bs), scales, output, act, fin);
  return hipGetLastError();
}

hipError_t launch_softmax_batch(int64_t n, const float* in, int64_t batch, int64_t batch_size,
                                int64_t groups, int64_t group_size, int64_t stride, float temp,
                                float* out, hipStream_t s) {
  if (batch * groups <= 0) return hipSuccess;
  hipLaunchKernelGGL(softmax_batch_k, dim3(nblk(batch * groups)), dim3(TPB), 0, s, n, in, batch,
                     batch_size, groups, group_size, stride, temp, out);
  return hipGetLastError();
}

hipError_t launch_xent_softmax(int64_t n, const float* pred, const float* truth, float* delta,
                               float* error, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(xent_softmax_k, dim3(nblk(n)), dim3(TPB), 0, s, n, pred, truth, delta,
                     error);
  return hipGetLastError();
}

hipError_t launch_vssum(int64_t n, const float* a, float* out, hipStream_t s) {
  hipLaunchKernelGGL(vssum_k, dim3(1), dim3(64), 0, s, n, a, out);
  return hipGetLastError();
}

}  // namespace tns
