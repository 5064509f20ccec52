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

// one thread per channel (FC layers: blockSize 1, groups = batch)
__global__ void means_vars_seq(const float* __restrict__ x, int64_t groups, int64_t N, int64_t bs,
                               float* __restrict__ means, float* __restrict__ vars, int quirk) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= N) return;
  const float S = (float)(groups * bs), S2 = (float)(groups * bs - 1);
  float m = 0.0f;
  for (int64_t b = 0; b < groups; ++b) m = m + vssum8(x + (i + b * N) * bs, bs);
  m = m / S;
  means[i] = m;
  float v = 0.0f;
  for (int64_t b = 0; b < groups; ++b) v = v + srss8(x + (i + b * N) * bs, bs, m, quirk);
  vars[i] = v / S2;
}

// one workgroup per channel (conv layers): 8 consecutive lanes own a block
// (lane l = the vssum / srss lane), block results meet in LDS and one thread
// adds them in group order
constexpr int MV_SLOTS = TPB / 8;
constexpr int MV_CHUNK = 1024;
constexpr int MV_UNR = 64;
__global__ __launch_bounds__(TPB) void means_vars_lanes(const float* __restrict__ x,
                                                        int64_t groups, int64_t N, int64_t bs,
                                                        float* __restrict__ means,
                                                        float* __restrict__ vars, int quirk) {
  __shared__ float tot[MV_CHUNK];
  __shared__ float mean_s;
  const int64_t i = blockIdx.x;
  const int l = threadIdx.x & 7, q = threadIdx.x >> 3;
  const int64_t nb = bs >> 3;
  const bool tail = (bs & 7) != 0;
  float m = 0.0f, v = 0.0f;
  for (int pass = 0; pass < 2; ++pass) {
    const float mu = pass ? mean_s : 0.0f;
    float run = 0.0f;
    for (int64_t j0 = 0; j0 < groups; j0 += MV_CHUNK) {
      const int64_t jn = groups - j0 < MV_CHUNK ? groups - j0 : MV_CHUNK;
      for (int64_t jj = q; jj < ((jn + MV_SLOTS - 1) / MV_SLOTS) * MV_SLOTS; jj += MV_SLOTS) {
        const bool on = jj < jn;
        const float* blk = x + ((j0 + (on ? jj : 0)) * N + i) * bs;
        float acc = 0.0f;
        if (on) {
          const float* p = blk + l;
          int64_t t = 0;
          // MV_UNR loads in flight per lane ahead of its (sequential) adds:
          // with one wave per channel-group set, memory-level parallelism
          // per lane is what bounds this pass
          for (; t + MV_UNR <= nb; t += MV_UNR) {
            float w[MV_UNR];
#pragma unroll
            for (int u = 0; u < MV_UNR; ++u) w[u] = p[8 * (t + u)];
#pragma unroll
            for (int u = 0; u < MV_UNR; ++u) {
              if (pass) {
                const float d = mu - w[u];
                acc = acc + d * d;
              } else {
                acc = acc + w[u];
              }
            }
          }
          for (; t < nb; ++t) {
            if (pass) {
              const float d = mu - p[8 * t];
              acc = acc + d * d;
            } else {
              acc = acc + p[8 * t];
            }
          }
        }
        const bool drop = pass && !tail && quirk;          // srss without a tail
        const float up = __shfl_down(acc, 4, 8);           // lane l+4
        float x0 = drop ? acc : acc + up;                  // lanes 0..3: x_l
        if (pass && tail && on && l == 0)                  // srss: tail into lane 0
          for (int64_t u = nb * 8; u < bs; ++u) {
            const float d = mu - blk[u];
            x0 = x0 + d * d;
          }
        const float h = x0 + __shfl_down(x0, 1, 8);        // x0+x1 (l=0), x2+x3 (l=2)
        float r = h + __shfl_down(h, 2, 8);                // (x0+x1)+(x2+x3)
        if (on && l == 0) {
          if (!pass)                                       // vssum: tail after the fold
            for (int64_t u = nb * 8; u < bs; ++u) r = r + blk[u];
          tot[jj] = r;
        }
      }
      __syncthreads();
      if (threadIdx.x == 0)
        for (int64_t jj = 0; jj < jn; ++jj) run = run + tot[jj];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      if (pass) {
        v = run / (float)(groups * bs - 1);
      } else {
        m = run / (float)(groups * bs);
        mean_s = m;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    means[i] = m;
    vars[i] = v;
  }
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

// conv blocks: one workgroup per channel, one thread per group computing its
// block's sdot_avx2 (same lanes, same fold); thread 0 sums them in group
// order and adds to dst as add_dots_seq does
__device__ __forceinline__ float sdot8_block(const float* pa, const float* pb, int64_t bs) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t blocks = bs >> 3;
  int64_t t = 0;
  for (; t + 4 <= blocks; t += 4) {  // 32 operand pairs ahead of the FMAs
    float wa[32], wb[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      wa[u] = pa[8 * t + u];
      wb[u] = pb[8 * t + u];
    }
#pragma unroll
    for (int u = 0; u < 32; ++u) acc[u & 7] = fmaf(wa[u], wb[u], acc[u & 7]);
  }
  for (; t < blocks; ++t)
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
  return (s0 + s1) + (s2 + s3);
}

__global__ __launch_bounds__(TPB) void add_dots_blocks(float* __restrict__ dst,
                                                       const float* __restrict__ a,
                                                       const float* __restrict__ b,
                                                       int64_t groups, int64_t N, int64_t bs) {
  __shared__ float part[TPB];
  const int64_t i = blockIdx.x;
  float sum = 0.0f;
  for (int64_t j0 = 0; j0 < groups; j0 += TPB) {
    const int64_t jn = groups - j0 < TPB ? groups - j0 : TPB;
    if (threadIdx.x < jn) {
      const int64_t g = j0 + threadIdx.x;
      part[threadIdx.x] = sdot8_block(a + (i + g * N) * bs, b + (i + g * N) * bs, bs);
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int64_t jj = 0; jj < jn; ++jj) sum = sum + part[jj];
    __syncthreads();
  }
  if (threadIdx.x == 0) dst[i] = dst[i] + sum;
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

__global__ void mean_var_delta_seq(const float* __restrict__ delta, const float* __restrict__ x,
                                   const float* __restrict__ mean, const float* __restrict__ var,
                                   int64_t groups, int64_t N, int64_t bs,
                                   float* __restrict__ mean_delta, float* __restrict__ var_delta) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= N) return;
  float m = 0.0f, v = 0.0f;
  const float mu = mean[i];
  for (int64_t j = 0; j < groups; ++j) {
    const float* dd = delta + (i + j * N) * bs;
    const float* xx = x + (i + j * N) * bs;
    m = m + vssum8(dd, bs);
    float t = 0.0f;
    for (int64_t k = 0; k < bs; ++k) t = t + (xx[k] - mu) * dd[k];
    v = v + t;
  }
  const float ve = var[i] > SEPS ? var[i] : SEPS;
  const float inv = -1.0f / sqrtf(ve);
  mean_delta[i] = m * inv;
  var_delta[i] = (float)((double)v * -0.5 * pow((double)ve, -1.5));
}

// conv blocks: one workgroup per channel, one thread per group — each
// group's block sums (vssum8 of delta, the sequential (x-mu)*delta chain) are
// independent; thread 0 adds them in group order as mean_var_delta_seq does
__global__ __launch_bounds__(TPB) void mean_var_delta_blocks(
    const float* __restrict__ delta, const float* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ var, int64_t groups, int64_t N, int64_t bs,
    float* __restrict__ mean_delta, float* __restrict__ var_delta) {
  __shared__ float ms[TPB], vs[TPB];
  const int64_t i = blockIdx.x;
  const float mu = mean[i];
  float m = 0.0f, v = 0.0f;
  for (int64_t j0 = 0; j0 < groups; j0 += TPB) {
    const int64_t jn = groups - j0 < TPB ? groups - j0 : TPB;
    if (threadIdx.x < jn) {
      const int64_t j = j0 + threadIdx.x;
      const float* dd = delta + (i + j * N) * bs;
      const float* xx = x + (i + j * N) * bs;
      ms[threadIdx.x] = vssum8(dd, bs);
      // the chain is sequential; its operands are loaded MV_UNR ahead
      float t = 0.0f;
      int64_t k = 0;
      for (; k + MV_UNR <= bs; k += MV_UNR) {
        float xa[MV_UNR], da[MV_UNR];
#pragma unroll
        for (int u = 0; u < MV_UNR; ++u) {
          xa[u] = xx[k + u];
          da[u] = dd[k + u];
        }
#pragma unroll
        for (int u = 0; u < MV_UNR; ++u) t = t + (xa[u] - mu) * da[u];
      }
      for (; k < bs; ++k) t = t + (xx[k] - mu) * dd[k];
      vs[threadIdx.x] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int64_t jj = 0; jj < jn; ++jj) {
        m = m + ms[jj];
        v = v + vs[jj];
      }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float ve = var[i] > SEPS ? var[i] : SEPS;
    const float inv = -1.0f / sqrtf(ve);
    mean_delta[i] = m * inv;
    var_delta[i] = (float)((double)v * -0.5 * pow((double)ve, -1.5));
  }
}

__global__ void normalize_delta_k(const float* __restrict__ x, const float* __restrict__ mean,
                                  const float* __restrict__ var,
                                  const float* __restrict__ mean_delta,
                                  const float* __restrict__ var_delta, float* __restrict__ delta,
                                  int64_t total, int64_t N, int64_t bs, float B) {
  for (int64_t e = (int64_t)blockIdx.x * TPB + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * TPB) {
    const int64_t i = (e / bs) % N;
    const float md = mean_delta[i] / B;
    const float vd = 2.0f * var_delta[i] / B;
    const float ve = var[i] > SEPS ? var[i] : SEPS;
    const float sd = sqrtf(ve);
    const float a = delta[e] / sd;
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

}  // namespace

hipError_t launch_means_vars(const float* x, int64_t groups, int64_t N, int64_t bs, float* means,
                             float* vars, int quirk, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  // one thread per channel for FC shapes (blockSize 1) and short blocks;
  // blocks of >= 64 use 8 lanes each (their chains are the reference's lanes)
  if (bs == 1 || (bs < 64 && groups * bs <= kSeqMax))
    hipLaunchKernelGGL(means_vars_seq, dim3(nblk(N)), dim3(TPB), 0, s, x, groups, N, bs, means,
                       vars, quirk);
  else
    hipLaunchKernelGGL(means_vars_lanes, dim3((unsigned)N), dim3(TPB), 0, s, x, groups, N, bs,
                       means, vars, quirk);
  return hipGetLastError();
}

hipError_t launch_normalize(float* x, int64_t groups, int64_t N, int64_t bs, const float* means,
                            int64_t mstride, const float* vars, int64_t vstride, hipStream_t s) {
  const int64_t total = groups * N * bs;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(normalize_k, dim3(nblk(total)), dim3(TPB), 0, s, x, total, N, bs, means,
                     mstride, vars, vstride);
  return hipGetLastError();
}

hipError_t launch_scale_add(float* x, int64_t groups, int64_t N, int64_t bs, const float* scales,
                            const float* biases, int64_t incb, hipStream_t s) {
  const int64_t total = groups * N * bs;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(scale_add_k, dim3(nblk(total)), dim3(TPB), 0, s, x, total, N, bs, scales,
                     biases, incb);
  return hipGetLastError();
}

hipError_t launch_add_dots(float* dst, const float* a, const float* b, int64_t groups, int64_t N,
                           int64_t bs, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  if (bs >= 64 && N <= 0x7fffffffLL)
    hipLaunchKernelGGL(add_dots_blocks, dim3((unsigned)N), dim3(TPB), 0, s, dst, a, b, groups, N,
                       bs);
  else
    hipLaunchKernelGGL(add_dots_seq, dim3(nblk(N)), dim3(TPB), 0, s, dst, a, b, groups, N, bs);
  return hipGetLastError();
}

hipError_t launch_add_sums(float* dst, const float* src, int64_t groups, int64_t N, int64_t bs,
                           hipStream_t s) {
  if (N <= 0) return hipSuccess;
  if (bs == 1 && N == 1)  // stride 1: sumv is vssum_avx2 over the groups
    return launch_backward_bias(dst, 1, src, groups, 1, 1, s);
  if (bs == 1) {
    hipLaunchKernelGGL(add_sums_seq, dim3(nblk(N)), dim3(TPB), 0, s, dst, src, groups, N);
    return hipGetLastError();
  }
  return launch_backward_bias(dst, N, src, bs, groups, 1, s);
}

hipError_t launch_mean_var_delta(const float* delta, const float* x, const float* mean,
                                 const float* var, int64_t groups, int64_t N, int64_t bs,
                                 float* mean_delta, float* var_delta, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  if (bs >= 64 && N <= 0x7fffffffLL)
    hipLaunchKernelGGL(mean_var_delta_blocks, dim3((unsigned)N), dim3(TPB), 0, s, delta, x, mean,
                       var, groups, N, bs, mean_delta, var_delta);
  else
    hipLaunchKernelGGL(mean_var_delta_seq, dim3(nblk(N)), dim3(TPB), 0, s, delta, x, mean, var,
                       groups, N, bs, mean_delta, var_delta);
  return hipGetLastError();
}

hipError_t launch_normalize_delta(const float* x, const float* mean, const float* var,
                                  const float* mean_delta, const float* var_delta, float* delta,
                                  int64_t groups, int64_t N, int64_t bs, hipStream_t s) {
  const int64_t total = groups * N * bs;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(normalize_delta_k, dim3(nblk(total)), dim3(TPB), 0, s, x, mean, var,
                     mean_delta, var_delta, delta, total, N, bs, (float)(groups * bs));
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
