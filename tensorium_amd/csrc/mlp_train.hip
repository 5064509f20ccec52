// mlp_train.hip — the connected-network train step (BASELINE config 5) as ONE
// fused HIP kernel: TNNet.Propagate (forward + backward) + TNNet.update for a
// stack of TConnectedLayer (nconnectedlayer.pas:157-359, optional batch norm)
// followed by TSoftmaxLayer (nsoftmaxlayer.pas:139-181), nnet.pas:275-450.
//
// The whole step is ~9 MFLOP at batch 32, far too small to fill 256 CUs and
// dominated by ~60 dependent stages; as separate launches it is launch-bound.
// Here one 1024-thread workgroup runs every stage back to back with
// workgroup barriers in between (all traffic stays in one CU's L1/L2 slice).
//
// Numerics mirror oracle/tns_oracle_train.c:
//  * forward gemm(NoTrans, Trans) = the reference's sdot_avx2 8-lane order:
//    each residue class k mod 8 is its own ascending f32-MFMA FMA chain, the
//    8 partial tiles are folded (l, l+4) then ((0+1)+(2+3)) — bit-exact;
//  * dW (TN) and dX (NN, beta = 1) are ascending-k FMA chains = f32 MFMA;
//  * per-channel BN / bias sums walk the reference's sequential order in one
//    thread; exp / ln / pow in double, rounded once.
#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int NT = 1024;
constexpr int NWAVES = NT / 64;
constexpr int KC = 128;  // largest k-chunk of the LDS-staged forward gemm

// Diagnostic build only (-DTNS_MLP_STAMPS, scripts/mlp_stamps.py): thread 0
// records s_memtime at stage boundaries into 64 uint32 pairs after the packed
// buffer (the caller allocates them).  Compiled out of the product.
#ifdef TNS_MLP_STAMPS
#define MLP_STAMP(i)                                                              \
  do {                                                                            \
    __syncthreads();                                                              \
    if (threadIdx.x == 0) {                                                       \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                 \
      unsigned* st_ = reinterpret_cast<unsigned*>(a.buf + a.stamp_off) + 2 * (i); \
      st_[0] = (unsigned)t_;                                                      \
      st_[1] = (unsigned)(t_ >> 32);                                              \
    }                                                                             \
  } while (0)
#else
#define MLP_STAMP(i) \
  do {               \
  } while (0)
#endif
__device__ constexpr float SEPS = 0.000001f;

// Per-layer views into the packed buffer.  The element offsets are computed
// on the host (MlpArgs::off) and read from the kernel arguments on each use,
// so no pointer set stays live in registers across the stages.
enum { F_W, F_B, F_DW, F_DB, F_SCALES, F_RMEAN, F_RVAR, F_DSCALES, F_OUT, F_DELTA, F_X, F_XNORM,
       F_MEAN, F_VAR, F_MDELTA, F_VDELTA };
struct Layer {
  const MlpArgs* a;
  int l;
  int64_t I, O;
  int act;
  __device__ Layer(const MlpArgs& args, int layer)
      : a(&args), l(layer), I(args.widths[layer]), O(args.widths[layer + 1]),
        act(args.acts[layer]) {}
  __device__ float* f(int which) const { return a->buf + a->off[l][which]; }
  __device__ float* W() const { return f(F_W); }
  __device__ float* b() const { return f(F_B); }
  __device__ float* dW() const { return f(F_DW); }
  __device__ float* db() const { return f(F_DB); }
  __device__ float* scales() const { return f(F_SCALES); }
  __device__ float* rmean() const { return f(F_RMEAN); }
  __device__ float* rvar() const { return f(F_RVAR); }
  __device__ float* dscales() const { return f(F_DSCALES); }
  __device__ float* out() const { return f(F_OUT); }
  __device__ float* delta() const { return f(F_DELTA); }
  __device__ float* x() const { return f(F_X); }
  __device__ float* xnorm() const { return f(F_XNORM); }
  __device__ float* mean() const { return f(F_MEAN); }
  __device__ float* var() const { return f(F_VAR); }
  __device__ float* mdelta() const { return f(F_MDELTA); }
  __device__ float* vdelta() const { return f(F_VDELTA); }
};

// One 32x32 MFMA output tile as an ascending chain: step s feeds lane
// (l31, h) the operands pa[s*sa] / pb[s*sb] for k = k0 + s*kstep (k0 already
// includes the lane half h); operands with k >= K or an out-of-range row
// (va / vb false) are 0.  Operands of U steps are loaded together (one memory
// latency per U steps), then consumed by U dependent MFMAs in step order.
template <int U = 8>
__device__ __forceinline__ void mfma_chain(floatx16& acc, int steps, const float* pa, int64_t sa,
                                           bool va, const float* pb, int64_t sb, bool vb,
                                           int64_t k0, int64_t kstep, int64_t K) {
  for (int s = 0; s < steps; s += U) {
    float av[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // the last batch may be partial: loads stay together
      const bool ok = (s + u < steps) && k0 + (int64_t)(s + u) * kstep < K;
      const int64_t ia = ok ? (int64_t)(s + u) * sa : 0, ib = ok ? (int64_t)(s + u) * sb : 0;
      const float x = pa[ia], y = pb[ib];
      av[u] = (ok && va) ? x : 0.0f;
      bv[u] = (ok && vb) ? y : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (s + u < steps) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
  }
}

// element (row, col) held by accumulator register e of this lane
__device__ __forceinline__ int acc_row(int e) {
  return (e & 3) + 8 * (e >> 2) + 4 * ((threadIdx.x & 63) >> 5);
}

__device__ __forceinline__ float vssum8(const float* a, int64_t n) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t blocks = n >> 3;
  for (int64_t t = 0; t < blocks; ++t)
    for (int l = 0; l < 8; ++l) acc[l] = acc[l] + a[8 * t + l];
  const float s0 = acc[0] + acc[4], s1 = acc[1] + acc[5], s2 = acc[2] + acc[6],
              s3 = acc[3] + acc[7];
  float r = (s0 + s1) + (s2 + s3);
  for (int64_t i = blocks * 8; i < n; ++i) r = r + a[i];
  return r;
}

// Forward gemm of one layer, out[B][O] partials per residue class r = k mod 8
// into lds[(r*B + m)*O + n], with wave w = (tile, r) and both operands staged
// through LDS in k-chunks of KCH by coalesced loads; each chain continues
// across chunks in ascending k (bit-identical to the direct chain).  The
// chunks alias the partial-sum region: every wave has passed the barrier
// after the last chunk before any partial is written.
template <int KCH>
__device__ __forceinline__ void gemm_chunked(float* lds, const float* in, const float* W, int64_t B,
                                             int64_t O, int64_t I, int tm, int tn) {
  constexpr int KP = KCH + 1;  // LDS row: an odd stride for the lanes' row reads
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  float* Xs = lds;
  float* Ws = Xs + tm * 32 * KP;
  const int rowsX = tm * 32, rows = (tm + tn) * 32;
  const bool active = wid < tm * tn * 8;
  const int r = wid & 7, tile = wid >> 3;
  const int m0 = (tile / tn) * 32, n0 = (tile % tn) * 32;
  const int l31 = lane & 31, h = lane >> 5;
  floatx16 acc;
  for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
  for (int64_t kc0 = 0; kc0 < I; kc0 += KCH) {
#pragma unroll 4
    for (int i = tid; i < rows * KCH; i += NT) {
      const int row = i / KCH, kk = i % KCH;
      const int64_t k = kc0 + kk;
      const bool isx = row < rowsX;
      const int64_t rr = isx ? row : row - rowsX;
      const bool ok = k < I && rr < (isx ? B : O);
      const float* src = isx ? in : W;
      const float v = src[ok ? rr * I + k : 0];
      lds[row * KP + kk] = ok ? v : 0.0f;
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int st = 0; st < KCH / 16; ++st) {  // k = kc0 + r + 8*(2*st + h)
        const int kk = r + 8 * (2 * st + h);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Xs[(m0 + l31) * KP + kk],
                                                   Ws[(n0 + l31) * KP + kk], acc, 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if (active)
    for (int e = 0; e < 16; ++e) {
      const int64_t m = m0 + acc_row(e), n = n0 + l31;
      if (m < B && n < O) lds[(r * B + m) * O + n] = acc[e];
    }
}

__global__ __launch_bounds__(NT) void mlp_train_kernel(MlpArgs a) {
  // 8 * B * O_max floats: partial sums of the forward gemm; between gemms,
  // up to three [B][O] blocks staged for the per-channel (column) passes, so
  // their sequential sums read LDS instead of waiting on memory per row
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  const int wid = tid >> 6;
  const int lane = tid & 63;
  const int64_t B = a.batch;
  const int L = a.nlayers;
  const int64_t C = a.widths[L];
  float* smx = a.buf + a.softmax_off;
  float* sm_out = smx;
  float* sm_delta = smx + B * C;
  float* sm_loss = smx + 2 * B * C;

  // ---- forward ------------------------------------------------------------
  MLP_STAMP(0);
  const float* in = a.X;
  for (int l = 0; l < L; ++l) {
    const Layer lay(a, l);
    const int64_t I = lay.I, O = lay.O, BO = B * O;
    for (int64_t e = tid; e < BO; e += NT) lay.delta()[e] = 0.0f;  // nnet.pas:287-296

    // gemm(RowMajor, NoTrans, Trans, B, O, I, 1, in, I, W, I, 0, out, O):
    // sdot_avx2 residue classes r = k mod 8, each an ascending MFMA chain
    const int tm = (int)((B + 31) / 32), tn = (int)((O + 31) / 32);
    const int64_t kr = (I + 7) / 8;            // k values per residue class
    const int steps = (int)((kr + 1) / 2);
    if (tm * tn * 8 <= NWAVES && a.lds_chunks) {
      // One (tile, residue) task per wave; both operands are k-contiguous
      // rows (an MFMA lane per row), so they are staged through LDS in
      // k-chunks by coalesced loads (gemm_chunked)
      if (I > 64)
        gemm_chunked<128>(lds, in, lay.W(), B, O, I, tm, tn);
      else
        gemm_chunked<64>(lds, in, lay.W(), B, O, I, tm, tn);
    } else
    for (int w = wid; w < tm * tn * 8; w += NWAVES) {
      const int r = w & 7, tile = w >> 3;
      const int64_t m0 = (int64_t)(tile / tn) * 32, n0 = (int64_t)(tile % tn) * 32;
      floatx16 acc;
      for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
      {
        const int l31 = lane & 31, h = lane >> 5;
        const int64_t m = m0 + l31, n = n0 + l31, k0 = r + 8 * h;
        // step s consumes k = r + 8*(2s + h) of residue class r
        mfma_chain(acc, steps, in + (m < B ? m : 0) * I + k0, 16, m < B,
                   lay.W() + (n < O ? n : 0) * I + k0, 16, n < O, k0, 16, I);
      }
      for (int e = 0; e < 16; ++e) {
        const int64_t m = m0 + acc_row(e), n = n0 + (lane & 31);
        if (m < B && n < O) lds[(r * B + m) * O + n] = acc[e];
      }
    }
    __syncthreads();
    for (int64_t e = tid; e < BO; e += NT) {
      float p[8];
      for (int q = 0; q < 8; ++q) p[q] = lds[q * BO + e];
      const float s0 = p[0] + p[4], s1 = p[1] + p[5], s2 = p[2] + p[6], s3 = p[3] + p[7];
      const float dot = (s0 + s1) + (s2 + s3);
      const float c0 = 0.0f * lay.out()[e];  // beta = 0 => 0*C (mulvs)
      const float y = c0 + 1.0f * dot;       // C := C + ALPHA*sdot
      lay.out()[e] = y;
      lds[e] = y;  // (this thread's own partial slot, already read)
    }
    __syncthreads();
    if (a.bn) {
      // per channel: MeansAndVars, rolling stats, x, normalize, x_norm, scale
      const float* col = lds;  // the layer output, [B][O]
      for (int64_t o = tid; o < O; o += NT) {
        // this channel's parameters, all loaded before any store: one memory
        // round trip instead of one per use
        const float rm0 = lay.rmean()[o], rv0 = lay.rvar()[o], sc = lay.scales()[o];
        float m = 0.0f;
#pragma unroll 8
        for (int64_t b = 0; b < B; ++b) m = m + col[b * O + o];
        m = m / (float)B;
        float v = 0.0f;
#pragma unroll 8
        for (int64_t b = 0; b < B; ++b) {
          const float t = col[b * O + o] - m;
          v = v + t * t;
        }
        v = v / (float)(B - 1);
        lay.mean()[o] = m;
        lay.var()[o] = v;
        const float mom = 0.05f;  // bnMomentum, nconnectedlayer.pas:67
        lay.rmean()[o] = fmaf(mom, m, rm0 * (1.0f - mom));
        lay.rvar()[o] = fmaf(mom, v, rv0 * (1.0f - mom));
        const float sd = sqrtf(v > SEPS ? v : SEPS);
#pragma unroll 8
        for (int64_t b = 0; b < B; ++b) {
          const float xv = col[b * O + o];
          lay.x()[b * O + o] = xv;
          const float xn = (xv - m) / sd;
          lay.xnorm()[b * O + o] = xn;
          lay.out()[b * O + o] = xn * sc;
        }
      }
      __syncthreads();
    }
    for (int64_t e = tid; e < BO; e += NT) {
      const int64_t o = e % O;
      lay.out()[e] = act_apply(lay.out()[e] + lay.b()[o], lay.act);  // forwardBias, activate
    }
    __syncthreads();
    in = lay.out();
    MLP_STAMP(1 + l);
  }

  // ---- softmax + cross-entropy (groups 1, temperature 1) ----------------------
  for (int64_t b = tid; b < B; b += NT) {
    const float* ip = in + b * C;
    float* op = sm_out + b * C;
    float largest = ip[0];
    for (int64_t i = 1; i < C; ++i)
      if (ip[i] > largest) largest = ip[i];
    float sum = 0.0f;
    for (int64_t i = 0; i < C; ++i) {
      const float e = (float)exp((double)((ip[i] - largest) / 1.0f));
      sum = sum + e;
      op[i] = e;
    }
    for (int64_t i = 0; i < C; ++i) op[i] = op[i] / sum;
  }
  __syncthreads();
  for (int64_t i = tid; i < B * C; i += NT) {
    const float t = a.truth[i], p = sm_out[i];
    sm_loss[i] = t != 0.0f ? (float)(-log((double)(p > SEPS ? p : SEPS))) : 0.0f;
    sm_delta[i] = t - p;
  }
  __syncthreads();
  if (tid == 0) *a.cost = vssum8(sm_loss, B * C);
  MLP_STAMP(20);

  // ---- backward ---------------------------------------------------------------
  for (int l = L - 1; l >= 0; --l) {
    const Layer lay(a, l);
    const int64_t I = lay.I, O = lay.O, BO = B * O;
    const float* lin = a.X;
    float* prev_delta = nullptr;
    if (l > 0) {
      const Layer prev(a, l - 1);
      lin = prev.out();
      prev_delta = prev.delta();  // state.delta = nil for layer 0 (nnet.pas:332-335)
    }
    // softmax backward: prev.delta() += delta; then clamp + activation gradient.
    // Stage delta (and x, x_norm for batch norm) in LDS for the column passes.
    float* sdel = lds;
    float* sx = lds + BO;
    float* sxn = lds + 2 * BO;
    for (int64_t e = tid; e < BO; e += NT) {
      float d = lay.delta()[e];
      if (l == L - 1) d = d + sm_delta[e];
      d = d < -1.0f ? -1.0f : (d > 1.0f ? 1.0f : d);  // delta.Clamp(-1, 1)
      d = d * grad_apply(lay.out()[e], lay.act);
      lay.delta()[e] = d;
      sdel[e] = d;
      if (a.bn) {
        sx[e] = lay.x()[e];
        sxn[e] = lay.xnorm()[e];
      }
    }
    __syncthreads();
    MLP_STAMP(50 + 2 * l);
    // per channel: bias_updates.addSums, then the BN backward chain
    for (int64_t o = tid; o < O; o += NT) {
      // this channel's parameters, all loaded before any store (one memory
      // round trip instead of one per use)
      const float db0 = lay.db()[o];
      float ds0 = 0.0f, sc = 0.0f, mu = 0.0f, var = 0.0f;
      if (a.bn) {
        ds0 = lay.dscales()[o];
        sc = lay.scales()[o];
        mu = lay.mean()[o];
        var = lay.var()[o];
      }
      float r = 0.0f;
#pragma unroll 8
      for (int64_t b = 0; b < B; ++b) r = r + sdel[b * O + o];
      lay.db()[o] = db0 + r;
      if (a.bn) {
        float dd = 0.0f;  // addDots (strided sdot: mul then add)
#pragma unroll 8
        for (int64_t b = 0; b < B; ++b) dd = dd + sxn[b * O + o] * sdel[b * O + o];
        lay.dscales()[o] = ds0 + dd;
        float m = 0.0f, v = 0.0f;
#pragma unroll 8
        for (int64_t b = 0; b < B; ++b) {
          const float d = sdel[b * O + o] * sc;  // forwardScale
          sdel[b * O + o] = d;                   // (own column only)
          m = m + d;
          v = v + (sx[b * O + o] - mu) * d;
        }
        const float ve = var > SEPS ? var : SEPS;
        const float md = m * (-1.0f / sqrtf(ve));
        const float vd = (float)((double)v * -0.5 * pow((double)ve, -1.5));
        lay.mdelta()[o] = md;
        lay.vdelta()[o] = vd;
        const float mdb = md / (float)B, vdb = 2.0f * vd / (float)B, sd = sqrtf(ve);
#pragma unroll 8
        for (int64_t b = 0; b < B; ++b) {
          const float q = sdel[b * O + o] / sd;
          const float t = (sx[b * O + o] - mu) * vdb + mdb;
          lay.delta()[b * O + o] = q + t;
        }
      }
    }
    __syncthreads();
    MLP_STAMP(51 + 2 * l);
    // dW += delta^T . in   (TN: M=O, N=I, K=B, beta 1)   and
    // prev_delta += delta . W (NN: M=B, N=I, K=O, beta 1), both ascending chains
    const int tmo = (int)((O + 31) / 32), tni = (int)((I + 31) / 32), tmb = (int)((B + 31) / 32);
    const int nw_dw = tmo * tni, nw_dx = prev_delta ? tmb * tni : 0;
    for (int w = wid; w < nw_dw + nw_dx; w += NWAVES) {
      floatx16 acc;
      const bool is_dw = w < nw_dw;
      const int t = is_dw ? w : w - nw_dw;
      const int64_t m0 = (int64_t)(t / tni) * 32, n0 = (int64_t)(t % tni) * 32;
      const int64_t Mx = is_dw ? O : B;
      float* Cp = is_dw ? lay.dW() : prev_delta;
      for (int e = 0; e < 16; ++e) {
        const int64_t m = m0 + acc_row(e), n = n0 + (lane & 31);
        acc[e] = (m < Mx && n < I) ? Cp[m * I + n] : 0.0f;
      }
      const int l31 = lane & 31, h = lane >> 5;
      const int64_t m = m0 + l31, n = n0 + l31, nc = n < I ? n : 0;
      if (is_dw) {  // a = delta[k][m], b = in[k][n], k = 2s + h over the batch
        const int64_t mc = m < O ? m : 0;
        mfma_chain(acc, (int)((B + 1) / 2), lay.delta() + h * O + mc, 2 * O, m < O,
                   lin + h * I + nc, 2 * I, n < I, h, 2, B);
      } else {      // a = delta[m][k], b = W[k][n], k = 2s + h over the outputs
        const int64_t mc = m < B ? m : 0;
        mfma_chain(acc, (int)((O + 1) / 2), lay.delta() + mc * O + h, 2, m < B,
                   lay.W() + h * I + nc, 2 * I, n < I, h, 2, O);
      }
      for (int e = 0; e < 16; ++e) {
        const int64_t m = m0 + acc_row(e), n = n0 + (lane & 31);
        if (m < Mx && n < I) Cp[m * I + n] = acc[e];
      }
    }
    __syncthreads();
    MLP_STAMP(21 + l);
  }

  // ---- update (TConnectedLayer.update, constant learning rate) ----------------
  const float lrb = a.lr / (float)B;
  const float wdec = -a.decay * (float)B;
  for (int l = 0; l < L; ++l) {
    const Layer lay(a, l);
    const int64_t O = lay.O, IO = lay.I * lay.O;
    for (int64_t o = tid; o < O; o += NT) {
      lay.b()[o] = fmaf(lrb, lay.db()[o], lay.b()[o]);
      lay.db()[o] = a.momentum * lay.db()[o];
      if (a.bn) {
        lay.scales()[o] = fmaf(lrb, lay.dscales()[o], lay.scales()[o]);
        lay.dscales()[o] = a.momentum * lay.dscales()[o];
      }
    }
    // UB elements per thread per round, their loads issued together (W and dW
    // live in one buffer: the compiler cannot move a load past a store)
    constexpr int UB = 8;
    float* W = lay.W();
    float* dW = lay.dW();
    for (int64_t e0 = tid; e0 < IO; e0 += (int64_t)NT * UB) {
      float w[UB], g[UB];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int64_t e = e0 + (int64_t)u * NT;
        w[u] = W[e < IO ? e : e0];
        g[u] = dW[e < IO ? e : e0];
      }
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int64_t e = e0 + (int64_t)u * NT;
        if (e < IO) {
          const float dw = fmaf(wdec, w[u], g[u]);  // weight_updates.axpy(-decay*batch, W)
          W[e] = fmaf(lrb, dw, w[u]);               // weights.axpy(lr/batch, dW)
          dW[e] = a.momentum * dw;                  // weight_updates.Multiply(momentum)
        }
      }
    }
    MLP_STAMP(40 + l);
  }
}

}  // namespace

int64_t mlp_buffer_floats(int nlayers, const int64_t* widths, int bn, int64_t B) {
  int64_t n = 0;
  for (int l = 0; l < nlayers; ++l) {
    const int64_t I = widths[l], O = widths[l + 1];
    n += 2 * I * O + 2 * O + 2 * B * O;
    if (bn) n += 4 * O + 2 * B * O + 4 * O;
  }
  return n + 3 * B * widths[nlayers];
}

hipError_t launch_mlp_train_step(const MlpArgs& args, hipStream_t s) {
  if (args.nlayers < 1 || args.nlayers > MLP_MAX_LAYERS) return hipErrorInvalidValue;
  MlpArgs a = args;
  int64_t p = 0;
  const int64_t B = a.batch;
  for (int l = 0; l < a.nlayers; ++l) {  // packed layout of ora_mlp_train_step
    const int64_t I = a.widths[l], O = a.widths[l + 1], IO = I * O, BO = B * O;
    int64_t* o = a.off[l];
    for (int f = 0; f < 16; ++f) o[f] = 0;
    o[F_W] = p; p += IO;
    o[F_B] = p; p += O;
    o[F_DW] = p; p += IO;
    o[F_DB] = p; p += O;
    if (a.bn) {
      o[F_SCALES] = p; p += O;
      o[F_RMEAN] = p; p += O;
      o[F_RVAR] = p; p += O;
      o[F_DSCALES] = p; p += O;
    }
    o[F_OUT] = p; p += BO;
    o[F_DELTA] = p; p += BO;
    if (a.bn) {
      o[F_X] = p; p += BO;
      o[F_XNORM] = p; p += BO;
      o[F_MEAN] = p; p += O;
      o[F_VAR] = p; p += O;
      o[F_MDELTA] = p; p += O;
      o[F_VDELTA] = p; p += O;
    }
  }
  a.softmax_off = p;
  a.stamp_off = p + 3 * B * a.widths[a.nlayers];
  int64_t omax = 0;
  for (int l = 0; l < a.nlayers; ++l) omax = a.widths[l + 1] > omax ? a.widths[l + 1] : omax;
  // partial sums (>= 3 [B][O] blocks); the forward gemm's k-chunks of both
  // operands reuse the same space when one (tile, residue) task per wave
  // covers every layer
  const int64_t tmx = (a.batch + 31) / 32, tnx = (omax + 31) / 32;
  size_t lds = (size_t)(8 * a.batch * omax) * sizeof(float);
  const size_t lds_chunks = (size_t)((tmx + tnx) * 32 * (KC + 1)) * sizeof(float);
  a.lds_chunks = tmx * tnx * 8 <= NWAVES && lds_chunks <= 160 * 1024;
  if (a.lds_chunks && lds_chunks > lds) lds = lds_chunks;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_train_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(mlp_train_kernel, dim3(1), dim3(NT), lds, s, a);
  return hipGetLastError();
}

}  // namespace tns
