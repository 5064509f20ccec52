// mlp_train.hip — the connected-network train step (BASELINE config 5) as ONE
// fused HIP kernel: TNNet.Propagate (forward + backward) + TNNet.update for a
// stack of TConnectedLayer (nconnectedlayer.pas:157-359, optional batch norm)
// followed by TSoftmaxLayer (nsoftmaxlayer.pas:139-181), nnet.pas:275-450.
//
// The whole step is ~9 MFLOP at batch 32, far too small to fill 256 CUs and
// dominated by dependent stages; as separate launches it is launch-bound.
// Here one 1024-thread workgroup runs every stage back to back with
// workgroup barriers in between (all traffic stays in one CU's L1/L2 slice),
// laid out for latency: the per-channel sequential sums are the only
// single-thread chains (the element-wise parts of BN, softmax and the update
// run on all 1024 threads), every stage issues its loads together, operands
// the next stage needs stay in LDS or registers, and the weight update of
// layer 0 is applied in its dW epilogue.
//
// Numerics mirror oracle/tns_oracle_train.c:
//  * forward gemm(NoTrans, Trans) = the reference's sdot_avx2 8-lane order:
//    each residue class k mod 8 is its own ascending f32-MFMA FMA chain, the
//    8 partial tiles are folded (l, l+4) then ((0+1)+(2+3)) — bit-exact;
//  * dW (TN) and dX (NN, beta = 1) are ascending-k FMA chains = f32 MFMA;
//  * per-channel BN / bias sums walk the reference's sequential order in one
//    thread; exp / ln / pow in double, rounded once;
//  * the cost is vssum_avx2's 8 lane chains (one lane each) and its fold.
#include "tns_act.hpp"
#include "tns_internal.hpp"

namespace tns {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
#ifndef TNS_MLP_NT
#define TNS_MLP_NT 1024
#endif
constexpr int NT = TNS_MLP_NT;  // (512: diagnostic builds, 256 VGPRs per thread)
constexpr int NWAVES = NT / 64;
// element slots per thread of the [B][O] passes: the two kernel instances
constexpr int EPT_S = 2048 / NT, EPT_L = 5120 / NT;
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
// MLP_MARK: thread 0's clock without a barrier (wave 0's own timeline)
#define MLP_MARK(i)                                                               \
  do {                                                                            \
    if (threadIdx.x == 0) {                                                       \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                 \
      unsigned* st_ = reinterpret_cast<unsigned*>(a.buf + a.stamp_off) + 2 * (64 + (i)); \
      st_[0] = (unsigned)t_;                                                      \
      st_[1] = (unsigned)(t_ >> 32);                                              \
    }                                                                             \
  } while (0)
#else
#define MLP_STAMP(i) \
  do {               \
  } while (0)
#define MLP_MARK(i) \
  do {              \
  } while (0)
#endif
__device__ constexpr float SEPS = 0.000001f;

// Workgroup barrier for LDS traffic only: waits for this wave's LDS
// operations, not for its global loads (prefetches stay in flight across it)
// or stores (nothing after it reads them from memory).  __syncthreads()
// drains every memory counter, so it is kept only where another thread reads
// global data written before it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Column blocks for the per-channel sequential sums: 8 LDS reads of rows
// b0..b0+7 (clamped to the last row; the caller skips the extra terms),
// issued back to back and held by one empty asm, so a chain waits once per
// block instead of once per term (hipcc otherwise placed each read right
// before the add that consumes it, with an lgkmcnt(0) wait each time).
__device__ __forceinline__ void col8(float (&v)[8], const float* col, int b0, int B, int stride) {
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = col[(b0 + u < B ? b0 + u : B - 1) * stride];
}
__device__ __forceinline__ void hold8(float (&v)[8]) {
  asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]),
               "+v"(v[6]), "+v"(v[7]));
}

// Per-layer views into the packed buffer.  The element offsets are computed
// on the host (MlpArgs::off) and read from the kernel arguments on each use,
// so no pointer set stays live in registers across the stages.
enum { F_W, F_B, F_DW, F_DB, F_SCALES, F_RMEAN, F_RVAR, F_DSCALES, F_OUT, F_DELTA, F_X, F_XNORM,
       F_MEAN, F_VAR, F_MDELTA, F_VDELTA };
struct Layer {
  const MlpArgs* a;
  int l;
  int I, O;
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
__device__ __forceinline__ void mfma_chain(floatx16& acc, int steps, const float* pa, int sa,
                                           bool va, const float* pb, int sb, bool vb,
                                           int k0, int kstep, int K) {
  for (int s = 0; s < steps; s += U) {
    float av[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // the last batch may be partial: loads stay together
      const bool ok = (s + u < steps) && k0 + (int)(s + u) * kstep < K;
      const int ia = ok ? (int)(s + u) * sa : 0, ib = ok ? (int)(s + u) * sb : 0;
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
__device__ __forceinline__ int acc_row(int e, int lane) {
  return (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
}

// threadIdx.x behind an empty asm: values derived from it are recomputed in
// each stage instead of being hoisted out of the layer loops as invariants
// (at 1024 threads a thread has 128 VGPRs, and the hoisted addresses of
// every stage spilled to scratch)
__device__ __forceinline__ int stage_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// Element slots per thread in the [B][O] passes (kernel template argument):
// 2 when B*max(O) <= 2048 (the MNIST net), else 5 (B*O <= 40960/8).

// Forward gemm of one layer, out[B][O] partials per residue class r = k mod 8
// into lds[(r*B + m)*O + n], with wave w = (tile, r) and both operands staged
// through LDS in k-chunks of KCH by coalesced loads; each chain continues
// across chunks in ascending k (bit-identical to the direct chain).  With
// 16-byte rows the chunks are loaded as float4, two chunks ahead into
// registers, so a chunk's global latency overlaps the MFMAs of the previous
// two.  The chunks alias the partial-sum region: every wave has passed the
// barrier after the last chunk before any partial is written.
// gmark: diagnostic stamps (wave 0's clock at its sub-steps; nullptr in the
// product, folded away)
__device__ __forceinline__ void gmark(unsigned* st, int i) {
  if (st && threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    st[2 * i] = (unsigned)t;
    st[2 * i + 1] = (unsigned)(t >> 32);
  }
}
template <int KCH>
__device__ __forceinline__ void gemm_chunked(float* lds, const float* in, const float* W, int B,
                                             int O, int I, int tm, int tn, int tid,
                                             unsigned* st = nullptr) {
  constexpr int KP = KCH + 1;  // LDS row: an odd stride for the lanes' row reads
  constexpr int QR = KCH / 4;  // float4 units per staged row
  constexpr int UV = (3 * 32 * QR + NT - 1) / NT;  // units per thread (tm + tn <= 3)
  const int wid = tid >> 6, lane = tid & 63;
  float* Xs = lds;
  float* Ws = Xs + tm * 32 * KP;
  const int rowsX = tm * 32, rows = (tm + tn) * 32;
  const bool active = wid < tm * tn * 8;
  const int r = wid & 7, tile = wid >> 3;
  const int m0 = (tile / tn) * 32, n0 = (tile % tn) * 32;
  const int l31 = lane & 31, h = lane >> 5;
  floatx16 acc;
  for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
  auto compute = [&]() {
    if (active) {
#pragma unroll
      for (int st = 0; st < KCH / 16; ++st) {  // k = kc0 + r + 8*(2*st + h)
        const int kk = r + 8 * (2 * st + h);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Xs[(m0 + l31) * KP + kk],
                                                   Ws[(n0 + l31) * KP + kk], acc, 0, 0, 0);
      }
    }
  };
  const bool vec = (I & 3) == 0 && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(W)) & 15) == 0;
  const int nch = (I + KCH - 1) / KCH;
  if (vec) {
    const int units = rows * QR;
    auto load = [&](int kc0, float4 (&v)[UV]) {
#pragma unroll
      for (int u = 0; u < UV; ++u) {
        const int idx = tid + u * NT;
        const int row = idx / QR, kq = idx % QR;
        const int k = kc0 + 4 * kq;
        const bool isx = row < rowsX;
        const int rr = isx ? row : row - rowsX;
        const bool ok = idx < units && k < I && rr < (isx ? B : O);
        const float* src = isx ? in : W;
        const float4 x = *reinterpret_cast<const float4*>(src + (ok ? rr * I + k : 0));
        v[u] = ok ? x : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      }
    };
    auto store = [&](const float4 (&v)[UV]) {
#pragma unroll
      for (int u = 0; u < UV; ++u) {
        const int idx = tid + u * NT;
        if (idx < units) {
          float* d = lds + (idx / QR) * KP + 4 * (idx % QR);
          d[0] = v[u].x; d[1] = v[u].y; d[2] = v[u].z; d[3] = v[u].w;
        }
      }
    };
    float4 r0[UV], r1[UV];
    gmark(st, 20);
    load(0, r0);
    if (nch > 1) load(KCH, r1);
    gmark(st, 21);
    for (int c = 0; c < nch; c += 2) {
      store(r0);
      gmark(st, 22);
      lds_barrier();
      gmark(st, 23);
      if (c + 2 < nch) load((c + 2) * KCH, r0);
      compute();
      gmark(st, 24);
      lds_barrier();
      gmark(st, 25);
      if (c + 1 < nch) {
        store(r1);
        lds_barrier();
        if (c + 3 < nch) load((c + 3) * KCH, r1);
        compute();
        lds_barrier();
      }
    }
  } else {
    for (int kc0 = 0; kc0 < I; kc0 += KCH) {
#pragma unroll 4
      for (int i = tid; i < rows * KCH; i += NT) {
        const int row = i / KCH, kk = i % KCH;
        const int k = kc0 + kk;
        const bool isx = row < rowsX;
        const int rr = isx ? row : row - rowsX;
        const bool ok = k < I && rr < (isx ? B : O);
        const float* src = isx ? in : W;
        const float v = src[ok ? rr * I + k : 0];
        lds[row * KP + kk] = ok ? v : 0.0f;
      }
      lds_barrier();
      compute();
      lds_barrier();
    }
  }
  if (active)
    for (int e = 0; e < 16; ++e) {
      const int m = m0 + acc_row(e, lane), n = n0 + l31;
      if (m < B && n < O) lds[(r * B + m) * O + n] = acc[e];
    }  gmark(st, 26);
}

// Backward gemm tasks of one wave (32x32 output tiles, ascending FMA chains
// over k, the loads of 16 steps issued together).  delta is read from its
// LDS copy sdel[B][O].
//  * dW tile (TN: dW += delta^T . in, k over the batch): acc starts from the
//    stored dW; with `upd` the tile's weights are loaded alongside (wv) for
//    TConnectedLayer.update, which the caller applies once no dX task of the
//    layer reads W any more;
//  * dX tile (NN: prev_delta += delta . W, k over the outputs): prev_delta
//    is the forward pass's zeroed delta, so the chain starts from +0; the
//    result goes to memory and to the LDS block `nxt` the next stage reads.
template <int U = 8>  // steps whose loads are issued together
__device__ __forceinline__ void dw_task(const float* sdel, int m0, int n0, int B,
                                        int O, int I, const float* lin, const float* dW,
                                        const float* W, bool upd, floatx16& acc, float (&wv)[16],
                                        int lane) {
  const int l31 = lane & 31, h = lane >> 5;
  for (int e = 0; e < 16; ++e) {
    const int m = m0 + acc_row(e, lane), n = n0 + l31;
    const bool ok = m < O && n < I;
    const int ix = ok ? m * I + n : 0;
    const float c = dW[ix];
    acc[e] = ok ? c : 0.0f;
    wv[e] = upd ? W[ix] : 0.0f;
  }
  const int m = m0 + l31, n = n0 + l31;
  const bool vm = m < O, vn = n < I;
  const int mc = vm ? m : 0, nc = vn ? n : 0;
  const int steps = (int)((B + 1) / 2);
  for (int s = 0; s < steps; s += U) {
    float av[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = 2 * (int)(s + u) + h;
      const bool ok = s + u < steps && k < B;
      const int kc = ok ? k : 0;
      const float x = sdel[kc * O + mc], y = lin[kc * I + nc];
      av[u] = (ok && vm) ? x : 0.0f;
      bv[u] = (ok && vn) ? y : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (s + u < steps) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
  }
}

// weight update of one dW tile (ora_sgd_update's weight part) or its plain store
__device__ __forceinline__ void dw_store(int m0, int n0, int O, int I, float* dW,
                                         float* W, bool upd, const floatx16& acc,
                                         const float (&wv)[16], float lrb, float wdec,
                                         float momentum, int lane) {
  const int l31 = lane & 31;
  for (int e = 0; e < 16; ++e) {
    const int m = m0 + acc_row(e, lane), n = n0 + l31;
    if (m < O && n < I) {
      if (upd) {
        const float dw = fmaf(wdec, wv[e], acc[e]);  // weight_updates.axpy(-decay*batch, W)
        W[m * I + n] = fmaf(lrb, dw, wv[e]);          // weights.axpy(lr/batch, dW)
        dW[m * I + n] = momentum * dw;                // weight_updates.Multiply(momentum)
      } else {
        dW[m * I + n] = acc[e];
      }
    }
  }
}

__device__ __forceinline__ void dx_task(const float* sdel, int m0, int n0, int B,
                                        int O, int I, const float* W, float* prev,
                                        float* nxt, int lane) {
  const int l31 = lane & 31, h = lane >> 5;
  floatx16 acc;
  for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
  const int m = m0 + l31, n = n0 + l31;
  const bool vm = m < B, vn = n < I;
  const int mc = vm ? m : 0, nc = vn ? n : 0;
  const int steps = (int)((O + 1) / 2);
  constexpr int U = 8;
  for (int s = 0; s < steps; s += U) {
    float av[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = 2 * (int)(s + u) + h;
      const bool ok = s + u < steps && k < O;
      const int kc = ok ? k : 0;
      const float x = sdel[mc * O + kc], y = W[kc * I + nc];
      av[u] = (ok && vm) ? x : 0.0f;
      bv[u] = (ok && vn) ? y : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (s + u < steps) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
  }
  for (int e = 0; e < 16; ++e) {
    const int mm = m0 + acc_row(e, lane), nn = n0 + l31;
    if (mm < B && nn < I) {
      prev[mm * I + nn] = acc[e];
      nxt[mm * I + nn] = acc[e];
    }
  }
}

// every layer's dW/dX tasks fit one per wave: the weight update of layer l
// is applied by its dW waves right after the stage's dX tasks are done
__device__ __forceinline__ bool defer_update(int B, int O, int I) {
  const int tmo = (O + 31) / 32, tni = (I + 31) / 32, tmb = (B + 31) / 32;
  return tmo * tni + tmb * tni <= NWAVES;
}

template <int EPT>
__global__ __launch_bounds__(NT) void mlp_train_kernel(MlpArgs a) {
  // [0, act_off): partial sums of the forward gemm (8 * B * O_max) or its
  // staged k-chunks; between gemms the [B][O] blocks and per-channel
  // statistics of the column passes.  [act_off, + B * max width): the block
  // handed from one stage to the next (forward activations, then the softmax
  // delta and each dX result), so no stage reads another thread's output
  // back from memory.
  extern __shared__ float lds[];
  float* act = lds + a.act_off;
  const int B = a.batch;
  const int L = a.nlayers;
  const int C = a.widths[L];
  const int Bi = (int)B, Ci = (int)C;  // LDS-resident sizes: 9*B*max(O) <= 40960
  float* smx = a.buf + a.softmax_off;
  float* sm_out = smx;
  float* sm_delta = smx + B * C;
  float* sm_loss = smx + 2 * B * C;
  const float lrb = a.lr / (float)B;
  const float wdec = -a.decay * (float)B;
  const float mom = a.momentum;

  // ---- forward ------------------------------------------------------------
  MLP_STAMP(0);
  const float* in = a.X;
  for (int l = 0; l < L; ++l) {
    const int tid = stage_tid(), wid = tid >> 6, lane = tid & 63;
    const Layer lay(a, l);
    const int I = lay.I, O = lay.O, BO = B * O;
    const int Oi = (int)O;
    float* out = lay.out();
    // ahead of the gemm: per element slot the stored C (beta = 0 still reads
    // it: 0*C), bias and BN scale; per channel (first slot) the rolling
    // statistics; delta zeroed (nnet.pas:287-296)
    float pc[EPT], pb[EPT], ps[EPT], yv[EPT];
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * NT;
      pc[q] = pb[q] = ps[q] = yv[q] = 0.0f;
      if (e < BO) {
        const int o = e % Oi;
        pc[q] = out[e];
        pb[q] = lay.b()[o];
        if (a.bn) ps[q] = lay.scales()[o];
        lay.delta()[e] = 0.0f;
      }
    }
    if (l == 1) MLP_MARK(0);
    float rm_pre = 0.0f, rv_pre = 0.0f;
    if (a.bn && tid < Oi) {
      rm_pre = lay.rmean()[tid];
      rv_pre = lay.rvar()[tid];
    }

    // gemm(RowMajor, NoTrans, Trans, B, O, I, 1, in, I, W, I, 0, out, O):
    // sdot_avx2 residue classes r = k mod 8, each an ascending MFMA chain
    const int tm = (int)((B + 31) / 32), tn = (int)((O + 31) / 32);
    const int kr = (I + 7) / 8;            // k values per residue class
    const int steps = (int)((kr + 1) / 2);
    if (l == 0) {
      // layer 0's partials come from mlp_l0_forward_kernel, in this layout
      if ((BO & 1) == 0) {  // 8*B*O floats = 2*B*O float4
        const float4* src = reinterpret_cast<const float4*>(a.l0part);
        for (int i = tid; i < (int)(2 * BO); i += NT) reinterpret_cast<float4*>(lds)[i] = src[i];
      } else {
        for (int i = tid; i < (int)(8 * BO); i += NT) lds[i] = a.l0part[i];
      }
    } else if (tm * tn * 8 <= NWAVES && a.lds_chunks) {
#ifdef TNS_MLP_STAMPS
      unsigned* gst = l == 1 ? reinterpret_cast<unsigned*>(a.buf + a.stamp_off) + 128 : nullptr;
#else
      unsigned* gst = nullptr;
#endif
      if (I > 64)
        gemm_chunked<128>(lds, in, lay.W(), B, O, I, tm, tn, tid, gst);
      else
        gemm_chunked<64>(lds, in, lay.W(), B, O, I, tm, tn, tid, gst);
    } else
    for (int w = wid; w < tm * tn * 8; w += NWAVES) {
      const int r = w & 7, tile = w >> 3;
      const int m0 = (int)(tile / tn) * 32, n0 = (int)(tile % tn) * 32;
      floatx16 acc;
      for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
      {
        const int l31 = lane & 31, h = lane >> 5;
        const int m = m0 + l31, n = n0 + l31, k0 = r + 8 * h;
        // step s consumes k = r + 8*(2s + h) of residue class r
        mfma_chain(acc, steps, in + (m < B ? m : 0) * I + k0, 16, m < B,
                   lay.W() + (n < O ? n : 0) * I + k0, 16, n < O, k0, 16, I);
      }
      for (int e = 0; e < 16; ++e) {
        const int m = m0 + acc_row(e, lane), n = n0 + (lane & 31);
        if (m < B && n < O) lds[(r * B + m) * O + n] = acc[e];
      }
    }
    if (l == 1) MLP_MARK(1);
    lds_barrier();
    if (l == 1) MLP_MARK(2);
    // fold the 8 residue partials (vextractf128 / vhaddps order), C := 0*C +
    // 1*sdot; without BN the bias and activation follow in the same pass
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * NT;
      if (e < BO) {
        float p[8];
        for (int j = 0; j < 8; ++j) p[j] = lds[j * BO + e];
        const float s0 = p[0] + p[4], s1 = p[1] + p[5], s2 = p[2] + p[6], s3 = p[3] + p[7];
        const float dot = (s0 + s1) + (s2 + s3);
        const float y = 0.0f * pc[q] + 1.0f * dot;  // beta = 0 => 0*C (mulvs); C + ALPHA*sdot
        if (a.bn) {
          yv[q] = y;
          lay.x()[e] = y;  // x := out before normalize
          lds[e] = y;      // (this thread's own partial slot, already read)
        } else {
          const float z = act_apply(y + pb[q], lay.act);  // forwardBias, activate
          out[e] = z;
          act[e] = z;
        }
      }
    }
    if (l == 1) MLP_MARK(3);
    if (a.bn) {
      lds_barrier();
      if (l == 1) MLP_MARK(4);
      // per channel: MeansAndVars (sequential over the batch), rolling stats;
      // mean and sd to LDS for the element pass
      float* st_m = lds + BO;
      float* st_sd = lds + BO + O;
      auto chain = [&](int o, float rm0, float rv0) {
        float m = 0.0f;
        for (int b0 = 0; b0 < Bi; b0 += 8) {
          float c[8];
          col8(c, lds + o, b0, Bi, Oi);
          hold8(c);
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (b0 + u < Bi) m = m + c[u];
        }
        m = m / (float)B;
        float v = 0.0f;
        for (int b0 = 0; b0 < Bi; b0 += 8) {
          float c[8];
          col8(c, lds + o, b0, Bi, Oi);
          hold8(c);
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (b0 + u < Bi) {
              const float t = c[u] - m;
              v = v + t * t;
            }
        }
        v = v / (float)(B - 1);
        lay.mean()[o] = m;
        lay.var()[o] = v;
        const float bmom = 0.05f;  // bnMomentum, nconnectedlayer.pas:67
        lay.rmean()[o] = fmaf(bmom, m, rm0 * (1.0f - bmom));
        lay.rvar()[o] = fmaf(bmom, v, rv0 * (1.0f - bmom));
        st_m[o] = m;
        st_sd[o] = sqrtf(v > SEPS ? v : SEPS);
      };
      if (tid < Oi) chain(tid, rm_pre, rv_pre);  // statistics prefetched
      for (int o = tid + NT; o < Oi; o += NT) chain(o, lay.rmean()[o], lay.rvar()[o]);
      if (l == 1) MLP_MARK(5);
      lds_barrier();
      if (l == 1) MLP_MARK(6);
      // per element: normalize, x_norm, scale, bias, activation
#pragma unroll
      for (int q = 0; q < EPT; ++q) {
        const int e = tid + q * NT;
        if (e < BO) {
          const int o = e % Oi;
          const float xn = (yv[q] - st_m[o]) / st_sd[o];
          lay.xnorm()[e] = xn;
          const float z = act_apply(xn * ps[q] + pb[q], lay.act);
          out[e] = z;
          act[e] = z;
        }
      }
    }
    if (l == 1) MLP_MARK(7);
    lds_barrier();
    if (l == 1) MLP_MARK(8);
    in = act;
    MLP_STAMP(1 + l);
  }

  // ---- softmax + cross-entropy (groups 1, temperature 1) ----------------------
  {
    const int tid = stage_tid();
    const int BC = Bi * Ci;
    float* sx = act;             // logits (the last layer's output)
    float* sex = lds;            // exp(x - largest)
    float* smax = lds + BC;      // per row
    float* ssum = smax + B;
    float pt[EPT];
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * NT;
      pt[q] = e < BC ? a.truth[e] : 0.0f;
    }
    for (int b = tid; b < Bi; b += NT) {
      const float* ip = sx + b * Ci;
      float largest = ip[0];
      for (int i = 1; i < Ci; ++i)
        if (ip[i] > largest) largest = ip[i];
      smax[b] = largest;
    }
    lds_barrier();
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * NT;
      if (e < BC) sex[e] = (float)exp((double)((sx[e] - smax[e / Ci]) / 1.0f));
    }
    lds_barrier();
    for (int b = tid; b < Bi; b += NT) {
      const float* ep = sex + b * Ci;
      float sum = 0.0f;
      for (int i = 0; i < Ci; ++i) sum = sum + ep[i];
      ssum[b] = sum;
    }
    lds_barrier();
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * NT;
      if (e < BC) {
        const float p = sex[e] / ssum[e / Ci];
        sm_out[e] = p;
        sm_loss[e] = pt[q] != 0.0f ? (float)(-log((double)(p > SEPS ? p : SEPS))) : 0.0f;
        const float d = pt[q] - p;
        sm_delta[e] = d;
        act[e] = d;  // (the logits are no longer read)
      }
    }
    // the global writes of the forward pass (layer outputs) are read by other
    // threads as dW operands below: one full barrier
    __syncthreads();
  }
  MLP_STAMP(20);

  // ---- backward ---------------------------------------------------------------
  for (int l = L - 1; l >= 0; --l) {
    const int tid = stage_tid(), wid = tid >> 6, lane = tid & 63;
    const Layer lay(a, l);
    const int I = lay.I, O = lay.O, BO = B * O;
    const int Oi = (int)O;
    const float* lin = a.X;
    float* prev_delta = nullptr;
    if (l > 0) {
      const Layer prev(a, l - 1);
      lin = prev.out();
      prev_delta = prev.delta();  // state.delta = nil for layer 0 (nnet.pas:332-335)
    }
    const int tmo = (int)((O + 31) / 32), tni = (int)((I + 31) / 32), tmb = (int)((B + 31) / 32);
    // (layer 0's dW and weight update: mlp_l0_dw_kernel, after this launch)
    const int nw_dw = l == 0 ? 0 : tmo * tni, nw_dx = prev_delta ? tmb * tni : 0;
    const bool defer = l > 0 && defer_update(B, O, I);
    // ahead of the stage: per element out / x / x_norm; per channel (first
    // slot) the parameters of the column pass and of the update
    float dv[EPT], xv[EPT], yo[EPT], xnv[EPT], vv[EPT];
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * NT;
      dv[q] = xv[q] = yo[q] = xnv[q] = vv[q] = 0.0f;
      if (e < BO) {
        yo[q] = lay.out()[e];
        if (a.bn) {
          xv[q] = lay.x()[e];
          xnv[q] = lay.xnorm()[e];
          vv[q] = lay.var()[e % Oi];
        }
      }
    }
    float db_pre = 0.0f, b_pre = 0.0f, ds_pre = 0.0f, sc_pre = 0.0f, mu_pre = 0.0f;
    if (tid < Oi) {
      db_pre = lay.db()[tid];
      b_pre = lay.b()[tid];
      if (a.bn) {
        ds_pre = lay.dscales()[tid];
        sc_pre = lay.scales()[tid];
        mu_pre = lay.mean()[tid];
      }
    }
    // delta (the softmax delta added into the zeroed one for the last layer,
    // else the dX result of the previous stage, both in `act`): clamp, times
    // the activation gradient; staged with x, x_norm for the column passes
    if (l == 2) MLP_MARK(10);
    float* sdel = lds;
    float* sx = lds + BO;
    float* sxn = lds + 2 * BO;
    float* st = lds + 3 * BO;  // per channel: scale, mean, sum m, sum v; then pow (double)
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + q * NT;
      if (e < BO) {
        float d = act[e];
        if (l == L - 1) d = 0.0f + d;  // delta (zeroed in the forward pass) + softmax delta
        d = d < -1.0f ? -1.0f : (d > 1.0f ? 1.0f : d);  // delta.Clamp(-1, 1)
        d = d * grad_apply(yo[q], lay.act);
        sdel[e] = d;
        dv[q] = d;
        if (a.bn) {
          sx[e] = xv[q];
          sxn[e] = xnv[q];
        } else {
          lay.delta()[e] = d;
        }
      }
    }
    if (l == 2) MLP_MARK(11);
    lds_barrier();
    if (l == 2) MLP_MARK(12);
    MLP_STAMP(50 + 2 * l);
    // per channel: bias_updates.addSums and, with BN, addDots (strided sdot:
    // mul then add), forwardScale and meansAndVarsDelta — four independent
    // sequential chains over the batch, interleaved in one loop; then this
    // layer's bias / scale update (TConnectedLayer.update: nothing later in
    // the step reads b, db, dscales, and scales only from LDS)
    // the double pow of meansAndVarsDelta depends on the forward variance
    // only: the last wave evaluates it for every channel while wave 0 runs
    // the chains (it was the longest single latency of the chain thread)
    double* st_pw = reinterpret_cast<double*>(st + ((4 * O + 1) & ~(int)1));
    if (a.bn && wid == NWAVES - 1)
      for (int o = lane; o < Oi; o += 64) {
        const float var = lay.var()[o];
        const float ve = var > SEPS ? var : SEPS;
#ifdef TNS_MLP_NOPOW  // (diagnostic timing build: wrong numbers)
        st_pw[o] = (double)ve;
#else
        st_pw[o] = pow((double)ve, -1.5);
#endif
      }
    auto chain = [&](int o, float db0, float b0, float ds0, float sc, float mu) {
      // rows past the batch add +0.0f, selected off the chains (every chain
      // starts at +0, so none is ever -0, and x + (+0) == x otherwise): the
      // chains hold only their adds
      float r = 0.0f, dd = 0.0f, m = 0.0f, v = 0.0f;
      for (int b0r = 0; b0r < Bi; b0r += 8) {
        float cs[8], cn[8], cx[8];
        col8(cs, sdel + o, b0r, Bi, Oi);
        if (a.bn) {
          col8(cn, sxn + o, b0r, Bi, Oi);
          col8(cx, sx + o, b0r, Bi, Oi);
          hold8(cn);
          hold8(cx);
        }
        hold8(cs);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const bool in = b0r + u < Bi;
          const float sv = cs[u];
          r = r + (in ? sv : 0.0f);
          if (a.bn) {
            const float d = sv * sc;  // forwardScale
            const float pd = cn[u] * sv, pv = (cx[u] - mu) * d;
            dd = dd + (in ? pd : 0.0f);
            m = m + (in ? d : 0.0f);
            v = v + (in ? pv : 0.0f);
          }
        }
      }
      const float dbn = db0 + r;
      lay.b()[o] = fmaf(lrb, dbn, b0);  // biases.axpy(lr/batch, bias_updates)
      lay.db()[o] = mom * dbn;          // bias_updates.Multiply(momentum)
      if (a.bn) {
        const float dsn = ds0 + dd;
        lay.scales()[o] = fmaf(lrb, dsn, sc);  // scales.axpy(lr/batch, scale_updates)
        lay.dscales()[o] = mom * dsn;          // scale_updates.Multiply(momentum)
        st[o] = sc;
        st[O + o] = mu;
        st[2 * O + o] = m;
        st[3 * O + o] = v;
      }
    };
    if (tid < Oi) chain(tid, db_pre, b_pre, ds_pre, sc_pre, mu_pre);  // prefetched
    for (int o = tid + NT; o < Oi; o += NT)
      chain(o, lay.db()[o], lay.b()[o], a.bn ? lay.dscales()[o] : 0.0f,
            a.bn ? lay.scales()[o] : 0.0f, a.bn ? lay.mean()[o] : 0.0f);
    if (l == 2) MLP_MARK(13);
    if (a.bn) {
      lds_barrier();
      if (l == 2) MLP_MARK(14);
      // per element: the channel's mean/variance deltas (the thread of batch
      // row 0 stores them), then normalizeDelta of the scaled delta
#pragma unroll
      for (int q = 0; q < EPT; ++q) {
        const int e = tid + q * NT;
        if (e < BO) {
          const int o = e % Oi;
          const float var = vv[q];
          const float ve = var > SEPS ? var : SEPS;
          const float sd = sqrtf(ve);
          const float md = st[2 * O + o] * (-1.0f / sd);
          const float vd = (float)((double)st[3 * O + o] * -0.5 * st_pw[o]);
          if (e < O) {
            lay.mdelta()[o] = md;
            lay.vdelta()[o] = vd;
          }
          const float d = dv[q] * st[o];
          const float qd = d / sd;
          const float t = (xv[q] - st[O + o]) * (2.0f * vd / (float)B) + md / (float)B;
          const float nd = qd + t;
          lay.delta()[e] = nd;
          sdel[e] = nd;
        }
      }
    }
    if (l == 2) MLP_MARK(15);
    lds_barrier();
    if (l == 2) MLP_MARK(16);
    MLP_STAMP(51 + 2 * l);
    // dW += delta^T . in   (TN: M=O, N=I, K=B, beta 1)   and
    // prev_delta += delta . W (NN: M=B, N=I, K=O, beta 1), both ascending
    // chains; layer 0 (no dX) updates its weights in the dW epilogue, other
    // layers after the stage's dX tasks (or in the pass after the backward)
    bool have = false;
    int hm0 = 0, hn0 = 0;
    floatx16 hacc;
    float hw[16];
    for (int w = wid; w < nw_dw + nw_dx; w += NWAVES) {
      if (w < nw_dw) {
        const int m0 = (int)(w / tni) * 32, n0 = (int)(w % tni) * 32;
        dw_task(sdel, m0, n0, B, O, I, lin, lay.dW(), lay.W(), l == 0 || defer, hacc, hw, lane);
        if (l == 2) MLP_MARK(17);
        if (defer) {
          have = true;
          hm0 = m0;
          hn0 = n0;
        } else {
          dw_store(m0, n0, O, I, lay.dW(), lay.W(), l == 0, hacc, hw, lrb, wdec, mom, lane);
        }
      } else {
        const int t = w - nw_dw;
        const int m0 = (int)(t / tni) * 32, n0 = (int)(t % tni) * 32;
        dx_task(sdel, m0, n0, B, O, I, lay.W(), prev_delta, act, lane);
      }
    }
    if (l == 2) MLP_MARK(18);
    lds_barrier();  // every dX task has read W and written its block to `act`
    if (l == 2) MLP_MARK(19);
    if (have) dw_store(hm0, hn0, O, I, lay.dW(), lay.W(), true, hacc, hw, lrb, wdec, mom, lane);
    MLP_STAMP(21 + l);
  }

  // ---- weight update of layers whose dW tasks were more than one per wave
  // (none in the MNIST net), after every dW store is visible ---------------------
  bool rest = false;
  for (int l = 1; l < L; ++l) rest = rest || !defer_update(B, a.widths[l + 1], a.widths[l]);
  if (rest) {
    const int tid = stage_tid();
    __syncthreads();
    for (int l = 1; l < L; ++l) {
      const Layer lay(a, l);
      if (defer_update(B, lay.O, lay.I)) continue;
      const int IO = lay.I * lay.O;
      float* W = lay.W();
      float* dW = lay.dW();
      constexpr int UB = 8;
      for (int e0 = tid; e0 < IO; e0 += (int)NT * UB) {
        float w[UB], g[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int e = e0 + (int)u * NT;
          w[u] = W[e < IO ? e : e0];
          g[u] = dW[e < IO ? e : e0];
        }
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int e = e0 + (int)u * NT;
          if (e < IO) {
            const float dw = fmaf(wdec, w[u], g[u]);  // weight_updates.axpy(-decay*batch, W)
            W[e] = fmaf(lrb, dw, w[u]);               // weights.axpy(lr/batch, dW)
            dW[e] = mom * dw;                         // weight_updates.Multiply(momentum)
          }
        }
      }
    }
  }
  MLP_STAMP(40);

  // ---- cost: loss.Sum() in the vssum_avx2 order: lane l of wave 0 sums
  // elements 8t + l in ascending t, lane 0 folds (l, l+4), the pairs and the
  // tail (sm_loss was written before the full barrier after the softmax) ----
  const int wid = stage_tid() >> 6, lane = threadIdx.x & 63;
  if (wid == 0) {
    const int n = B * C, blocks = n >> 3;
    float acc = 0.0f;
    if (lane < 8)
      for (int t = 0; t < blocks; ++t) acc = acc + sm_loss[8 * t + lane];
    const float a0 = __shfl(acc, 0), a1 = __shfl(acc, 1), a2 = __shfl(acc, 2),
                a3 = __shfl(acc, 3), a4 = __shfl(acc, 4), a5 = __shfl(acc, 5),
                a6 = __shfl(acc, 6), a7 = __shfl(acc, 7);
    if (lane == 0) {
      const float s0 = a0 + a4, s1 = a1 + a5, s2 = a2 + a6, s3 = a3 + a7;
      float r = (s0 + s1) + (s2 + s3);
      for (int i = blocks * 8; i < n; ++i) r = r + sm_loss[i];
      *a.cost = r;
    }
  }
}


// ---- layer 0 outside the single-CU launch ------------------------------------
// Layer 0's gemms are the step's only large ones (784 x 64 at batch 32: 1.6 M
// FMAs each, ~12.5 k MFMA cycles on one CU); they run as their own launches
// over several CUs, before and after the fused kernel.

// Forward residue partials of layer 0 (the same chains as gemm_chunked):
// block = one 32x32 output tile x 4 residue classes (one per wave); both
// operands' tile rows staged through LDS in k-chunks of KCH, float4 loads two
// chunks ahead; partial r of (m, n) to part[(r*B + m)*O + n].
// NCMAX > 0 (I <= NCMAX*KCH): every chunk's loads issued at the start into
// registers (the block moves ~200 KB through one CU; two chunks in flight
// left it waiting on memory latency once per chunk), two LDS buffers, one
// barrier per chunk.
template <int KCH, int VEC, int NCMAX>
__global__ __launch_bounds__(256) void mlp_l0_forward_kernel(const float* X, const float* W,
                                                             int64_t B, int64_t O, int64_t I,
                                                             float* part) {
  // VEC = 4: float4 units (16-byte rows); 1: single floats
  // NCMAX forms: rows padded to KCH + 4 (16-byte aligned: one ds_write_b128 a
  // unit; the fragment reads then meet two lanes a bank); else KCH + 1
#ifdef TNS_MLP_L0_KP1
  constexpr int KP = KCH + 1;
#else
  constexpr int KP = NCMAX > 0 ? KCH + 4 : KCH + 1;
#endif
  constexpr int QR = KCH / VEC, UV = (64 * QR + 255) / 256;
  __shared__ __attribute__((aligned(16))) float lds[(NCMAX > 0 ? 2 : 1) * 64 * KP];
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, l31 = lane & 31, h = lane >> 5;
  const int tn = (int)((O + 31) / 32), tile = blockIdx.x >> 1;
  const int64_t m0 = (int64_t)(tile / tn) * 32, n0 = (int64_t)(tile % tn) * 32;
  const int r = 4 * (blockIdx.x & 1) + wid;
  floatx16 acc;
  for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
  // NCMAX forms: buffer loads, rows 8u..8u+7 of unit u are all X rows (u <
  // 4) or all W rows, out-of-range units read 0 through an offset past the
  // buffer (no select, so no branch around the load that would make the
  // compiler wait between the loads)
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X), 0, (int)(B * I * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(W), 0, (int)(O * I * 4), 0x00020000);
  auto load = [&](int64_t kc0, float4 (&v)[UV]) {
    if constexpr (NCMAX > 0) {
      static_assert(VEC == 4 && QR == 32 && UV == 8, "unit u = rows 8u .. 8u+7");
#pragma unroll
      for (int u = 0; u < UV; ++u) {
        const int row = (tid >> 5) + 8 * u, kq = tid & 31;
        const int64_t k = kc0 + 4 * kq;
        const int64_t g = u < 4 ? m0 + row : n0 + row - 32;
        const bool ok = k < I && g < (u < 4 ? B : O);
        const unsigned off = ok ? (unsigned)((g * I + k) * 4) : 0x80000000u;
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        const u4 x = __builtin_amdgcn_raw_buffer_load_b128(u < 4 ? rx : rw, off, 0, 0);
        v[u] = make_float4(__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(x.z),
                           __uint_as_float(x.w));
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < UV; ++u) {
      const int idx = tid + u * 256;
      const int row = idx / QR, kq = idx % QR;
      const int64_t k = kc0 + VEC * kq;
      const bool isx = row < 32;
      const int64_t g = isx ? m0 + row : n0 + row - 32;
      const bool ok = idx < 64 * QR && k < I && g < (isx ? B : O);
      const float* src = (isx ? X : W) + (ok ? g * I + k : 0);
      if constexpr (VEC == 4) {
        const float4 x = *reinterpret_cast<const float4*>(src);
        v[u] = ok ? x : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      } else {
        const float x = *src;
        v[u].x = ok ? x : 0.0f;
      }
    }
  };
  auto store = [&](const float4 (&v)[UV], int buf = 0) {
#pragma unroll
    for (int u = 0; u < UV; ++u) {
      const int idx = tid + u * 256;
      if (idx < 64 * QR) {
        float* d = lds + buf * 64 * KP + (idx / QR) * KP + VEC * (idx % QR);
        if constexpr (VEC == 4 && KP % 4 == 0) {
          *reinterpret_cast<float4*>(d) = v[u];
          continue;
        }
        d[0] = v[u].x;
        if constexpr (VEC == 4) {
          d[1] = v[u].y; d[2] = v[u].z; d[3] = v[u].w;
        }
      }
    }
  };
  auto compute = [&](int buf = 0) {
    const float* L = lds + buf * 64 * KP;
#pragma unroll
    for (int st = 0; st < KCH / 16; ++st) {  // k = kc0 + r + 8*(2*st + h)
      const int kk = r + 8 * (2 * st + h);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(L[l31 * KP + kk], L[(32 + l31) * KP + kk],
                                                 acc, 0, 0, 0);
    }
  };
  const int64_t nch = (I + KCH - 1) / KCH;
  if constexpr (NCMAX > 0) {
    // (chunks past the last load zeros from clamped addresses: no branch
    // between the loads, so the waits before each store count exactly)
    float4 rr[NCMAX][UV];
#pragma unroll
    for (int c = 0; c < NCMAX; ++c) load((int64_t)c * KCH, rr[c]);
    asm volatile("" ::: "memory");  // (keeps every load above the first store)
#pragma unroll
    for (int c = 0; c < NCMAX; ++c) {
      if (c < nch) {
        store(rr[c], c & 1);
        __syncthreads();  // (also: every wave is past compute(c - 2) of this buffer)
        compute(c & 1);
      }
    }
  } else {
  float4 r0[UV], r1[UV];
  load(0, r0);
  if (nch > 1) load(KCH, r1);
  for (int64_t c = 0; c < nch; c += 2) {
    store(r0);
    __syncthreads();
    if (c + 2 < nch) load((c + 2) * KCH, r0);
    compute();
    __syncthreads();
    if (c + 1 < nch) {
      store(r1);
      __syncthreads();
      if (c + 3 < nch) load((c + 3) * KCH, r1);
      compute();
      __syncthreads();
    }
  }
  }
  for (int e = 0; e < 16; ++e) {
    const int64_t m = m0 + acc_row(e, lane), n = n0 + l31;
    if (m < B && n < O) part[(r * B + m) * O + n] = acc[e];
  }
}

// dW0 += delta0^T . X (TN, k over the batch) and TConnectedLayer.update's
// weight part, one 32x32 tile per wave (delta0 is final once the fused
// kernel has ended)
__global__ __launch_bounds__(64) void mlp_l0_dw_kernel(const float* delta, const float* X,
                                                       float* dW, float* W, int64_t B, int64_t O,
                                                       int64_t I, float lrb, float wdec,
                                                       float momentum) {
  const int lane = threadIdx.x;
  const int tni = (int)((I + 31) / 32);
  const int64_t m0 = (int64_t)(blockIdx.x / tni) * 32, n0 = (int64_t)(blockIdx.x % tni) * 32;
  floatx16 acc;
  float wv[16];
  dw_task<16>(delta, m0, n0, B, O, I, X, dW, W, true, acc, wv, lane);  // (B <= 32: one batch)
  dw_store(m0, n0, O, I, dW, W, true, acc, wv, lrb, wdec, momentum, lane);
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
  // [0, act_off): partial sums (8 [B][O] blocks; >= 3 blocks + statistics in
  // the backward), or the forward gemm's k-chunks of both operands when one
  // (tile, residue) task per wave covers every layer; then the [B][O_max]
  // hand-off block
  const int64_t tmx = (a.batch + 31) / 32, tnx = (omax + 31) / 32;
  const int64_t part = 8 * a.batch * omax, blk = a.batch * omax;
  const int64_t chunks = (tmx + tnx) * 32 * (KC + 1);
  constexpr int64_t LDS_FLOATS = 160 * 1024 / 4;
  a.lds_chunks = tmx * tnx * 8 <= NWAVES && chunks + blk + 4 <= LDS_FLOATS;
  int64_t act_off = a.lds_chunks && chunks > part ? chunks : part;
  act_off = (act_off + 3) & ~(int64_t)3;  // 16-byte aligned hand-off block
  a.act_off = act_off;
  const size_t lds = (size_t)(act_off + blk) * sizeof(float);
  if (act_off + blk > LDS_FLOATS) return hipErrorInvalidValue;
  if (lds > 64 * 1024) {
    const hipError_t e2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_train_kernel<EPT_S>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)lds);
    const hipError_t e5 = hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_train_kernel<EPT_L>),
                                              hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)lds);
    if (e2 != hipSuccess) return e2;
    if (e5 != hipSuccess) return e5;
  }
  // layer 0: forward partials over several CUs, then the fused step, then
  // layer 0's dW + weight update over several CUs
  const int64_t B0 = a.batch, I0 = a.widths[0], O0 = a.widths[1];
  if (!a.l0part) return hipErrorInvalidValue;
  const float* W0 = a.buf + a.off[0][F_W];
  const bool vec0 = I0 % 4 == 0 && ((reinterpret_cast<uintptr_t>(a.X) |
                                     reinterpret_cast<uintptr_t>(W0)) & 15) == 0;
  const unsigned fblocks = (unsigned)(2 * ((B0 + 31) / 32) * ((O0 + 31) / 32));
#ifndef TNS_MLP_L0_TWO
  if (vec0 && I0 <= 8 * 128)
    hipLaunchKernelGGL((mlp_l0_forward_kernel<128, 4, 8>), dim3(fblocks), dim3(256), 0, s, a.X,
                       W0, B0, O0, I0, a.l0part);
  else
#endif
  if (vec0)
    hipLaunchKernelGGL((mlp_l0_forward_kernel<128, 4, 0>), dim3(fblocks), dim3(256), 0, s, a.X, W0,
                       B0, O0, I0, a.l0part);
  else
    hipLaunchKernelGGL((mlp_l0_forward_kernel<64, 1, 0>), dim3(fblocks), dim3(256), 0, s, a.X, W0,
                       B0, O0, I0, a.l0part);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  if (blk <= EPT_S * NT)
    hipLaunchKernelGGL(mlp_train_kernel<EPT_S>, dim3(1), dim3(NT), lds, s, a);
  else
    hipLaunchKernelGGL(mlp_train_kernel<EPT_L>, dim3(1), dim3(NT), lds, s, a);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  const unsigned dblocks = (unsigned)(((O0 + 31) / 32) * ((I0 + 31) / 32));
  hipLaunchKernelGGL(mlp_l0_dw_kernel, dim3(dblocks), dim3(64), 0, s,
                     a.buf + a.off[0][F_DELTA], a.X, a.buf + a.off[0][F_DW],
                     a.buf + a.off[0][F_W], B0, O0, I0, a.lr / (float)B0,
                     -a.decay * (float)B0, a.momentum);
  return hipGetLastError();
}

}  // namespace tns
