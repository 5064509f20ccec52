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
__device__ constexpr float SEPS = 0.000001f;

struct Layer {
  int64_t I, O;
  int act;
  float *W, *b, *dW, *db, *scales, *rmean, *rvar, *dscales, *out, *delta, *x, *xnorm, *mean,
      *var, *mdelta, *vdelta;
};

__device__ void layer_at(const MlpArgs& a, int want, Layer& L, float** softmax_base) {
  float* p = a.buf;
  const int64_t B = a.batch;
  for (int l = 0; l < a.nlayers; ++l) {
    Layer t;
    t.I = a.widths[l];
    t.O = a.widths[l + 1];
    t.act = a.acts[l];
    const int64_t IO = t.I * t.O, O = t.O, BO = B * t.O;
    t.W = p; p += IO;
    t.b = p; p += O;
    t.dW = p; p += IO;
    t.db = p; p += O;
    t.scales = t.rmean = t.rvar = t.dscales = nullptr;
    t.x = t.xnorm = t.mean = t.var = t.mdelta = t.vdelta = nullptr;
    if (a.bn) {
      t.scales = p; p += O;
      t.rmean = p; p += O;
      t.rvar = p; p += O;
      t.dscales = p; p += O;
    }
    t.out = p; p += BO;
    t.delta = p; p += BO;
    if (a.bn) {
      t.x = p; p += BO;
      t.xnorm = p; p += BO;
      t.mean = p; p += O;
      t.var = p; p += O;
      t.mdelta = p; p += O;
      t.vdelta = p; p += O;
    }
    if (l == want) L = t;
  }
  if (softmax_base) *softmax_base = p;
}

// One 32x32 MFMA output tile: acc += sum over steps s of A[m][k(s,h)]*B[k(s,h)][n]
// with the lane maps of v_mfma_f32_32x32x2_f32 (lane l: m = l&31 of A, n = l&31
// of B, k-slot h = l>>5).  kfun(s, h) gives the k consumed in step s by half h
// (ascending per accumulator); out-of-range values are supplied as 0 by fa/fb.
template <class FA, class FB>
__device__ __forceinline__ void mfma_tile(floatx16& acc, int steps, FA fa, FB fb) {
  const int lane = threadIdx.x & 63;
  const int l31 = lane & 31, h = lane >> 5;
  for (int s = 0; s < steps; ++s) {
    const float av = fa(l31, s, h);
    const float bv = fb(l31, s, h);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
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

__global__ __launch_bounds__(NT) void mlp_train_kernel(MlpArgs a) {
  extern __shared__ float lds[];  // 8 * B * O_max partial sums of the forward gemm
  const int tid = threadIdx.x;
  const int wid = tid >> 6;
  const int lane = tid & 63;
  const int64_t B = a.batch;
  const int L = a.nlayers;
  const int64_t C = a.widths[L];
  float* smx;
  Layer lay;
  layer_at(a, 0, lay, &smx);
  float* sm_out = smx;
  float* sm_delta = smx + B * C;
  float* sm_loss = smx + 2 * B * C;

  // ---- forward ------------------------------------------------------------
  const float* in = a.X;
  for (int l = 0; l < L; ++l) {
    layer_at(a, l, lay, nullptr);
    const int64_t I = lay.I, O = lay.O, BO = B * O;
    for (int64_t e = tid; e < BO; e += NT) lay.delta[e] = 0.0f;  // nnet.pas:287-296

    // gemm(RowMajor, NoTrans, Trans, B, O, I, 1, in, I, W, I, 0, out, O):
    // sdot_avx2 residue classes r = k mod 8, each an ascending MFMA chain
    const int tm = (int)((B + 31) / 32), tn = (int)((O + 31) / 32);
    const int64_t kr = (I + 7) / 8;            // k values per residue class
    const int steps = (int)((kr + 1) / 2);
    for (int w = wid; w < tm * tn * 8; w += NWAVES) {
      const int r = w & 7, tile = w >> 3;
      const int64_t m0 = (int64_t)(tile / tn) * 32, n0 = (int64_t)(tile % tn) * 32;
      floatx16 acc;
      for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
      mfma_tile(acc, steps,
                [&](int l31, int s, int h) {
                  const int64_t m = m0 + l31, k = r + 8 * (2 * (int64_t)s + h);
                  return (m < B && k < I) ? in[m * I + k] : 0.0f;
                },
                [&](int l31, int s, int h) {
                  const int64_t n = n0 + l31, k = r + 8 * (2 * (int64_t)s + h);
                  return (n < O && k < I) ? lay.W[n * I + k] : 0.0f;
                });
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
      const float c0 = 0.0f * lay.out[e];  // beta = 0 => 0*C (mulvs)
      lay.out[e] = c0 + 1.0f * dot;        // C := C + ALPHA*sdot
    }
    __syncthreads();
    if (a.bn) {
      // per channel: MeansAndVars, rolling stats, x, normalize, x_norm, scale
      for (int64_t o = tid; o < O; o += NT) {
        float m = 0.0f;
        for (int64_t b = 0; b < B; ++b) m = m + lay.out[b * O + o];
        m = m / (float)B;
        float v = 0.0f;
        for (int64_t b = 0; b < B; ++b) {
          const float t = lay.out[b * O + o] - m;
          v = v + t * t;
        }
        v = v / (float)(B - 1);
        lay.mean[o] = m;
        lay.var[o] = v;
        const float mom = 0.05f;  // bnMomentum, nconnectedlayer.pas:67
        lay.rmean[o] = fmaf(mom, m, lay.rmean[o] * (1.0f - mom));
        lay.rvar[o] = fmaf(mom, v, lay.rvar[o] * (1.0f - mom));
        const float sd = sqrtf(v > SEPS ? v : SEPS);
        for (int64_t b = 0; b < B; ++b) {
          const float xv = lay.out[b * O + o];
          lay.x[b * O + o] = xv;
          const float xn = (xv - m) / sd;
          lay.xnorm[b * O + o] = xn;
          lay.out[b * O + o] = xn * lay.scales[o];
        }
      }
      __syncthreads();
    }
    for (int64_t e = tid; e < BO; e += NT) {
      const int64_t o = e % O;
      lay.out[e] = act_apply(lay.out[e] + lay.b[o], lay.act);  // forwardBias, activate
    }
    __syncthreads();
    in = lay.out;
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

  // ---- backward ---------------------------------------------------------------
  for (int l = L - 1; l >= 0; --l) {
    layer_at(a, l, lay, nullptr);
    const int64_t I = lay.I, O = lay.O, BO = B * O;
    Layer prev;
    const float* lin = a.X;
    float* prev_delta = nullptr;
    if (l > 0) {
      layer_at(a, l - 1, prev, nullptr);
      lin = prev.out;
      prev_delta = prev.delta;  // state.delta = nil for layer 0 (nnet.pas:332-335)
    }
    // softmax backward: prev.delta += delta; then clamp + activation gradient
    for (int64_t e = tid; e < BO; e += NT) {
      float d = lay.delta[e];
      if (l == L - 1) d = d + sm_delta[e];
      d = d < -1.0f ? -1.0f : (d > 1.0f ? 1.0f : d);  // delta.Clamp(-1, 1)
      lay.delta[e] = d * grad_apply(lay.out[e], lay.act);
    }
    __syncthreads();
    // per channel: bias_updates.addSums, then the BN backward chain
    for (int64_t o = tid; o < O; o += NT) {
      float r = 0.0f;
      for (int64_t b = 0; b < B; ++b) r = r + lay.delta[b * O + o];
      lay.db[o] = lay.db[o] + r;
      if (a.bn) {
        float dd = 0.0f;  // addDots (strided sdot: mul then add)
        for (int64_t b = 0; b < B; ++b) dd = dd + lay.xnorm[b * O + o] * lay.delta[b * O + o];
        lay.dscales[o] = lay.dscales[o] + dd;
        const float sc = lay.scales[o], mu = lay.mean[o];
        float m = 0.0f, v = 0.0f;
        for (int64_t b = 0; b < B; ++b) {
          const float d = lay.delta[b * O + o] * sc;  // forwardScale
          lay.delta[b * O + o] = d;
          m = m + d;
          v = v + (lay.x[b * O + o] - mu) * d;
        }
        const float ve = lay.var[o] > SEPS ? lay.var[o] : SEPS;
        const float md = m * (-1.0f / sqrtf(ve));
        const float vd = (float)((double)v * -0.5 * pow((double)ve, -1.5));
        lay.mdelta[o] = md;
        lay.vdelta[o] = vd;
        const float mdb = md / (float)B, vdb = 2.0f * vd / (float)B, sd = sqrtf(ve);
        for (int64_t b = 0; b < B; ++b) {
          const float q = lay.delta[b * O + o] / sd;
          const float t = (lay.x[b * O + o] - mu) * vdb + mdb;
          lay.delta[b * O + o] = q + t;
        }
      }
    }
    __syncthreads();
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
      float* Cp = is_dw ? lay.dW : prev_delta;
      for (int e = 0; e < 16; ++e) {
        const int64_t m = m0 + acc_row(e), n = n0 + (lane & 31);
        acc[e] = (m < Mx && n < I) ? Cp[m * I + n] : 0.0f;
      }
      if (is_dw) {
        mfma_tile(acc, (int)((B + 1) / 2),
                  [&](int l31, int s, int h) {
                    const int64_t m = m0 + l31, k = 2 * (int64_t)s + h;
                    return (m < O && k < B) ? lay.delta[k * O + m] : 0.0f;
                  },
                  [&](int l31, int s, int h) {
                    const int64_t n = n0 + l31, k = 2 * (int64_t)s + h;
                    return (n < I && k < B) ? lin[k * I + n] : 0.0f;
                  });
      } else {
        mfma_tile(acc, (int)((O + 1) / 2),
                  [&](int l31, int s, int h) {
                    const int64_t m = m0 + l31, k = 2 * (int64_t)s + h;
                    return (m < B && k < O) ? lay.delta[m * O + k] : 0.0f;
                  },
                  [&](int l31, int s, int h) {
                    const int64_t n = n0 + l31, k = 2 * (int64_t)s + h;
                    return (n < I && k < O) ? lay.W[k * I + n] : 0.0f;
                  });
      }
      for (int e = 0; e < 16; ++e) {
        const int64_t m = m0 + acc_row(e), n = n0 + (lane & 31);
        if (m < Mx && n < I) Cp[m * I + n] = acc[e];
      }
    }
    __syncthreads();
  }

  // ---- update (TConnectedLayer.update, constant learning rate) ----------------
  const float lrb = a.lr / (float)B;
  const float wdec = -a.decay * (float)B;
  for (int l = 0; l < L; ++l) {
    layer_at(a, l, lay, nullptr);
    const int64_t O = lay.O, IO = lay.I * lay.O;
    for (int64_t o = tid; o < O; o += NT) {
      lay.b[o] = fmaf(lrb, lay.db[o], lay.b[o]);
      lay.db[o] = a.momentum * lay.db[o];
      if (a.bn) {
        lay.scales[o] = fmaf(lrb, lay.dscales[o], lay.scales[o]);
        lay.dscales[o] = a.momentum * lay.dscales[o];
      }
    }
    for (int64_t e = tid; e < IO; e += NT) {
      float dw = fmaf(wdec, lay.W[e], lay.dW[e]);  // weight_updates.axpy(-decay*batch, W)
      const float w = fmaf(lrb, dw, lay.W[e]);     // weights.axpy(lr/batch, dW)
      lay.W[e] = w;
      lay.dW[e] = a.momentum * dw;                  // weight_updates.Multiply(momentum)
    }
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

hipError_t launch_mlp_train_step(const MlpArgs& a, hipStream_t s) {
  int64_t omax = 0;
  for (int l = 0; l < a.nlayers; ++l) omax = a.widths[l + 1] > omax ? a.widths[l + 1] : omax;
  const size_t lds = (size_t)(8 * a.batch * omax) * sizeof(float);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mlp_train_kernel, dim3(1), dim3(NT), lds, s, a);
  return hipGetLastError();
}

}  // namespace tns
