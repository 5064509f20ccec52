/*
 * tns_oracle_train.c — TEST INFRASTRUCTURE ONLY (see tns_oracle.h header).
 *
 * CPU restatement of the reference's batch-norm, softmax / cross-entropy,
 * SGD update and connected-layer train step (BASELINE config 5):
 *   TTensor.MeansAndVars        ntensors.pas:9102-9177
 *   blockNormalize/_snormvv     ntensors.pas:8693-8718, 4331-4385
 *   forwardScale / forwardBias  ntensors.pas:7687-7727
 *   addSums / addDots           ntensors.pas:7729-7830
 *   sMeanAndVarianceDelta       ntensors.pas:8831-8899 (+ sVarinceDelta_avx 8721)
 *   sNormalizeDelta             ntensors.pas:8902-8951 (+ sNormalizeDelta_avx 8761)
 *   softmax / softmaxCrossEntropy  nsoftmaxlayer.pas:83-137
 *   TConnectedLayer.forward/backward/update  nconnectedlayer.pas:157-359
 *   TNNet.forward/backward/update/cost       nnet.pas:275-403, 551-564
 *
 * Where the reference's AVX2 kernels are approximate or buggy (snormvss_avx
 * uses rcpss; srss drops upper lanes when N%8==0 — SURVEY Appendix B.5/B.6)
 * the scalar Pascal form is restated instead (quirk switches reproduce the
 * srss / sVarinceDelta_avx lane drop).  Transcendentals (exp, ln, Power) are
 * evaluated in double and rounded once, as the device does; FPC evaluates
 * them in extended precision, so a last-ulp difference from the reference
 * itself is possible (parity unpinned).
 *   conv layer with batch norm: nConvolutionLayer.pas:457-671 with
 *   TBaseLayer.batchNorm / batchNormBack (nbaselayer.pas:336-395)
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "tns_oracle.h"

static const float SEPS = 0.000001f; /* sEPSILON, ntensors.pas:95 */

/* vssum_avx2 (ntensors.pas:3592-3620): 8 lanes over full blocks, fold
 * lane_l + lane_{l+4}, hadd twice, then the remainder sequentially. */
float ora_vssum(int64_t n, const float* a) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t blocks = n >> 3;
  for (int64_t t = 0; t < blocks; t++)
    for (int l = 0; l < 8; l++) acc[l] = acc[l] + a[8 * t + l];
  float s0 = acc[0] + acc[4], s1 = acc[1] + acc[5], s2 = acc[2] + acc[6], s3 = acc[3] + acc[7];
  float r = (s0 + s1) + (s2 + s3);
  for (int64_t i = blocks * 8; i < n; i++) r = r + a[i];
  return r;
}

/* MeansAndVars: per channel i, m = sum_b sumv(bs, x_{b,i}) / (G*bs);
 * v = sum_b rss(bs, m, x_{b,i}) / (G*bs - 1)  (unbiased).  Scalar sums. */
/* srss (ntensors.pas:1493-1523), the stride-1 rssv of an AVX2 host
 * (vsRSS 3646-3658): 8 lanes of (mean - a)^2 sums over the full 8-blocks;
 * when a tail exists, lanes l and l+4 are folded and the tail added to lane
 * 0 in order; then ((x0 + x1) + (x2 + x3)).  With no tail (N % 8 == 0) the
 * reference skips the fold and drops lanes 4..7 — reproduced only when
 * quirk != 0 (TNS_OPT_SRSS_QUIRK); otherwise the lanes are folded as with a
 * tail (reference quirk 6). */
float ora_srss(int64_t n, float mean, const float* a, int quirk) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t blocks = n >> 3;
  for (int64_t t = 0; t < blocks; t++)
    for (int l = 0; l < 8; l++) {
      const float d = mean - a[8 * t + l];
      acc[l] = acc[l] + d * d;
    }
  float x[4];
  if ((n & 7) == 0 && quirk) {
    for (int l = 0; l < 4; l++) x[l] = acc[l];
  } else {
    for (int l = 0; l < 4; l++) x[l] = acc[l] + acc[l + 4];
    for (int64_t i = blocks * 8; i < n; i++) {
      const float d = mean - a[i];
      x[0] = x[0] + d * d;
    }
  }
  return (x[0] + x[1]) + (x[2] + x[3]);
}

/* MeansAndVars (ntensors.pas:9102-9177): per channel, m := m + sumv(block)
 * over the groups in order (sumv = vsSumI -> vssum_avx2 for stride 1),
 * m / S; then v := v + rssv(block, m) (srss), v / S2. */
void ora_means_and_vars_q(const float* x, int64_t groups, int64_t N, int64_t bs, float* means,
                          float* vars, int quirk) {
  const float S = (float)(groups * bs), S2 = (float)(groups * bs - 1);
  for (int64_t i = 0; i < N; i++) {
    float m = 0.0f;
    for (int64_t b = 0; b < groups; b++) m = m + ora_vssum(bs, x + (i + b * N) * bs);
    m = m / S;
    means[i] = m;
    float v = 0.0f;
    for (int64_t b = 0; b < groups; b++) v = v + ora_srss(bs, m, x + (i + b * N) * bs, quirk);
    vars[i] = v / S2;
  }
}

void ora_means_and_vars(const float* x, int64_t groups, int64_t N, int64_t bs, float* means,
                        float* vars) {
  ora_means_and_vars_q(x, groups, N, bs, means, vars, 0);
}

/* blockNormalize: bs == 1 -> _snormvv: (x-m)/sqrt(max(v,eps));
 * bs > 1 -> _snormblkvv/snormvss: (x-m)/max(sqrt(v),eps). */
void ora_normalize(float* x, int64_t groups, int64_t N, int64_t bs, const float* means,
                   const float* vars) {
  for (int64_t g = 0; g < groups; g++)
    for (int64_t i = 0; i < N; i++) {
      float* d = x + (g * N + i) * bs;
      if (bs == 1) {
        float sd = sqrtf(vars[i] > SEPS ? vars[i] : SEPS);
        d[0] = (d[0] - means[i]) / sd;
      } else {
        float sd = sqrtf(vars[i]);
        sd = sd > SEPS ? sd : SEPS;
        for (int64_t j = 0; j < bs; j++) d[j] = (d[j] - means[i]) / sd;
      }
    }
}

/* forwardScale -> vsMulB: c[j] := c[j] * s[i] */
void ora_forward_scale(float* x, int64_t groups, int64_t N, int64_t bs, const float* scales) {
  for (int64_t g = 0; g < groups; g++)
    for (int64_t i = 0; i < N; i++) {
      float* d = x + (g * N + i) * bs;
      for (int64_t j = 0; j < bs; j++) d[j] = d[j] * scales[i];
    }
}

/* addDots: dst[i] += sum over (group, block) of x_norm*delta.
 * bs == 1: dotvv(groups, .., stride nDst) = strided cblas_sdot scalar loop
 * (mul then add).  bs > 1: sdot (8-lane FMA) per block, summed. */
void ora_add_dots(float* dst, const float* a, const float* b, int64_t groups, int64_t N,
                  int64_t bs) {
  for (int64_t i = 0; i < N; i++) {
    if (bs == 1) {
      float r = 0.0f;
      for (int64_t g = 0; g < groups; g++) r = r + a[i + g * N] * b[i + g * N];
      dst[i] = dst[i] + r;
    } else {
      float sum = 0.0f;
      for (int64_t g = 0; g < groups; g++)
        sum = sum + ora_sdot(bs, a + (i + g * N) * bs, b + (i + g * N) * bs);
      dst[i] = dst[i] + sum;
    }
  }
}

/* addSums blockSize == 1 branch: dst[i] += sumv(groups, src+i, stride N)
 * (strided -> scalar vsSumI loop; stride 1, i.e. N == 1 -> vssum_avx2). */
void ora_add_sums(float* dst, const float* src, int64_t groups, int64_t N, int64_t bs) {
  if (bs == 1 && N == 1) {
    dst[0] = dst[0] + ora_vssum(groups, src);
  } else if (bs == 1) {
    for (int64_t i = 0; i < N; i++) {
      float r = 0.0f;
      for (int64_t g = 0; g < groups; g++) r = r + src[i + g * N];
      dst[i] = dst[i] + r;
    }
  } else {
    ora_backward_bias(N, dst, groups, bs, src);
  }
}

/* sVarinceDelta_avx (ntensors.pas:8721-8757), the per-block routine the
 * configured USE_AVX2 build calls from sMeanAndVarianceDelta (8856-8859):
 *   8 lanes over the full 8-blocks, acc_l := acc_l + (x - mean) * delta
 *   (vsubps, vmulps, vaddps: each rounded; 8729-8736);
 *   with a tail (N % 8 != 0): x_l := acc_l + acc_{l+4} (vextractf128 + addps,
 *   8742-8744), then every tail element added into lane 0 in order
 *   (vsubss, vmulss, vaddss, 8746-8753);
 *   then haddps twice: (x0 + x1) + (x2 + x3) (8755-8756).
 * Without a tail the fold is skipped and lanes 4..7 are dropped (the jz at
 * 8741 jumps straight to the haddps) — reproduced only when quirk != 0
 * (TNS_OPT_SRSS_QUIRK, reference quirk 6); otherwise the lanes are folded as
 * with a tail.  For N < 8 all lanes are +0 and the result is the tail's
 * sequential sum. */
float ora_var_delta_avx(int64_t n, float mean, const float* delta, const float* x, int quirk) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t blocks = n >> 3;
  for (int64_t t = 0; t < blocks; t++)
    for (int l = 0; l < 8; l++) {
      const float d = x[8 * t + l] - mean;
      const float p = d * delta[8 * t + l];
      acc[l] = acc[l] + p;
    }
  float r[4];
  if ((n & 7) == 0 && quirk) {
    for (int l = 0; l < 4; l++) r[l] = acc[l];
  } else {
    for (int l = 0; l < 4; l++) r[l] = acc[l] + acc[l + 4];
    for (int64_t i = blocks * 8; i < n; i++) {
      const float d = x[i] - mean;
      const float p = d * delta[i];
      r[0] = r[0] + p;
    }
  }
  return (r[0] + r[1]) + (r[2] + r[3]);
}

/* sMeanAndVarianceDelta (ntensors.pas:8831-8899) with the USE_AVX2 forms:
 * per channel i, over the groups j in order, m := m + vsSumI(block)
 * (vssum_avx2) and v := v + sVarinceDelta_avx(block) (8853, 8856-8859);
 * then mean_delta = m * (-1/sqrt(max(var, eps))) and
 * variance_delta = v * -0.5 * Power(max(var, eps), -3/2) (8869-8870). */
void ora_mean_var_delta_q(const float* delta, const float* x, const float* mean,
                          const float* var, int64_t groups, int64_t N, int64_t bs,
                          float* mean_delta, float* var_delta, int quirk) {
  for (int64_t i = 0; i < N; i++) {
    float m = 0.0f, v = 0.0f;
    for (int64_t j = 0; j < groups; j++) {
      const float* dd = delta + (i + j * N) * bs;
      const float* xx = x + (i + j * N) * bs;
      m = m + ora_vssum(bs, dd);
      v = v + ora_var_delta_avx(bs, mean[i], dd, xx, quirk);
    }
    float ve = var[i] > SEPS ? var[i] : SEPS;
    float inv = -1.0f / sqrtf(ve);
    mean_delta[i] = m * inv;
    var_delta[i] = (float)((double)v * -0.5 * pow((double)ve, -1.5));
  }
}

void ora_mean_var_delta(const float* delta, const float* x, const float* mean,
                        const float* var, int64_t groups, int64_t N, int64_t bs,
                        float* mean_delta, float* var_delta) {
  ora_mean_var_delta_q(delta, x, mean, var, groups, N, bs, mean_delta, var_delta, 0);
}

/* sNormalizeDelta (AVX2 sNormalizeDelta_avx order):
 * d := d/std + ((x-mean)*(2*vd/B) + md/B),  B = groups*bs */
void ora_normalize_delta(const float* x, const float* mean, const float* var,
                         const float* mean_delta, const float* var_delta, float* delta,
                         int64_t groups, int64_t N, int64_t bs) {
  const float B = (float)(groups * bs);
  for (int64_t j = 0; j < groups; j++)
    for (int64_t i = 0; i < N; i++) {
      float md = mean_delta[i] / B;
      float vd = 2.0f * var_delta[i] / B;
      float ve = var[i] > SEPS ? var[i] : SEPS;
      float sd = sqrtf(ve);
      float* dd = delta + (i + j * N) * bs;
      const float* xx = x + (i + j * N) * bs;
      for (int64_t k = 0; k < bs; k++) {
        float a = dd[k] / sd;
        float t = (xx[k] - mean[i]) * vd + md;
        dd[k] = a + t;
      }
    }
}

/* ---- TBaseLayer.batchNorm (nbaselayer.pas:336-370) --------------------------
 * output [groups][N][bs] in place: training: MeansAndVars, rolling update
 * (Multiply(1-m), then axpy(m, stat) as a saxpy FMA), CopyTo(x),
 * blockNormalize, copyTo(x_norm); otherwise blockNormalize with the rolling
 * statistics; then forwardScale (vsMulB) and forwardBias (vsAddB). */
void ora_batch_norm(float* out, int64_t groups, int64_t N, int64_t bs, const float* scales,
                    const float* biases, float* rolling_mean, float* rolling_variance,
                    float momentum, int32_t training, float* mean, float* variance, float* x,
                    float* x_norm, int32_t quirk) {
  const int64_t n = groups * N * bs;
  if (training) {
    ora_means_and_vars_q(out, groups, N, bs, mean, variance, quirk);
    const float keep = 1.0f - momentum;
    for (int64_t i = 0; i < N; i++) {
      rolling_mean[i] = rolling_mean[i] * keep;
      rolling_mean[i] = fmaf(momentum, mean[i], rolling_mean[i]);
      rolling_variance[i] = rolling_variance[i] * keep;
      rolling_variance[i] = fmaf(momentum, variance[i], rolling_variance[i]);
    }
    memcpy(x, out, sizeof(float) * n);
    ora_normalize(out, groups, N, bs, mean, variance);
    memcpy(x_norm, out, sizeof(float) * n);
  } else {
    ora_normalize(out, groups, N, bs, rolling_mean, rolling_variance);
  }
  ora_forward_scale(out, groups, N, bs, scales);
  ora_add_bias(N, out, bs, biases, 1, groups);
}

/* ---- convolutional layer with batch norm (training) ----------------------- */
void ora_conv_forward_train(int64_t batch, int64_t C, int64_t H, int64_t W, const float* input,
                            const float* weights, int64_t filters, int64_t kSize, int64_t stride,
                            int64_t padding, int64_t dilation, int32_t act, const float* scales,
                            const float* biases, float* rolling_mean, float* rolling_variance,
                            float momentum, int32_t training, float* mean, float* variance,
                            float* x, float* x_norm, float* workspace, float* out,
                            int32_t quirk) {
  /* state.input.Conv2D(weights, output, ...) (nConvolutionLayer.pas:508) */
  ora_conv2d(batch, C, H, W, input, weights, filters, kSize, kSize, padding, padding, stride,
             stride, dilation, dilation, workspace, out);
  const int64_t bs = (H + 2 * padding - (dilation * (kSize - 1) + 1)) / stride + 1;
  const int64_t bsw = (W + 2 * padding - (dilation * (kSize - 1) + 1)) / stride + 1;
  const int64_t blk = bs * bsw, n = batch * filters * blk;
  ora_batch_norm(out, batch, filters, blk, scales, biases, rolling_mean, rolling_variance,
                 momentum, training, mean, variance, x, x_norm, quirk);
  ora_activate(out, n, act);
}

int ora_conv_backward_bn(int64_t batch, int64_t C, int64_t H, int64_t W, const float* input,
                         const float* weights, int64_t filters, int64_t kSize, int64_t stride,
                         int64_t padding, int64_t dilation, int32_t act, const float* output,
                         float* delta, const float* scales, const float* x, const float* x_norm,
                         const float* mean, const float* variance, float* scale_updates,
                         float* mean_delta, float* variance_delta, float* weight_updates,
                         float* workspace, float* state_delta, int32_t quirk) {
  const int64_t oh = ora_conv_backward_oh(H, kSize, stride, padding, dilation);
  const int64_t ow = ora_conv_backward_oh(W, kSize, stride, padding, dilation);
  if (!oh || !ow) return -1;
  const int64_t blk = oh * ow;
  if (ora_gradient(output, batch * filters * blk, act, delta)) return -2;
  /* batchNormBack (nbaselayer.pas:372-395) */
  ora_add_dots(scale_updates, x_norm, delta, batch, filters, blk);
  ora_forward_scale(delta, batch, filters, blk, scales);
  ora_mean_var_delta_q(delta, x, mean, variance, batch, filters, blk, mean_delta, variance_delta,
                       quirk);
  ora_normalize_delta(x, mean, variance, mean_delta, variance_delta, delta, batch, filters, blk);
  return ora_conv_backward_core(batch, C, H, W, input, weights, filters, kSize, stride, padding,
                                dilation, delta, weight_updates, workspace, state_delta);
}

/* softmax (nsoftmaxlayer.pas:83-106) over n elements with stride. */
void ora_softmax(int64_t n, const float* in, float temp, int64_t stride, float* out) {
  if (n == 0) return;
  float largest = in[0];
  for (int64_t i = 1; i < n; i++)
    if (in[i * stride] > largest) largest = in[i * stride];
  float sum = 0.0f;
  for (int64_t i = 0; i < n; i++) {
    float e = (float)exp((double)((in[i * stride] - largest) / temp));
    sum = sum + e;
    out[i * stride] = e;
  }
  for (int64_t i = 0; i < n; i++) out[i * stride] = out[i * stride] / sum;
}

/* softmaxCrossEntropy (123-137) */
void ora_softmax_xent(int64_t n, const float* pred, const float* truth, float* delta,
                      float* error) {
  for (int64_t i = 0; i < n; i++) {
    float t = truth[i], p = pred[i];
    error[i] = t != 0.0f ? (float)(-log((double)(p > SEPS ? p : SEPS))) : 0.0f;
    delta[i] = t - p;
  }
}

/* vsClamp (ntensors.pas:5235-5250) */
void ora_clamp(float* x, int64_t n, float lo, float hi) {
  for (int64_t i = 0; i < n; i++) {
    if (x[i] < lo) x[i] = lo;
    else if (x[i] > hi) x[i] = hi;
  }
}

/* ------------------------------------------------------------------------ */
/* Feed-forward (connected) network train step                               */
/* ------------------------------------------------------------------------ */
/* Parameter / state layout per layer l (inputs I, outputs O), all float:
 *   W[O*I], b[O], dW[O*I], db[O], and when bn: scales[O], rolling_mean[O],
 *   rolling_var[O], dscales[O];  activations out[B*O], delta[B*O],
 *   x[B*O], x_norm[B*O], mean[O], var[O], mean_delta[O], var_delta[O]. */
typedef struct {
  int64_t I, O;
  int32_t act, bn;
  float *W, *b, *dW, *db, *scales, *rmean, *rvar, *dscales;
  float *out, *delta, *x, *xnorm, *mean, *var, *mdelta, *vdelta;
} ora_fc;

static void fc_forward(ora_fc* L, const float* in, int64_t B, float bn_momentum) {
  /* gemm(NT, batch, outputs, inputs, 1, X, inputs, W, inputs, 0, out, outputs) */
  ora_sgemm(101, 111, 112, B, L->O, L->I, 1.0f, in, L->I, L->W, L->I, 0.0f, L->out, L->O);
  if (L->bn) {
    ora_means_and_vars(L->out, B, L->O, 1, L->mean, L->var);
    for (int64_t i = 0; i < L->O; i++) { /* Multiply(1-m) then axpy(m, stat) */
      L->rmean[i] = L->rmean[i] * (1.0f - bn_momentum);
      L->rmean[i] = fmaf(bn_momentum, L->mean[i], L->rmean[i]);
      L->rvar[i] = L->rvar[i] * (1.0f - bn_momentum);
      L->rvar[i] = fmaf(bn_momentum, L->var[i], L->rvar[i]);
    }
    memcpy(L->x, L->out, sizeof(float) * B * L->O);
    ora_normalize(L->out, B, L->O, 1, L->mean, L->var);
    memcpy(L->xnorm, L->out, sizeof(float) * B * L->O);
    ora_forward_scale(L->out, B, L->O, 1, L->scales);
  }
  ora_add_bias(L->O, L->out, 1, L->b, 1, B);
  ora_activate(L->out, B * L->O, L->act);
}

static void fc_backward(ora_fc* L, const float* in, float* prev_delta, int64_t B) {
  ora_clamp(L->delta, B * L->O, -1.0f, 1.0f);
  ora_gradient(L->out, B * L->O, L->act, L->delta);
  ora_add_sums(L->db, L->delta, B, L->O, 1);
  if (L->bn) {
    ora_add_dots(L->dscales, L->xnorm, L->delta, B, L->O, 1);
    ora_forward_scale(L->delta, B, L->O, 1, L->scales);
    ora_mean_var_delta(L->delta, L->x, L->mean, L->var, B, L->O, 1, L->mdelta, L->vdelta);
    ora_normalize_delta(L->x, L->mean, L->var, L->mdelta, L->vdelta, L->delta, B, L->O, 1);
  }
  /* gemm(TN, outputs, inputs, batch, 1, delta, outputs, X, inputs, 1, dW, inputs) */
  ora_sgemm(101, 112, 111, L->O, L->I, B, 1.0f, L->delta, L->O, in, L->I, 1.0f, L->dW, L->I);
  if (prev_delta) /* gemm(NN, batch, inputs, outputs, 1, delta, outputs, W, inputs, 1, prev) */
    ora_sgemm(101, 111, 111, B, L->I, L->O, 1.0f, L->delta, L->O, L->W, L->I, 1.0f,
              prev_delta, L->I);
}

static void axpy_(int64_t n, float a, const float* x, float* y) {
  for (int64_t i = 0; i < n; i++) y[i] = fmaf(a, x[i], y[i]); /* saxpy_avx2 */
}
static void scal_(int64_t n, float a, float* x) {
  for (int64_t i = 0; i < n; i++) x[i] = a * x[i]; /* sscal vmulps */
}

/* TConnectedLayer.update (nconnectedlayer.pas:324-359) and
 * TConvolutionalLayer.update (nConvolutionLayer.pas:673-705), with
 * lrb = learning_rate / batch and ndb = -decay * batch computed by the caller:
 *   biases.axpy(lrb, bias_updates); bias_updates *= momentum;
 *   scales.axpy(lrb, scale_updates); scale_updates *= momentum  (if scales);
 *   weight_updates.axpy(ndb, weights); weights.axpy(lrb, weight_updates);
 *   weight_updates *= momentum. */
void ora_sgd_update(int64_t nw, float* W, float* dW, int64_t n, float* b, float* db,
                    float* scales, float* dscales, float lrb, float ndb, float momentum) {
  axpy_(n, lrb, db, b);
  scal_(n, momentum, db);
  if (scales) {
    axpy_(n, lrb, dscales, scales);
    scal_(n, momentum, dscales);
  }
  axpy_(nw, ndb, W, dW);
  axpy_(nw, lrb, dW, W);
  scal_(nw, momentum, dW);
}

static void fc_update(ora_fc* L, float lr, float momentum, float decay, int64_t batch) {
  ora_sgd_update(L->O * L->I, L->W, L->dW, L->O, L->b, L->db, L->bn ? L->scales : NULL,
                 L->bn ? L->dscales : NULL, lr / (float)batch, -decay * (float)batch, momentum);
}

/* One TNNet.Propagate + update over a stack of connected layers followed by
 * a softmax layer (nnet.pas:405-450, 371-403).  `buf` holds, per layer, the
 * arrays described above packed back to back in the order
 *   W b dW db [scales rmean rvar dscales] out delta [x xnorm mean var mdelta vdelta]
 * plus, at the end, softmax out[B*C], delta[B*C], loss[B*C].  Returns the
 * cost (loss.Sum() via vssum_avx2; TNNet.cost divides by 1 cost layer). */
float ora_mlp_train_step(int32_t nlayers, const int64_t* widths, const int32_t* acts,
                         int32_t bn, int64_t B, const float* X, const float* truth, float lr,
                         float momentum, float decay, float* buf) {
  ora_fc L[32];
  if (nlayers > 32) return NAN;
  float* p = buf;
  for (int l = 0; l < nlayers; l++) {
    ora_fc* f = &L[l];
    f->I = widths[l];
    f->O = widths[l + 1];
    f->act = acts[l];
    f->bn = bn;
    int64_t IO = f->I * f->O, O = f->O, BO = B * f->O;
    f->W = p; p += IO;
    f->b = p; p += O;
    f->dW = p; p += IO;
    f->db = p; p += O;
    if (bn) {
      f->scales = p; p += O;
      f->rmean = p; p += O;
      f->rvar = p; p += O;
      f->dscales = p; p += O;
    }
    f->out = p; p += BO;
    f->delta = p; p += BO;
    if (bn) {
      f->x = p; p += BO;
      f->xnorm = p; p += BO;
      f->mean = p; p += O;
      f->var = p; p += O;
      f->mdelta = p; p += O;
      f->vdelta = p; p += O;
    }
  }
  const int64_t C = widths[nlayers];
  float* sm_out = p; p += B * C;
  float* sm_delta = p; p += B * C;
  float* sm_loss = p; p += B * C;

  /* forward: each layer's delta is zeroed first (nnet.pas:287-296) */
  const float* in = X;
  for (int l = 0; l < nlayers; l++) {
    memset(L[l].delta, 0, sizeof(float) * B * L[l].O);
    fc_forward(&L[l], in, B, 0.05f); /* bnMomentum := 0.05 (nconnectedlayer.pas:67) */
    in = L[l].out;
  }
  /* softmax layer: groups = 1, temperature 1 */
  for (int64_t b = 0; b < B; b++) ora_softmax(C, in + b * C, 1.0f, 1, sm_out + b * C);
  ora_softmax_xent(B * C, sm_out, truth, sm_delta, sm_loss);
  float cost = ora_vssum(B * C, sm_loss);

  /* backward: softmax adds its delta into the previous layer's delta */
  for (int64_t i = 0; i < B * C; i++)
    L[nlayers - 1].delta[i] = L[nlayers - 1].delta[i] + sm_delta[i];
  for (int l = nlayers - 1; l >= 0; l--) {
    const float* lin = l == 0 ? X : L[l - 1].out;
    float* prev_delta = l == 0 ? NULL : L[l - 1].delta; /* state.delta = nil for layer 0 */
    fc_backward(&L[l], lin, prev_delta, B);
  }
  /* update (constant learning-rate policy) */
  for (int l = 0; l < nlayers; l++) fc_update(&L[l], lr, momentum, decay, B);
  return cost;
}

int64_t ora_mlp_buffer_floats(int32_t nlayers, const int64_t* widths, int32_t bn, int64_t B) {
  int64_t n = 0;
  for (int l = 0; l < nlayers; l++) {
    int64_t I = widths[l], O = widths[l + 1];
    n += 2 * I * O + 2 * O + 2 * B * O;
    if (bn) n += 4 * O + 2 * B * O + 4 * O;
  }
  return n + 3 * B * widths[nlayers];
}
