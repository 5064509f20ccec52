/*
 * tns_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of Tensorium's fp32 SGEMM + im2col-convolution hot path
 * (reference: /root/reference/source, Free Pascal + inline AVX2 asm).  Used
 * only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as
 * the checker — never by the product path (libtensorium_hip.so).
 *
 * PARITY UNPINNED by reference artefacts: the reference ships no tests,
 * golden vectors or fixtures, and its Pascal sources cannot be compiled here
 * (no fpc/lazbuild/dcc).  This restatement is pinned instead by hand-derived
 * known-answer vectors that exercise the reference's documented operation
 * order (tests/golden/), by exact small-integer arithmetic, and by float64
 * cross-checks.  See DESIGN.md §Oracle.
 *
 * Every function cites the reference lines it restates.
 */
#ifndef TNS_ORACLE_H
#define TNS_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* worker count of the restated steroids TOPool (steroids.pas:281-296:
 * max(ProcessorCount, 4) by default).  n<=0 restores the default. */
void    ora_set_threads(int n);
int     ora_get_threads(void);

/* saxpy_avx2 (ntensors.pas:1308-1435): y[i] = fma(a, x[i], y[i]) for every i
 * (the 4x8, 8 and scalar loops all use vfmadd231). */
void    ora_saxpy(int64_t N, float a, const float* x, float* y);
/* sdot_avx2 (ntensors.pas:1233-1306): 8 FMA lanes, masked FMA tail,
 * s_l = lane_l + lane_{l+4}, result (s0+s1)+(s2+s3). */
float   ora_sdot(int64_t N, const float* A, const float* B);

/* cblas_sgemm (ntensors.pas:2231-2286) with sgemm_nn/nt/tn/tt
 * (1957-2206), threaded over rows like MP.&For (steroids.pas:606-641). */
void    ora_sgemm(int32_t order, int32_t transA, int32_t transB,
                  int64_t M, int64_t N, int64_t K, float alpha,
                  const float* A, int64_t lda, const float* B, int64_t ldb,
                  float beta, float* C, int64_t ldc);
/* Same computation restricted to rows [row0,row1) of C (CPU-baseline sample). */
void    ora_sgemm_rows(int32_t transA, int32_t transB, int64_t row0, int64_t row1,
                       int64_t M, int64_t N, int64_t K, float alpha,
                       const float* A, int64_t lda, const float* B, int64_t ldb,
                       float beta, float* C, int64_t ldc);
/* cblas_sgemm_batch_strided (ntensors.pas:2288-2304). */
void    ora_sgemm_batch_strided(int32_t order, int32_t transA, int32_t transB,
                                int64_t M, int64_t N, int64_t K, float alpha,
                                const float* A, int64_t lda, int64_t strideA,
                                const float* B, int64_t ldb, int64_t strideB,
                                float beta, float* C, int64_t ldc, int64_t strideC,
                                int64_t batch);

/* sim2Col (ntensors.pas:11415-11491) and sim2colStridedBatched (11493-11532). */
void    ora_im2col(int64_t C, int64_t H, int64_t W, int64_t kH, int64_t kW,
                   int64_t padH, int64_t padW, int64_t strideY, int64_t strideX,
                   int64_t dilY, int64_t dilX, const float* im, int64_t imOffset,
                   float* col, int64_t colOffset);
void    ora_im2col_strided_batched(int64_t C, int64_t H, int64_t W, int64_t kH, int64_t kW,
                   int64_t padH, int64_t padW, int64_t strideY, int64_t strideX,
                   int64_t dilY, int64_t dilX, const float* im, int64_t imStride,
                   int64_t imOffset, float* col, int64_t colStride, int64_t colOffset,
                   int64_t batch);
/* c2i / scol2im (ntensors.pas:11650-11763), single-threaded order, and
 * scol2imStridedBatched (11833-11879). */
void    ora_col2im(int64_t C, int64_t H, int64_t W, int64_t kH, int64_t kW,
                   int64_t padH, int64_t padW, int64_t strideY, int64_t strideX,
                   int64_t dilY, int64_t dilX, const float* col, int64_t colOffset,
                   float* im, int64_t imOffset);
void    ora_col2im_strided_batched(int64_t C, int64_t H, int64_t W, int64_t kH, int64_t kW,
                   int64_t padH, int64_t padW, int64_t strideY, int64_t strideX,
                   int64_t dilY, int64_t dilX, const float* col, int64_t colStride,
                   int64_t colOffset, float* im, int64_t imStride, int64_t imOffset,
                   int64_t batch);

/* vsAddB (ntensors.pas:4066-4093) via TTensor.forwardBias (7709-7727). */
void    ora_add_bias(int64_t N, float* a, int64_t blockSize, const float* b,
                     int64_t incb, int64_t batch);
/* addSums (ntensors.pas:7729-7781), non-AVX summation order. */
void    ora_backward_bias(int64_t nDst, float* dst, int64_t groups, int64_t blockSize,
                          const float* src);

/* activate_array / gradient_array (nactivation.pas:508-717), scalar
 * formulas (272-501); leaky uses the AVX2 leaky_array constant 0.1f. */
int     ora_activate(float* x, int64_t N, int32_t act);
int     ora_gradient(const float* x, int64_t N, int32_t act, float* delta);

/* TTensor.Conv2D (ntensors.pas:8252-8349): im2col (unless 1x1/s1/d1) then
 * per-image gemm(NN, filters, outHW, C*k^2, 1, W, .., 0, out_b, ..). */
void    ora_conv2d(int64_t batch, int64_t C, int64_t H, int64_t W,
                   const float* input, const float* weights, int64_t filters,
                   int64_t kH, int64_t kW, int64_t wPadding, int64_t hPadding,
                   int64_t xStride, int64_t yStride, int64_t xDilation, int64_t yDilation,
                   float* workspace, float* out);
/* TConvolutionalLayer.forward after fuseBatchNorm (nConvolutionLayer.pas:
 * 457-569): Conv2D -> forwardBias -> activate. */
void    ora_conv_forward(int64_t batch, int64_t C, int64_t H, int64_t W,
                         const float* input, const float* weights, const float* biases,
                         int64_t filters, int64_t kSize, int64_t stride, int64_t padding,
                         int64_t dilation, int32_t act, float* workspace, float* out);
/* TConvolutionalLayer.backward without batch-norm (nConvolutionLayer.pas:
 * 571-671): delta *= f'(output); bias_updates.addSums(delta); im2col(input);
 * weight_updates += delta_b.col_b^T per image (NT, beta 1); if state_delta:
 * col = W^T.delta (TN strided batched, beta 0) and col2im-accumulate.
 * The backward im2col / col2im pad with padding*dilation (640, 665); returns
 * -1 when that geometry does not give the layer's outH x outW columns. */
int     ora_conv_backward(int64_t batch, int64_t C, int64_t H, int64_t W,
                          const float* input, const float* weights, int64_t filters,
                          int64_t kSize, int64_t stride, int64_t padding, int64_t dilation,
                          int32_t act, const float* output, float* delta, float* bias_updates,
                          float* weight_updates, float* workspace, float* state_delta);
/* output rows of the backward's im2col (padding*dilation) when they equal
 * the layer's outH (no dilation), else 0 (refused geometry) */
int64_t ora_conv_backward_oh(int64_t H, int64_t kSize, int64_t stride, int64_t padding,
                             int64_t dilation);
int     ora_conv_backward_core(int64_t batch, int64_t C, int64_t H, int64_t W,
                               const float* input, const float* weights, int64_t filters,
                               int64_t kSize, int64_t stride, int64_t padding, int64_t dilation,
                               const float* delta, float* weight_updates, float* workspace,
                               float* state_delta);
/* TConvolutionalLayer.forward in training with batch norm (nConvolutionLayer.
 * pas:457-569 -> TBaseLayer.batchNorm, nbaselayer.pas:336-370): Conv2D, then
 * (training) MeansAndVars, rolling updates with bnMomentum, x := output,
 * blockNormalize, x_norm := output, or (inference) blockNormalize with the
 * rolling statistics; forwardScale, forwardBias, activate. */
void    ora_conv_forward_train(int64_t batch, int64_t C, int64_t H, int64_t W,
                               const float* input, const float* weights, int64_t filters,
                               int64_t kSize, int64_t stride, int64_t padding, int64_t dilation,
                               int32_t act, const float* scales, const float* biases,
                               float* rolling_mean, float* rolling_variance, float momentum,
                               int32_t training, float* mean, float* variance, float* x,
                               float* x_norm, float* workspace, float* out, int32_t quirk);
/* TBaseLayer.batchNorm (nbaselayer.pas:336-370) over out [groups][N][bs] in
 * place (see tns_oracle_train.c). */
void ora_batch_norm(float* out, int64_t groups, int64_t N, int64_t bs, const float* scales,
                    const float* biases, float* rolling_mean, float* rolling_variance,
                    float momentum, int32_t training, float* mean, float* variance, float* x,
                    float* x_norm, int32_t quirk);

/* TConvolutionalLayer.backward with batch norm: Derivative, batchNormBack
 * (nbaselayer.pas:372-395: addDots into scale_updates, forwardScale,
 * MeansAndVarsDelta, normalizeDelta — no bias_updates term), then the
 * weight and input gradients as ora_conv_backward. */
int     ora_conv_backward_bn(int64_t batch, int64_t C, int64_t H, int64_t W,
                             const float* input, const float* weights, int64_t filters,
                             int64_t kSize, int64_t stride, int64_t padding, int64_t dilation,
                             int32_t act, const float* output, float* delta,
                             const float* scales, const float* x, const float* x_norm,
                             const float* mean, const float* variance, float* scale_updates,
                             float* mean_delta, float* variance_delta, float* weight_updates,
                             float* workspace, float* state_delta, int32_t quirk);
/* fuseBatchNorm (nConvolutionLayer.pas:102-126). */
void    ora_fuse_batchnorm(int64_t filters, int64_t filterSize, float* weights,
                           float* biases, const float* scales, const float* rollingMean,
                           const float* rollingVariance);

/* ---- batch-norm / softmax / SGD / connected-layer train step -------------
 * (tns_oracle_train.c; tolerance oracle: exp/ln/Power evaluated in double) */
float   ora_vssum(int64_t n, const float* a);
void    ora_sgd_update(int64_t nw, float* W, float* dW, int64_t n, float* b, float* db,
                       float* scales, float* dscales, float lrb, float ndb, float momentum);
void    ora_means_and_vars(const float* x, int64_t groups, int64_t N, int64_t bs, float* means,
                           float* vars);
void    ora_means_and_vars_q(const float* x, int64_t groups, int64_t N, int64_t bs,
                             float* means, float* vars, int quirk);
float   ora_srss(int64_t n, float mean, const float* a, int quirk);
void    ora_normalize(float* x, int64_t groups, int64_t N, int64_t bs, const float* means,
                      const float* vars);
void    ora_forward_scale(float* x, int64_t groups, int64_t N, int64_t bs, const float* scales);
void    ora_add_dots(float* dst, const float* a, const float* b, int64_t groups, int64_t N,
                     int64_t bs);
void    ora_add_sums(float* dst, const float* src, int64_t groups, int64_t N, int64_t bs);
void    ora_mean_var_delta(const float* delta, const float* x, const float* mean,
                           const float* var, int64_t groups, int64_t N, int64_t bs,
                           float* mean_delta, float* var_delta);
void    ora_mean_var_delta_q(const float* delta, const float* x, const float* mean,
                             const float* var, int64_t groups, int64_t N, int64_t bs,
                             float* mean_delta, float* var_delta, int quirk);
/* sVarinceDelta_avx (ntensors.pas:8721-8757): one block's sum of
 * (x - mean) * delta in the reference's 8-lane order (quirk: see .c) */
float   ora_var_delta_avx(int64_t n, float mean, const float* delta, const float* x, int quirk);
void    ora_normalize_delta(const float* x, const float* mean, const float* var,
                            const float* mean_delta, const float* var_delta, float* delta,
                            int64_t groups, int64_t N, int64_t bs);
void    ora_softmax(int64_t n, const float* in, float temp, int64_t stride, float* out);
void    ora_softmax_xent(int64_t n, const float* pred, const float* truth, float* delta,
                         float* error);
void    ora_clamp(float* x, int64_t n, float lo, float hi);
float   ora_mlp_train_step(int32_t nlayers, const int64_t* widths, const int32_t* acts,
                           int32_t bn, int64_t B, const float* X, const float* truth, float lr,
                           float momentum, float decay, float* buf);
int64_t ora_mlp_buffer_floats(int32_t nlayers, const int64_t* widths, int32_t bn, int64_t B);

/* non-convolutional YOLOv3 layers (forward): shortcut = addvv + activation
 * (naddlayer.pas:667-720), upsample (nupsamplelayer.pas:83-113), yolo
 * (nyololayer.pas:786-825) */
int     ora_shortcut(int64_t n, const float* a, const float* b, float* out, int32_t act);
void    ora_upsample(int64_t planes, int64_t h, int64_t w, int64_t stride, float scale,
                     const float* in, float* out);
void    ora_yolo_forward(int64_t batch, int64_t anchors, int64_t classes, int64_t hw,
                         const float* in, float* out);

/* counter-based synthetic data (splitmix64 -> u in [lo,hi)), keyed by
 * (seed, stream, index) so CPU and GPU regenerate identical tensors. */
void    ora_fill_uniform(float* x, int64_t n, uint64_t seed, uint64_t stream,
                         float lo, float hi);

#ifdef __cplusplus
}
#endif
#endif
