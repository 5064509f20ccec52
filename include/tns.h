/*
 * tns.h — C ABI of libtensorium_hip.so, the MI355X (gfx950) backend for
 * Tensorium's fp32 SGEMM + im2col-convolution hot path.
 *
 * Two boundaries, both plain cdecl (SysV x86-64), no C++ or torch types:
 *
 *  A. Op-table drop-ins (host pointers).  Each function has exactly the
 *     parameter list of one TTensor<Single> class-var procedure pointer
 *     (source/ntensors.pas:345-385, bound in TTensorOps.initSingle,
 *     ntensors.pas:12651-12758).  A Pascal maintainer assigns e.g.
 *       TSingleTensor.gemm := @tns_cblas_sgemm;
 *     after initSingle, exactly like the USE_OPENBLAS / USE_MKL overrides at
 *     ntensors.pas:12735-12756.  These return void (the Pascal pointer types
 *     have no status channel): a failure is recorded in a thread-local error
 *     string read with tns_last_error(); an optional fatal hook
 *     (tns_set_error_hook) lets the binding raise like SAFE_CALL does
 *     (nncuda.pas:216-275).  The shim stages host buffers through device
 *     scratch that it owns; results are complete when the call returns.
 *
 *  B. Device-resident backend (device pointers + element offsets), the HIP
 *     twin of TNNCuda<T> (source/nncuda.pas:35-157) / TNNOpenCL<T>
 *     (source/nnopencl.pas:222-319).  Calls are stream-ordered and
 *     asynchronous on the context's stream; tns_hip_finish() synchronises,
 *     as TNNCuda.finish does (nncuda.pas:1575).  Every call returns a status
 *     (0 = TNS_OK); tns_last_error() carries the message.
 *
 * Enumerations keep the reference's ordinal values: CBLAS_LAYOUT /
 * CBLAS_TRANSPOSE (ntensors.pas:106-128, {$Z4} => 4-byte enums) and
 * TActivationType (ntypes.pas:66-71).
 */
#ifndef TNS_H
#define TNS_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TNS_ABI_VERSION 1

/* ---- enums (reference ordinals) ---------------------------------------- */
enum { TNS_CblasRowMajor = 101, TNS_CblasColMajor = 102 };           /* ntensors.pas:106-107 */
enum { TNS_CblasNoTrans = 111, TNS_CblasTrans = 112 };               /* ntensors.pas:119-120 */

/* TActivationType, ntypes.pas:66-71 */
enum {
  TNS_acLOGISTIC = 0, TNS_acRELU = 1, TNS_acRELU6 = 2, TNS_acRELIE = 3,
  TNS_acLINEAR = 4, TNS_acRAMP = 5, TNS_acTANH = 6, TNS_acPLSE = 7,
  TNS_acREVLEAKY = 8, TNS_acLEAKY = 9, TNS_acELU = 10, TNS_acLOGGY = 11,
  TNS_acSTAIR = 12, TNS_acHARDTAN = 13, TNS_acLHTAN = 14, TNS_acSELU = 15
};

/* status codes (boundary B) */
enum {
  TNS_OK = 0,
  TNS_ERR_ARG = 1,        /* invalid argument (shape, enum, null pointer) */
  TNS_ERR_HIP = 2,        /* a HIP runtime call failed                    */
  TNS_ERR_NOMEM = 3,      /* device allocation failed                     */
  TNS_ERR_UNSUPPORTED = 4 /* enum value the backend does not implement    */
};

/* ---- library / error channel ------------------------------------------- */
int         tns_abi_version(void);
const char* tns_last_error(void);          /* thread-local, "" when none   */
void        tns_clear_error(void);
typedef void (*tns_error_hook_t)(int code, const char* msg);
void        tns_set_error_hook(tns_error_hook_t hook);
int         tns_device_count(void);

/* =========================================================================
 * A. Op-table drop-ins (host pointers)
 * ========================================================================= */

/* TTensor<Single>.gemm  — ntensors.pas:345-347, CPU impl cblas_sgemm
 * ntensors.pas:2231-2286.  Row-major only (Order is accepted and ignored,
 * as the reference ignores it).  beta<>1 pre-scales C (beta=0 => 0*C, so
 * NaN/Inf in C propagate, ntensors.pas:2259-2261). */
void tns_cblas_sgemm(int32_t Order, int32_t TransA, int32_t TransB,
                     int64_t M, int64_t N, int64_t K, float ALPHA,
                     const float* A, int64_t lda, const float* B, int64_t ldb,
                     float BETA, float* C, int64_t ldc);

/* TTensor<Single>.gemmStridedBatched — ntensors.pas:348-351, CPU impl
 * cblas_sgemm_batch_strided ntensors.pas:2288-2304. */
void tns_cblas_sgemm_batch_strided(int32_t Layout, int32_t TransA, int32_t TransB,
                                   int64_t M, int64_t N, int64_t K, float alpha,
                                   const float* A, int64_t lda, int64_t strideA,
                                   const float* B, int64_t ldb, int64_t strideB,
                                   float beta, float* C, int64_t ldc, int64_t strideC,
                                   int64_t batch_size);

/* TTensor<Single>.im2Colvv — ntensors.pas:362-366, CPU impl sim2Col
 * ntensors.pas:11415-11491.  multiThread is a Pascal boolean (1 byte). */
void tns_im2col(int64_t aChannels, int64_t aHeight, int64_t aWidth,
                int64_t kernelHeight, int64_t kernelWidth, int64_t padHeight,
                int64_t padWidth, int64_t strideY, int64_t strideX,
                int64_t dilationY, int64_t dilationX,
                const float* inData, int64_t inOffset,
                float* outData, int64_t outOffset, uint8_t multiThread);

/* TTensor<Single>.col2imvv — ntensors.pas:367-371, CPU impl scol2im
 * ntensors.pas:11717-11763 (accumulates into im; never zeroes it). */
void tns_col2im(int64_t aChannels, int64_t aHeight, int64_t aWidth,
                int64_t kernelHeight, int64_t kernelWidth, int64_t padHeight,
                int64_t padWidth, int64_t strideY, int64_t strideX,
                int64_t dilationY, int64_t dilationX,
                const float* inData, int64_t inOffset,
                float* outData, int64_t outOffset, int64_t batch,
                uint8_t multiThread);

/* TTensor<Single>.im2colStridedBatchedvv — ntensors.pas:372-378, CPU impl
 * sim2colStridedBatched ntensors.pas:11493-11532. */
void tns_im2col_strided_batched(int64_t aChannels, int64_t aHeight, int64_t aWidth,
                                int64_t kernelHeight, int64_t kernelWidth,
                                int64_t padHeight, int64_t padWidth,
                                int64_t strideY, int64_t strideX,
                                int64_t dilationY, int64_t dilationX,
                                const float* im, int64_t imStride, int64_t imOffset,
                                float* col, int64_t colStride, int64_t colOffset,
                                int64_t batchCount);

/* TTensor<Single>.col2imStridedBatchedvv — ntensors.pas:379-385, CPU impl
 * scol2imStridedBatched ntensors.pas:11833-11879. */
void tns_col2im_strided_batched(int64_t aChannels, int64_t aHeight, int64_t aWidth,
                                int64_t kernelHeight, int64_t kernelWidth,
                                int64_t padHeight, int64_t padWidth,
                                int64_t strideY, int64_t strideX,
                                int64_t dilationY, int64_t dilationX,
                                const float* inData, int64_t inStride, int64_t inOffset,
                                float* outData, int64_t outStride, int64_t outOffset,
                                int64_t batchCount);

/* =========================================================================
 * B. Device-resident backend (TNNCuda<T> twin).  Pointers are device
 *    pointers (hipMalloc / torch); offsets are in ELEMENTS, as TCUMem+offset.
 * ========================================================================= */
typedef struct tns_ctx tns_ctx;

/* TNNCuda.Create(deviceIndex) — nncuda.pas:448-467.  Creates its own
 * non-blocking stream unless one is attached with tns_hip_set_stream. */
int  tns_hip_create(int32_t deviceIndex, tns_ctx** out);
int  tns_hip_destroy(tns_ctx* ctx);
int  tns_hip_set_stream(tns_ctx* ctx, void* hipStream);   /* hipStream_t */
/* The context's stream, after it has been made to wait for any pipelined
 * conv-backward dW products still pending on the side stream
 * (TNS_OPT_BWD_OVERLAP = 2), so work enqueued on it sees their results. */
void* tns_hip_get_stream(tns_ctx* ctx);   /* NULL on error: tns_last_error() */
/* Pipelined conv backward (TNS_OPT_BWD_OVERLAP = 2): the number of dW
 * products still pending on the side stream (0 once joined; -1 for a null
 * context).  Diagnostic: it shows which calls left the pipeline running. */
int  tns_hip_pending_dw(tns_ctx* ctx);
int  tns_hip_finish(tns_ctx* ctx);                         /* nncuda.pas:1575 */

/* createDeviceBuffer / freeDeviceBuffer / writeBuffer / readBuffer —
 * nncuda.pas:104-107 (sizes in BYTES for copies, as the reference). */
int  tns_hip_malloc(tns_ctx* ctx, int64_t nElements, float** out);
int  tns_hip_free(tns_ctx* ctx, float* p);
int  tns_hip_write_buffer(tns_ctx* ctx, float* dev, int64_t bytes, const void* host);
int  tns_hip_read_buffer(tns_ctx* ctx, const float* dev, int64_t bytes, void* host);

/* TNNCuda.gemm — nncuda.pas:624-725.  Same semantics as cblas_sgemm. */
int tns_hip_gemm(tns_ctx* ctx, uint8_t transA, uint8_t transB,
                 int64_t M, int64_t N, int64_t K, float ALPHA,
                 const float* A, int64_t aOffset, int64_t lda,
                 const float* B, int64_t bOffset, int64_t ldb,
                 float BETA, float* C, int64_t cOffset, int64_t ldc);

/* TNNCuda.gemmStridedBatched — nncuda.pas:809.  strideA = 0 shares A
 * (conv weights, nConvolutionLayer.pas:1078). */
int tns_hip_gemm_strided_batched(tns_ctx* ctx, uint8_t transA, uint8_t transB,
                                 int64_t M, int64_t N, int64_t K, float ALPHA,
                                 const float* A, int64_t aOffset, int64_t lda, int64_t strideA,
                                 const float* B, int64_t bOffset, int64_t ldb, int64_t strideB,
                                 float BETA, float* C, int64_t cOffset, int64_t ldc, int64_t strideC,
                                 int64_t batchCount);

/* TNNCuda.gemmBatched — nncuda.pas:727-760 (cublasSgemmBatched_64 over
 * arrays of matrix pointers).  A, B, C are arrays of batchCount pointers,
 * device-resident as the reference builds them with writeBuffer
 * (nConvolutionLayer.pas:1083-1085) or host-resident; the element offsets
 * apply to every entry.  The arrays are read in stream order (the call
 * waits for them); equally spaced entries whose GEMMs are independent (no
 * C entry overlaps another C entry or any A / B entry) run as one
 * strided-batched launch, all others GEMM by GEMM in array order, so an
 * entry may read what an earlier one wrote.  Results as tns_hip_gemm. */
int tns_hip_gemm_batched(tns_ctx* ctx, uint8_t transA, uint8_t transB,
                         int64_t M, int64_t N, int64_t K, float ALPHA,
                         const float* const* A, int64_t aOffset, int64_t lda,
                         const float* const* B, int64_t bOffset, int64_t ldb,
                         float BETA, float* const* C, int64_t cOffset, int64_t ldc,
                         int64_t batchCount);

/* TNNCuda.im2col — nncuda.pas:1144 (output layout = CPU sim2Col). */
int tns_hip_im2col(tns_ctx* ctx, int64_t aChannels, int64_t aHeight, int64_t aWidth,
                   int64_t kernelHeight, int64_t kernelWidth, int64_t padHeight, int64_t padWidth,
                   int64_t strideY, int64_t strideX, int64_t dilationY, int64_t dilationX,
                   const float* im, int64_t imOffset, float* col, int64_t colOffset);

/* Strided-batched im2col (one launch for the whole batch). */
int tns_hip_im2col_strided_batched(tns_ctx* ctx, int64_t aChannels, int64_t aHeight, int64_t aWidth,
                   int64_t kernelHeight, int64_t kernelWidth, int64_t padHeight, int64_t padWidth,
                   int64_t strideY, int64_t strideX, int64_t dilationY, int64_t dilationX,
                   const float* im, int64_t imStride, int64_t imOffset,
                   float* col, int64_t colStride, int64_t colOffset, int64_t batchCount);

/* TNNCuda.col2im — nncuda.pas:1212.  Race-free gather; per-pixel sum in the
 * CPU scol2im's ascending kernel-index order (ntensors.pas:11650-11715),
 * including its dilation formula (input_row := (kernel_row-pad)*dil). */
int tns_hip_col2im(tns_ctx* ctx, int64_t aChannels, int64_t aHeight, int64_t aWidth,
                   int64_t kernelHeight, int64_t kernelWidth, int64_t padHeight, int64_t padWidth,
                   int64_t strideY, int64_t strideX, int64_t dilationY, int64_t dilationX,
                   const float* col, int64_t colOffset, float* im, int64_t imOffset);

int tns_hip_col2im_strided_batched(tns_ctx* ctx, int64_t aChannels, int64_t aHeight, int64_t aWidth,
                   int64_t kernelHeight, int64_t kernelWidth, int64_t padHeight, int64_t padWidth,
                   int64_t strideY, int64_t strideX, int64_t dilationY, int64_t dilationX,
                   const float* col, int64_t colStride, int64_t colOffset,
                   float* im, int64_t imStride, int64_t imOffset, int64_t batchCount);

/* TNNCuda.forwardBias — nncuda.pas:582.  dst[(b*srcSize+i)*bs + j] += src[i*incb],
 * bs = dstSize/(srcSize*batch)  (vsAddB, ntensors.pas:4066-4093). */
int tns_hip_forward_bias(tns_ctx* ctx, int64_t dstSize, float* dst, int64_t offset,
                         int64_t srcSize, const float* src, int64_t incb, int64_t batch);

/* TNNCuda.backwardBias — dst[i] += sum_b sum_j src[(b*dstSize+i)*bs + j]
 * (addSums, ntensors.pas:7729-7781). */
int tns_hip_backward_bias(tns_ctx* ctx, int64_t dstSize, float* dst, int64_t srcSize,
                          const float* src, int64_t srcOffset, int64_t incb, int64_t batch);

/* TNNCuda.ActivateArray / DeriveArray — nncuda.pas:524, 562; formulas
 * nactivation.pas:272-501, 508-717. */
int tns_hip_activate_array(tns_ctx* ctx, int64_t N, float* x, int64_t offset, int32_t activation);
int tns_hip_derive_array(tns_ctx* ctx, int64_t N, const float* x, int64_t offset,
                         int32_t activation, float* delta);

/* BLAS-1 / elementwise support (TNNCuda.axpy/scale/fill/copy/clamp). */
int tns_hip_axpy(tns_ctx* ctx, int64_t N, float a, const float* x, int64_t xOffset, int64_t incx,
                 float* y, int64_t yOffset, int64_t incy);
int tns_hip_scale(tns_ctx* ctx, int64_t N, float a, float* x, int64_t stride);
/* TConnectedLayer.update (nconnectedlayer.pas:324-359) /
 * TConvolutionalLayer.update (nConvolutionLayer.pas:673-705) in one pass:
 * biases += lrOverBatch*bias_updates, bias_updates *= momentum, the same for
 * scales (NULL pair when the layer has no batch norm), weight_updates +=
 * negDecayTimesBatch*weights, weights += lrOverBatch*weight_updates,
 * weight_updates *= momentum (each axpy one FMA, each scale one multiply).
 * The caller computes lrOverBatch = learning_rate / batch and
 * negDecayTimesBatch = -decay * batch in single precision as the reference. */
int tns_hip_sgd_update(tns_ctx* ctx, int64_t nWeights, float* weights, float* weight_updates,
                       int64_t n, float* biases, float* bias_updates, float* scales,
                       float* scale_updates, float lrOverBatch, float negDecayTimesBatch,
                       float momentum);
int tns_hip_fill(tns_ctx* ctx, int64_t N, float* x, int64_t offset, float val, int64_t stride);
int tns_hip_copy(tns_ctx* ctx, int64_t N, const float* src, int64_t srcOffset, int64_t inca,
                 float* dst, int64_t dstOffset, int64_t incb);
int tns_hip_clamp(tns_ctx* ctx, int64_t N, float alpha, const float* src, float* dst,
                  int64_t stride, int64_t offset);
/* TNNCuda.addvv / subvv / mulvv / fmavv (nncuda.pas:120-123):
 * dst[i*incc] = src1[i*inca] op src2[i*incb] (offsets in elements); fmavv:
 * src1*src2 rounded, then + src3 rounded (no fused multiply-add, as the CPU
 * sfmavss).  fmavss (nncuda.pas:137): dst = src*scalar + bias over N
 * contiguous elements at offset.  inverseSqrt (nncuda.pas:151):
 * dst = 1/sqrt(max(src, 1e-6)) strided; alpha unused (as the reference). */
int tns_hip_addvv(tns_ctx* ctx, int64_t N, const float* src1, int64_t src1Offset, int64_t inca,
                  const float* src2, int64_t src2Offset, int64_t incb, float* dst,
                  int64_t dstOffset, int64_t incc);
int tns_hip_subvv(tns_ctx* ctx, int64_t N, const float* src1, int64_t src1Offset, int64_t inca,
                  const float* src2, int64_t src2Offset, int64_t incb, float* dst,
                  int64_t dstOffset, int64_t incc);
int tns_hip_mulvv(tns_ctx* ctx, int64_t N, const float* src1, int64_t src1Offset, int64_t inca,
                  const float* src2, int64_t src2Offset, int64_t incb, float* dst,
                  int64_t dstOffset, int64_t incc);
int tns_hip_fmavv(tns_ctx* ctx, int64_t N, const float* src1, int64_t src1Offset, int64_t inca,
                  const float* src2, int64_t src2Offset, int64_t incb, const float* src3,
                  int64_t src3Offset, int64_t incc, float* dst, int64_t dstOffset,
                  int64_t incd);
int tns_hip_fmavss(tns_ctx* ctx, int64_t N, const float* src, int64_t offset, float scalar,
                   float bias, float* dst);
int tns_hip_inverse_sqrt(tns_ctx* ctx, int64_t N, float alpha, const float* src, float* dst,
                         int64_t stride, int64_t offset);

/* ---- non-convolutional YOLOv3 layers (forward) ------------------------- */
/* TAddLayer.forward (naddlayer.pas:667-720), single input of equal size:
 * out = activate(a + b) (addvv, then the layer's activation). */
int tns_hip_shortcut(tns_ctx* ctx, int64_t N, const float* a, int64_t aOffset, const float* b,
                     int64_t bOffset, float* out, int64_t outOffset, int32_t activation);
/* TNNCuda.upSample (nncuda.pas:136, 1267-1286; CPU upsample()
 * nupsamplelayer.pas:83-113).  outHeight/outWidth are the SMALL tensor's
 * height and width (the reference's naming); planes = aBatch*aChannels.
 * isForward != 0: out[(p*H*s + y)*W*s + x] = scale * in[(p*H + y div s)*W + x div s].
 * isForward == 0: in[...] += scale*out[...] over each input pixel's s x s
 * outputs in the CPU loop order (row outer), deterministic; zeroIn != 0
 * starts from 0 (the reverse layer's output.fill(0)). */
int tns_hip_upsample(tns_ctx* ctx, int64_t aBatch, int64_t aChannels, int64_t outHeight,
                     int64_t outWidth, float* in, int64_t stride, int32_t isForward, float scale,
                     float* out, int32_t zeroIn);
/* TYoloLayer.forward inference part (nyololayer.pas:786-825): out = in with
 * the logistic applied to entries 0, 1 and 4 .. 4+classes of every anchor;
 * data [batch][anchors][classes+5][hw].  (Route/concat = tns_hip_copy of
 * whole tensors, TTensor.concat ntensors.pas:12045-12061.) */
int tns_hip_yolo_forward(tns_ctx* ctx, int64_t batch, int64_t anchors, int64_t classes,
                         int64_t hw, const float* in, float* out);

/* ---- batch norm / softmax (TNNCuda twins, nncuda.pas:1056-1510; CPU
 * semantics ntensors.pas:7687-7830, 8693-8951, 9102-9177,
 * nsoftmaxlayer.pas:83-137).  Data is [groups][channels][blockSize]. ---- */
/* meansAndVars: blockSize = srcSize/(dstSize*groups); unbiased variance */
int tns_hip_means_and_vars(tns_ctx* ctx, int64_t srcSize, int64_t dstSize, int64_t groups,
                           const float* src, int64_t offset, float* means, float* vars);
/* TNNCuda.means / TNNCuda.variances — nncuda.pas:1330-1369, the pair the
 * reference's batchNormGPU (nbaselayer.pas:583-584) and
 * TConnectedLayer.forwardGPU (nconnectedlayer.pas:664-665) call.  Same
 * blockSize and results as the two halves of tns_hip_means_and_vars (CPU
 * MeansAndVars order, ntensors.pas:9102-9177: vssum_avx2 lanes per block for
 * the mean, srss lanes about the GIVEN means for the unbiased variance,
 * TNS_OPT_SRSS_QUIRK applying to the latter). */
int tns_hip_means(tns_ctx* ctx, int64_t srcSize, int64_t dstSize, int64_t groups,
                  const float* src, int64_t offset, float* means);
int tns_hip_variances(tns_ctx* ctx, int64_t srcSize, int64_t dstSize, int64_t groups,
                      const float* src, int64_t offset, const float* means, float* vars);
/* normalize: blockSize = dstSize/(srcSize*groups); bs==1: (x-m)/sqrt(max(v,eps)),
 * bs>1: (x-m)/max(sqrt(v),eps) */
int tns_hip_normalize(tns_ctx* ctx, int64_t srcSize, int64_t dstSize, int64_t groups,
                      const float* means, int64_t meansStride, const float* vars,
                      int64_t varsStride, float* dst, int64_t dstOffset);
/* forwardScale / forwardScaleAdd: dst[(b*S+i)*bs+j] = dst*scale[i*incb] (+ bias[i*incb]) */
int tns_hip_forward_scale(tns_ctx* ctx, int64_t dstSize, float* dst, int64_t offset,
                          int64_t scaleSize, const float* scale, int64_t incb, int64_t batch);
int tns_hip_forward_scale_add(tns_ctx* ctx, int64_t dstSize, float* dst, int64_t offset,
                              int64_t scaleSize, const float* scales, const float* biases,
                              int64_t incb, int64_t batch);
/* meansAndVarsDelta / normalizeDelta (sMeanAndVarianceDelta / sNormalizeDelta) */
int tns_hip_means_and_vars_delta(tns_ctx* ctx, int64_t srcSize, int64_t dstSize, int64_t groups,
                                 const float* delta, const float* x, int64_t offset,
                                 const float* mean, const float* variance, float* mean_delta,
                                 float* variance_delta);
int tns_hip_normalize_delta(tns_ctx* ctx, int64_t deltaSize, int64_t meanSize, int64_t groups,
                            float* delta, const float* x, int64_t offset, const float* mean,
                            const float* variance, const float* mean_delta,
                            const float* variance_delta);
/* addDots: dst[i] += sum x_norm*delta over (group, block) */
int tns_hip_add_dots(tns_ctx* ctx, int64_t N, int64_t dstSize, int64_t groups,
                     const float* src1, const float* src2, int64_t srcOffset, float* dst);
/* TSoftmaxLayer.softmaxBatch / softmaxCrossEntropy */
int tns_hip_softmax_batch(tns_ctx* ctx, int64_t N, const float* input, int64_t iOffset,
                          int64_t batch, int64_t batch_size, int64_t groups, int64_t group_size,
                          int64_t stride, float temp, float* output, int64_t oOffset);
int tns_hip_cross_entropy_softmax(tns_ctx* ctx, int64_t N, const float* pred, const float* truth,
                                  float* delta, float* error);
/* TTensor.Sum in the vssum_avx2 order (cost), result written to *out (device) */
int tns_hip_sum(tns_ctx* ctx, int64_t N, const float* src, int64_t offset, float* out);

/* ---- fused connected-network train step (BASELINE config 5) ------------
 * One TNNet.Propagate + TNNet.update (nnet.pas:275-450) for nlayers
 * TConnectedLayer (widths[l] -> widths[l+1], activation acts[l], batch norm
 * when bn != 0) followed by a TSoftmaxLayer, as ONE kernel launch.  buf holds
 * the packed parameters and state (layout: oracle/tns_oracle.h
 * ora_mlp_train_step), sized tns_mlp_buffer_floats().  *cost (device) gets
 * the softmax layer's loss.Sum().  Limits: nlayers <= 32,
 * 9*batch*max(widths[1..]) <= 40960 (one CU's LDS). */
int64_t tns_mlp_buffer_floats(int32_t nlayers, const int64_t* widths, int32_t bn, int64_t batch);
int tns_hip_mlp_train_step(tns_ctx* ctx, int32_t nlayers, const int64_t* widths,
                           const int32_t* acts, int32_t bn, int64_t batch, const float* X,
                           const float* truth, float learningRate, float momentum, float decay,
                           float* buf, float* cost);

/* ---- layer drivers (host logic of the reference, running on device) ---- */

/* TTensor.Conv2D — ntensors.pas:8252-8349.  input: batch x C x H x W,
 * weights: filters x (C*kH*kW) row-major, out: batch x filters x oH x oW.
 * im2col is skipped for 1x1 / stride 1 / dilation 1 (ntensors.pas:8286-8312).
 * workspace: >= batch*C*kH*kW*oH*oW floats, or NULL to use ctx scratch.
 * NOTE: mirrors the reference's slot swap: xDilation is passed as dilationY
 * (ntensors.pas:8303); harmless for square dilation. */
int tns_hip_conv2d(tns_ctx* ctx, int64_t batch, int64_t C, int64_t H, int64_t W,
                   const float* input, const float* weights, int64_t filters,
                   int64_t kH, int64_t kW, int64_t wPadding, int64_t hPadding,
                   int64_t xStride, int64_t yStride, int64_t xDilation, int64_t yDilation,
                   float* workspace, float* out);

/* TConvolutionalLayer.forward / forwardGPU with fused (folded) BN —
 * nConvolutionLayer.pas:457-569 / 1022-1153: Conv2D -> forwardBias ->
 * activate.  fused selects the schedule (same arithmetic, same bits, in all):
 *   TNS_CONV_UNFUSED  (0) the three reference stages (im2col, GEMM, bias+act)
 *   TNS_CONV_FUSED    (1) library's choice among the two below
 *   TNS_CONV_IM2COL   (2) im2col into workspace + SGEMM with bias+act epilogue
 *   TNS_CONV_IMPLICIT (3) implicit GEMM: the SGEMM gathers its B tiles from
 *                         the image (no col matrix, workspace unused); a
 *                         3-channel 3x3 layer with 16 or 32 filters runs the
 *                         direct kernel instead (same fmaf chains) */
enum { TNS_CONV_UNFUSED = 0, TNS_CONV_FUSED = 1, TNS_CONV_IM2COL = 2, TNS_CONV_IMPLICIT = 3 };
int tns_hip_conv_forward(tns_ctx* ctx, int64_t batch, int64_t C, int64_t H, int64_t W,
                         const float* input, const float* weights, const float* biases,
                         int64_t filters, int64_t kSize, int64_t stride, int64_t padding,
                         int64_t dilation, int32_t activation, float* workspace,
                         float* out, int32_t fused);

/* TConvolutionalLayer.forward in TRAINING with batch norm (nConvolutionLayer.
 * pas:457-569 -> TBaseLayer.batchNorm, nbaselayer.pas:336-370): Conv2D into
 * out; training != 0: MeansAndVars -> mean/variance, rolling_mean/variance
 * *= (1 - bnMomentum) then += bnMomentum*stat (axpy), x := out,
 * blockNormalize, x_norm := out; training == 0: blockNormalize with the
 * rolling statistics; then forwardScale(scales), forwardBias(biases),
 * activate.  Tensors [batch][filters][oH*oW]; statistics per filter.  The
 * layer's bnMomentum is 0.1 (nbaselayer.pas:188).  In-place and
 * bit-exact against the reference order (one fused pass after the stats). */
int tns_hip_conv_forward_train(tns_ctx* ctx, int64_t batch, int64_t C, int64_t H, int64_t W,
                               const float* input, const float* weights, int64_t filters,
                               int64_t kSize, int64_t stride, int64_t padding, int64_t dilation,
                               int32_t activation, const float* scales, const float* biases,
                               float* rolling_mean, float* rolling_variance, float bnMomentum,
                               int32_t training, float* mean, float* variance, float* x,
                               float* x_norm, float* workspace, float* out);

/* TConvolutionalLayer.backward without batch-norm (nConvolutionLayer.pas:
 * 571-671): delta *= f'(output) (Derivative), bias_updates += addSums(delta),
 * im2col(input), weight_updates += delta_b . col_b^T per image (NT, beta 1),
 * and if state_delta != NULL: col = W^T . delta (TN strided batched, beta 0)
 * then col2im accumulates into state_delta.  delta is updated in place.
 * workspace (batch*C*k*k*outH*outW floats) may be NULL (context scratch).
 * The backward im2col / col2im pad with padding*dilation (640, 665); a
 * dilation whose columns differ from the layer's outH x outW (92-100) is
 * refused with TNS_ERR_UNSUPPORTED ("same" paddings work at any dilation).
 * At dilation > 1 this REPRODUCES THE REFERENCE, not the calculus:
 *  - state_delta follows scol2im's input_row := (kernel_row - pad)*dil
 *    (ntensors.pas:11650-11715) with pad = padding*dilation, which is not
 *    the adjoint of im2col — it is not the true input gradient (reference
 *    quirk 3);
 *  - tns_hip_conv_forward(_train) at dilation > 1 writes out_dim(H, padding,
 *    kSize, dilation, stride) columns per filter, while this backward takes
 *    delta / output with the layer's (H + 2*padding - kSize)/stride + 1
 *    (nConvolutionLayer.pas:92-100): the two agree only where those sizes
 *    coincide ("same" paddings), exactly as in the reference. */
int tns_hip_conv_backward(tns_ctx* ctx, int64_t batch, int64_t C, int64_t H, int64_t W,
                          const float* input, const float* weights, int64_t filters,
                          int64_t kSize, int64_t stride, int64_t padding, int64_t dilation,
                          int32_t activation, const float* output, float* delta,
                          float* bias_updates, float* weight_updates, float* workspace,
                          float* state_delta);
/* The same with batch norm (isBatchNormalized, nConvolutionLayer.pas:601-602):
 * batchNormBack (nbaselayer.pas:372-395) replaces the bias term —
 * scale_updates += addDots(x_norm, delta); delta *= scales (forwardScale);
 * MeansAndVarsDelta(delta, x, mean, variance) -> mean_delta / variance_delta;
 * normalizeDelta — then the weight / input gradients as above.  x, x_norm,
 * mean, variance are the forward's (tns_hip_conv_forward_train). */
int tns_hip_conv_backward_bn(tns_ctx* ctx, int64_t batch, int64_t C, int64_t H, int64_t W,
                             const float* input, const float* weights, int64_t filters,
                             int64_t kSize, int64_t stride, int64_t padding, int64_t dilation,
                             int32_t activation, const float* output, float* delta,
                             const float* scales, const float* x, const float* x_norm,
                             const float* mean, const float* variance, float* scale_updates,
                             float* mean_delta, float* variance_delta, float* weight_updates,
                             float* workspace, float* state_delta);

/* ---- several GPUs from ONE process (config 4) ---------------
 * gemmStridedBatched over n devices (devices[i] for slot i; a device may
 * appear twice): HOST pointers, as the op-table gemmStridedBatched
 * (ntensors.pas:348-351), cblas_sgemm semantics.  The batch is split into n
 * contiguous shards (the first batchCount % n one GEMM longer); each slot
 * has its own context, stream and host thread and pipelines its shard's
 * uploads, GEMMs and downloads.  A shared operand (strideA or strideB = 0,
 * the conv weights of nConvolutionLayer.pas:773) crosses PCIe once, to slot
 * 0, and reaches the other devices by peer copies (xGMI).  Results are bit
 * identical to the single-device call.  Returns a status. */
int tns_hip_sgemm_strided_batched_multi(const int32_t* devices, int32_t n, uint8_t transA,
                                        uint8_t transB, int64_t M, int64_t N, int64_t K,
                                        float alpha, const float* A, int64_t lda,
                                        int64_t strideA, const float* B, int64_t ldb,
                                        int64_t strideB, float beta, float* C, int64_t ldc,
                                        int64_t strideC, int64_t batchCount);
/* Spread the op-table drop-ins tns_cblas_sgemm_batch_strided / tns_cblas_sgemm
 * over these devices (n <= 1: the default single context again), so an
 * unmodified Pascal binding drives several GPUs. */
int tns_set_op_devices(const int32_t* devices, int32_t n);

/* ---- telemetry (TTensorMetrics-style per-op device timing) ------------ */
int    tns_hip_set_telemetry(tns_ctx* ctx, int32_t enable);
double tns_hip_op_ms(tns_ctx* ctx, int32_t op);   /* accumulated ms per op */
enum { TNS_OP_GEMM = 0, TNS_OP_IM2COL = 1, TNS_OP_COL2IM = 2, TNS_OP_BIAS = 3,
       TNS_OP_ACTIVATE = 4, TNS_OP_COUNT = 5 };

/* ---- tuning / options -------------------------------------------------- */
/* SGEMM tile-shape variants (the production path picks one per problem;
 * these force one, for sweeps).  variant < 0 = heuristic.  Some shapes are
 * NN-with-aligned-operands only and return TNS_ERR_UNSUPPORTED otherwise. */
int         tns_gemm_variant_count(void);
/* k-major-A conv tiles of the backward's col = W^T . delta (TNS_OPT_DX_TILE = v) */
int         tns_conv_dx_tile_count(void);
/* implicit transposed-convolution forms of the conv backward's state.delta
 * (TNS_OPT_DX_CONV = v) */
int         tns_conv_dx_conv_count(void);
/* residue-sequential dW forms of the conv backward (TNS_OPT_DW_RES = v) */
int         tns_conv_dw_res_count(void);
/* implicit-im2col dW tiles of the conv backward (TNS_OPT_DW_TILE = v) */
int         tns_conv_dw_tile_count(void);
/* plane-sized implicit-conv tiles (TNS_OPT_CONV_VARIANT = 100 + v) */
int         tns_conv_tile_variant_count(void);
const char* tns_conv_tile_variant_name(int32_t variant);
/* two-pass slab conv forms: the im2col matrix in the GEMM's LDS slot order,
 * then B by LDS-DMA (TNS_OPT_CONV_VARIANT = 500 + v) */
int         tns_conv_slab_count(void);
const char* tns_conv_slab_name(int32_t variant);
/* 1x1 stride-1 conv forms reading the input planes by LDS-DMA (planes of a
 * multiple of 4 pixels; TNS_OPT_CONV_VARIANT = 600 + v) */
int         tns_conv1x1_count(void);
const char* tns_conv1x1_name(int32_t variant);
/* ping-pong implicit-conv tiles (TNS_OPT_CONV_VARIANT = 200 + v) */
int         tns_conv_pp_variant_count(void);
const char* tns_conv_pp_variant_name(int32_t variant);
/* LDS-DMA-ring implicit-conv tiles (TNS_OPT_CONV_VARIANT = 300 + v) */
int         tns_conv_dma_variant_count(void);
const char* tns_conv_dma_variant_name(int32_t variant);
/* input-patch conv tiles, 3x3 stride-1 pad-1 (TNS_OPT_CONV_VARIANT = 400 + v) */
int         tns_conv_patch_variant_count(void);
const char* tns_conv_patch_variant_name(int32_t variant);
/* VALU chain variants of the sdot-order NT product (TNS_OPT_SDOT_FORM = 1 + v) */
int         tns_sdot_chains_variant_count(void);
const char* tns_sdot_chains_variant_name(int32_t variant);
/* residue-register forms of the sdot-order NT product (TNS_OPT_SDOT_FORM =
 * 64 + v) */
int         tns_sdot_rc_variant_count(void);
const char* tns_sdot_rc_variant_name(int32_t variant);
const char* tns_gemm_variant_name(int32_t variant);
int tns_hip_gemm_variant(tns_ctx* ctx, int32_t variant, uint8_t transA, uint8_t transB,
                         int64_t M, int64_t N, int64_t K, float ALPHA,
                         const float* A, int64_t aOffset, int64_t lda, int64_t strideA,
                         const float* B, int64_t bOffset, int64_t ldb, int64_t strideB,
                         float BETA, float* C, int64_t cOffset, int64_t ldc, int64_t strideC,
                         int64_t batchCount);

/* TNS_OPT_STRICT_BETA0 (default 1): beta==0 computes 0*C like the reference
 * (NaN/Inf in C propagate).  0 = BLAS convention (C not read).
 * TNS_OPT_CONV_VARIANT (default -1 = heuristic): forces the tile shape of the
 * implicit-GEMM convolution (tuning; index as tns_gemm_variant_name, 100 + v
 * for plane-sized tile v of tns_conv_tile_variant_name, 200 + v for ping-pong
 * tile v of tns_conv_pp_variant_name, 300 + v for LDS-DMA-ring tile v of
 * tns_conv_dma_variant_name, 400 + v for input-patch tile v of
 * tns_conv_patch_variant_name, 500 + v for slab form v of tns_conv_slab_name,
 * 600 + v for 1x1 form v of tns_conv1x1_name).
 * TNS_OPT_CONV_PAD (default -1 = by cost): 1 gathers from a zero-padded copy
 * of the images, 0 bounds-checks the window inside the GEMM.
 * TNS_OPT_NT_SDOT (default 1): gemm(NoTrans, Trans) sums in the reference's
 * sdot_avx2 order (8 residue chains, ntensors.pas:1233-1306, 1957-2005), bit
 * for bit; 0 = one ascending-k chain per element (faster, within 1e-4).
 * TNS_OPT_SRSS_QUIRK (library default 0): 1 reproduces the reference's srss
 * dropping lanes 4..7 of the variance sum when a block is a multiple of 8
 * long (ntensors.pas:1493-1523, meansAndVars with blockSize % 8 == 0; and
 * sVarinceDelta_avx, 8739-8741).  The Pascal binding's initHIP and
 * useHipOpTable (pascal/nnHip.pas) set it to 1 by default, so a drop-in
 * reproduces the configured USE_AVX2 CPU build.
 * TNS_OPT_TT_EXACT (default 1): gemm(Trans, Trans) sums in the reference's
 * scalar s_tt order (mul, mul, add each rounded; ntensors.pas:2159-2182) on
 * the VALU, bit for bit; 0 = the fp32 MFMA kernel (faster, within 1e-4).
 * TNS_OPT_SDOT_FORM (default -1 = by shape): kernel of the sdot-order NT
 * product (tuning / tests; same result bit for bit): 0 = the MFMA kernel
 * (one wave per residue class), 1 + v = VALU chain kernel variant v (one
 * lane per few residue chains, for few outputs over a long k), 64 + v =
 * residue-register form v (one or two waves keep an output tile's eight
 * residue chains in their registers; many tiles over a short k).
 * TNS_OPT_DX_FUSED (default 1): the conv backward's state.delta of 1x1
 * stride-1, dilation-1 layers with >= 8192 pixels per image by one kernel that runs
 * each window tap's filter chain and adds it to the image pixel in scol2im's
 * order (no col matrix); 2 = that kernel on every stride-1 layer it fits;
 * 0 = the reference's two stages, TN GEMM into the workspace + col2im (same
 * bits in all three).
 * TNS_OPT_DX_TILE (default -1 = by shape): the first of those two stages,
 * col_b = W^T . delta_b, for all images in one launch of a k-major-A conv
 * tile (conv_tile4.hip, the delta planes as a 1x1 convolution's images) where
 * one applies; -2 = the TN GEMM always; v >= 0 forces form v of
 * tns_conv_dx_tile_count() (tests; same bits in every form).
 * TNS_OPT_DX_CONV (default -1 = by shape): the conv backward's state.delta of
 * stride-1, dilation-1 3x3 layers (C a multiple of 64, filters of 32) by one
 * implicit transposed convolution over the delta planes: each window tap's
 * filter chain, added to the image pixel in scol2im's (kr, kc) order for the
 * taps it does not skip — the TN GEMM + col2im sums, no col matrix (uses a
 * filters*C*9-float tap-major copy of the weights in the context's scratch);
 * -2 = off; v >= 0 forces form v of tns_conv_dx_conv_count() (same bits).
 * TNS_OPT_DW_TILE (default -1 = by shape): the conv backward's dW product
 * (the reference's per-image sdot-order NT GEMM over the im2col matrix) by
 * a kernel that generates the im2col rows in its staging (dw_tile.hip: no
 * col matrix, no im2col pass) where one applies; -2 = im2col + the sdot
 * kernels always; v >= 0 forces form v of tns_conv_dw_tile_count() (same
 * bits in every form).
 * TNS_OPT_DW_RES (default -1 = by shape): the conv backward's dW product as
 * the sdot order's eight residue chains run one after another per output
 * tile over residue-major copies of delta and the im2col matrix, folded in
 * sdot's order, then added to weight_updates image by image (dw_res.hip; the
 * copies and the per-group partial planes live in the context's scratch);
 * by shape on the 3x3 layers with >= 64 filters; -2 = off; v >= 0 forces
 * form v of tns_conv_dw_res_count() (same bits; ignored while
 * TNS_OPT_DW_TILE forces a tile).  Memory: the residue-major copies (about
 * the im2col matrix plus delta) and the group planes live in the context's
 * scratch, allocated IN ADDITION to the caller's workspace (which then holds
 * nothing for dW); -2 bounds the backward's dW memory to the workspace.
 * TNS_OPT_BWD_OVERLAP (default 1): the conv backward runs the dW product and
 * the state.delta chain (which read delta and write disjoint outputs)
 * concurrently, the latter on a side stream of the context that the
 * context's stream waits for before the call returns its work; 0 = in
 * sequence (also whenever telemetry is on).  Same results either way.
 * Memory: when dW reads an im2col matrix and state.delta takes the TN +
 * col2im chain, the overlap gives that chain its own batch*C*k*k*oH*oW-float
 * col buffer, allocated by the context IN ADDITION to the caller's workspace
 * (which then holds dW's col matrix only); if that allocation fails, or the
 * side stream cannot be created, the call runs in sequence within the
 * caller's workspace instead of failing.  Set 0 to bound the backward's
 * memory to the workspace.  2 = pipelined: each call enqueues its dW on the
 * side stream (behind the earlier calls' dW) and returns without joining it;
 * a later call whose operands meet a pending dW's (below), tns_hip_finish and
 * tns_hip_get_stream first make the context's stream wait for the side
 * stream.  The dW of layer L then runs under the following calls' derive /
 * state.delta work and the non-conv layers' calls between them; a later
 * backward call that writes into a pending dW's delta or input waits for that
 * dW first.  The caller must not read or modify a pending call's
 * weight_updates, nor modify its input or delta, by other means (work
 * enqueued on the stream outside this API, or host accesses) before a join:
 * tns_hip_finish, an entry point whose operands include them, or
 * tns_hip_get_stream (which joins before it hands the stream out, so work the
 * caller then enqueues on it is ordered after every pending dW).  Same results; state.delta always gets its own col buffer
 * (the memory note above).  pascal/nnHip.pas initHIP selects this mode by
 * default (pipelineBackward = true): there every access goes through the API.
 * Since round 6 no entry point joins unconditionally during a pipelined
 * pass: the non-conv ones (gemm, im2col / col2im, bias, activation, BLAS-1,
 * addvv & co, shortcut, upsample, yolo, batch norm, softmax, sgd_update)
 * join only when they write a pending dW's delta or input, read or write its
 * weight_updates (or the caller's workspace that dW's im2col fills), or take
 * a context scratch slot the side stream still uses — so TNet.backward's
 * shortcut / route / upsample calls between two conv layers keep the
 * pipeline running.  Context management, host copies, gemmBatched, the conv
 * forward drivers and the fused train step still join.
 * TNS_OPT_SCRATCH_CAP (default 0 = none): largest context scratch buffer in
 * floats; a larger request fails as a failed allocation does (tests reach the
 * fallback paths with it).
 * TNS_OPT_DERIVE_SUMS (default 0): 1 = the conv backward's Derivative and
 * addSums (no batch norm) in one pass where the sums' chain kernel applies
 * (planes under 16384 pixels); 0 = two passes (measured level: 15.06 vs
 * 15.00 ms a pipelined YOLOv3 pass, profiles/r04_bwd_schedules2.json).  Same
 * bits.
 * Environment switches read once per process (A/B timing only; every setting
 * gives the same bits): TNS_STREAM_PRIO=0 — the pipelined dW stream at the
 * default queue priority instead of the lowest (and the context's own stream
 * at the default instead of the highest); TNS_BN_FUSED=0 — batchNormBack as
 * its separate passes instead of the one chain pass + normalizeDelta;
 * TNS_DX_C1=0 — the 1x1 layers' state.delta on the TN product / conv_dx forms
 * instead of conv1x1's W^T product; TNS_ACC4=0 — the dW accumulate pass in
 * its scalar form. */
enum { TNS_OPT_STRICT_BETA0 = 0, TNS_OPT_CONV_VARIANT = 1, TNS_OPT_CONV_PAD = 2,
       TNS_OPT_NT_SDOT = 3, TNS_OPT_SRSS_QUIRK = 4, TNS_OPT_TT_EXACT = 5,
       TNS_OPT_SDOT_FORM = 6, TNS_OPT_DX_FUSED = 7, TNS_OPT_DX_TILE = 8,
       TNS_OPT_DW_TILE = 9, TNS_OPT_BWD_OVERLAP = 10, TNS_OPT_DX_CONV = 11,
       TNS_OPT_DW_RES = 12, TNS_OPT_DERIVE_SUMS = 13, TNS_OPT_SCRATCH_CAP = 14 };
int tns_set_option(int32_t opt, int64_t value);

#ifdef __cplusplus
}
#endif
#endif /* TNS_H */
