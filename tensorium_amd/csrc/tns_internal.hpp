// tns_internal.hpp — shared declarations of libtensorium_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tns.h"

namespace tns {

// ---- error channel ---------------------------------------------------------
int set_error(int code, const char* fmt, ...);
const char* hip_err_str(hipError_t e);

#define TNS_HIP_TRY(expr)                                                              \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return ::tns::set_error(TNS_ERR_HIP, "%s failed: %s (%s:%d)", #expr,            \
                              ::tns::hip_err_str(_e), __FILE__, __LINE__);             \
  } while (0)

// ---- SGEMM -----------------------------------------------------------------
// Epilogue applied after the K loop (fused conv path):
//   EPI_NONE          C = acc
//   EPI_BIAS_ACT      C = act(acc + bias[row])   (forwardBias + activate)
//   EPI_ADD           C = C + acc (acc from +0; one add — a 1x1 col2im fused)
enum EpiKind { EPI_NONE = 0, EPI_BIAS_ACT = 1, EPI_ADD = 2 };
// logistic / tanh (exp in double) are applied after the GEMM, not in its
// epilogue (tns_act.hpp)
constexpr bool act_transcendental(int act) { return act == 0 || act == 6; }

// beta handling, decided on the host:
//   BETA_ZERO   acc starts at 0 (C not read)       — BLAS convention
//   BETA_ONE    acc starts at C                     — matMul accumulate
//   BETA_SCALE  acc starts at beta*C (single mul)   — reference mulvs, incl.
//               strict beta=0 (0*C keeps NaN/Inf like ntensors.pas:2259)
//   BETA_STORE  C := the product term alone (sdot kernel only: per-image
//               partial sums that a later in-order pass adds to C)
enum BetaMode { BETA_ZERO = 0, BETA_ONE = 1, BETA_SCALE = 2, BETA_STORE = 3 };

struct GemmArgs {
  int64_t M, N, K;
  float alpha, beta;
  int beta_mode;
  const float* A;
  int64_t lda, strideA;
  const float* B;
  int64_t ldb, strideB;
  float* C;
  int64_t ldc, strideC;
  int64_t batch;
  // epilogue
  int epi;
  const float* bias;  // per row of C (filters)
  int act;            // TActivationType ordinal
  // implicit-GEMM convolution: when conv != 0 the batch is
  // folded into N (column n = image n / conv_ohw, pixel n % conv_ohw; the
  // launch has batch == 1) and B is the im2col matrix of the images at
  // B + image*strideB (conv_H x conv_W each), generated inside the GEMM's
  // staging loads (buffer loads over conv_bytes) and never written to memory;
  // C of image i starts at C + i*strideC.
  //   conv == 1: the images are zero-padded copies (conv_pH = conv_pW = 0);
  //   conv == 2: unpadded images, window bounds checked (pads conv_pH/pW).
  // k-table, two int arrays of ktab_n = K + KTAB_PAD entries for the stored
  // image size and k = (c*kH + kr)*kW + kc:
  //   ktab[k]          = 4*(c*H*W + kr*dY*W + kc*dX)   (byte offset)
  //   ktab[ktab_n + k] = kr*dY | (kc*dX) << 16          (window offsets)
  // entries k >= K are sentinels {0x80000000, 0x4000 | 0x4000 << 16} (out of
  // range: the buffer load returns 0).
  int conv;
  const int* ktab;
  int ktab_n;
  int conv_H, conv_W, conv_ow, conv_ohw, conv_sY, conv_sX, conv_pH, conv_pW;
  int conv_bytes;
  // conv_tile4 DX forms on one pixel class of a stride-2 layer (dx_cls != 0):
  // columns = the class's pixels (2 qy + py, 2 qx + px) of images dx_imgW
  // wide (py = dx_cls >> 1 & 1, px = dx_cls >> 2 & 1); k = the class's taps
  // (count dx_taps >> 16, nibble i = tap i's forward-window bit fr*3 + fc)
  int dx_cls, dx_taps, dx_imgW;
  // diagnostic builds (-DTNS_GEMM_STAMPS) only: per-block timeline records
  unsigned* stamps;
};

hipError_t launch_sgemm(const GemmArgs& a, bool transA, bool transB, hipStream_t s);
// large aligned NN (M, N multiples of the tile, K of 32; sgemm_nn_big.hip):
// form v of sgemm_nn_big_count(); pick = -1 when none applies by heuristic
int sgemm_nn_big_count();
const char* sgemm_nn_big_name(int v);
int sgemm_nn_big_pick(const GemmArgs& a);
hipError_t launch_sgemm_nn_big(int v, const GemmArgs& a, hipStream_t s);
// the 256x256 NN tile on the ping-pong schedule (sgemm_nn_pp.hip; form 5)
bool sgemm_nn_pp_applies(const GemmArgs& a);
hipError_t launch_sgemm_nn_pp(const GemmArgs& a, hipStream_t s, bool bperm = false);
// the same tile with one wave per SIMD (4 waves of 128 x 128), A and B by
// LDS-DMA into swizzled row images, interleaved columns (b128 B reads,
// 16-byte C traffic) — sgemm_nn_w4.hip, nn_big form 6
bool sgemm_nn_w4_applies(const GemmArgs& a);
hipError_t launch_sgemm_nn_w4(const GemmArgs& a, hipStream_t s);
// gemm(NoTrans, Trans) in the reference's sdot_avx2 order (sgemm_sdot.hip);
// plain epilogue only
hipError_t launch_sgemm_nt_sdot(const GemmArgs& a, hipStream_t s);
// the same product on the VALU, one lane per few residue chains
// (sgemm_sdot_chains.hip): for few outputs over a long k
hipError_t launch_sdot_chains(const GemmArgs& a, int variant, hipStream_t s);
int sdot_chains_variant_count();
const char* sdot_chains_variant_name(int v);
// the same product with an output tile's residue chains in one or two
// waves' registers (sgemm_sdot_rc.hip)
int sdot_rc_variant_count();
const char* sdot_rc_variant_name(int v);
bool sdot_rc_applies(const GemmArgs& a);
hipError_t launch_sdot_rc(int v, const GemmArgs& a, hipStream_t s);
// TNS_OPT_SDOT_FORM: -1 heuristic, 0 the MFMA kernel, 1 + v chains variant v,
// 64 + v residue-register form v
constexpr int SDOT_FORM_RC = 64;
void set_sdot_form(int form);
// gemm(Trans, Trans) in the reference's scalar s_tt order (sgemm_tt.hip);
// plain epilogue only
hipError_t launch_sgemm_tt(const GemmArgs& a, hipStream_t s);
// C[e] := (...((C[e] + part[0][e]) + part[1][e]) ...) + part[batch-1][e]
hipError_t launch_add_in_order(float* C, const float* part, int64_t n, int64_t batch,
                               hipStream_t s);
// implicit-GEMM convolution: NN, B generated from the image (a.conv must be set)
hipError_t launch_sgemm_conv(const GemmArgs& a, hipStream_t s);
hipError_t launch_sgemm_conv_variant(int variant, const GemmArgs& a, hipStream_t s);
// implicit-GEMM convolution on plane-sized tiles (conv_tile.hip): unpadded
// images (a.conv == 2 fields, a.conv_pH/pW = padding), kernel size ks 1 or
// 3, K % 32 == 0, M % tile rows == 0; variant v of conv_tile_count()
int conv_tile_count();
const char* conv_tile_name(int v);
int conv_tile_pick(const GemmArgs& a, int ks);
hipError_t launch_conv_tile(int v, const GemmArgs& a, int ks, int dil, hipStream_t s);
// two-pass conv forward (conv_slab.hip): the im2col matrix written once in
// the GEMM's LDS slot order, then a GEMM with B by LDS-DMA; form v of
// conv_slab_count(); conv_slab_pick = -1 where conv_tile4 stays
struct ConvSlabArgs {
  const float* input;    // [batch][C][H][W]
  const float* weights;  // [M][K], K = C*ks*ks
  const float* bias;     // fused bias + activation when not null
  float* out;            // [batch][M][oh*ow]
  int64_t batch, C, H, W, M, K, ks, stride, pad, dil, ow, ohw;
  int act;
};
// 1x1 / stride-1 layers with a multiple of 4 pixels per plane straight from
// the input planes (conv1x1.hip, B by LDS-DMA): form v of conv1x1_count();
// conv1x1_pick = -1 where the other paths stay
int conv1x1_count();
const char* conv1x1_name(int v);
int conv1x1_pick(int64_t M, int64_t N, int64_t K, int64_t P);
hipError_t launch_conv1x1(int v, const float* weights, const float* x, const float* bias,
                          float* out, int64_t batch, int64_t M, int64_t K, int64_t P, int act,
                          hipStream_t s, bool add = false);
// out[c][r] = in[r][c] (rows x cols)
hipError_t launch_transpose(const float* in, float* out, int64_t rows, int64_t cols,
                            hipStream_t s);
int conv_slab_count();
const char* conv_slab_name(int v);
int conv_slab_pick(int64_t M, int64_t N, int64_t K, int64_t ks);
int64_t conv_slab_floats(int v, int64_t N, int64_t K);  // slab scratch, -1: no such form
hipError_t launch_conv_slab(int v, const ConvSlabArgs& c, float* slab, hipStream_t s);
// the same tiles with k-permuted LDS images read by ds_read_b128
// (conv_tile4.hip; K % the form's k-tile == 0): conv_tile variants
// conv_tile_count() - conv_tile4_count() + v
int conv_tile4_count();
// conv_tile4 forms that read A from a pre-permuted copy of the weights
// (conv_tile4_permute into M*K floats of scratch first); conv_tile_is_ap
// takes a conv_tile index (conv_tile.hip)
bool conv_tile4_is_ap(int v);
bool conv_tile_is_ap(int v);
hipError_t conv_tile4_permute(const float* A, float* Ap, int64_t M, int64_t K, hipStream_t s);
const char* conv_tile4_name(int v);
int conv_tile4_bk(int v);
hipError_t launch_conv_tile4(int v, const GemmArgs& a, int ks, int dil, hipStream_t s);
// conv backward col_b = W^T . delta_b (all images, col [batch][C*ks*ks][oh*ow],
// beta = 0) on conv_tile4's k-major-A forms: form v of conv_tile4_ta_count(),
// conv_tile4_dx_pick = -1 where none applies
int conv_tile4_ta_count();
const char* conv_tile4_ta_name(int v);
int conv_tile4_dx_pick(int64_t M, int64_t N, int64_t K, int64_t ks);
hipError_t launch_conv_tile4_dx(int v, const float* w, const float* delta, float* col,
                                int64_t batch, int64_t C, int64_t ks, int64_t F, int64_t oh,
                                int64_t ow, hipStream_t s, bool add_into = false);
// (add_into, 1x1 only: col is state.delta itself, each element C + col)
// state.delta of a stride-1 3x3 layer as one implicit transposed convolution
// over the delta planes (conv_tile4.hip DX forms): wt = the weights tap-major
// (launch_transpose_taps), im = state.delta, added to in scol2im's order;
// conv_tile4_dx3_pick = -1 where none applies
int conv_tile4_dx3_count();
const char* conv_tile4_dx3_name(int v);
int conv_tile4_dx3_pick(int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F, int64_t ks,
                        int64_t pad);
hipError_t launch_conv_tile4_dx3(int v, const float* wt, const float* delta, float* im,
                                 int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F,
                                 int64_t ks, int64_t pad, int64_t oh, int64_t ow, hipStream_t s);
hipError_t launch_transpose_taps(const float* w, float* wt, int64_t F, int64_t C, int64_t K2,
                                 hipStream_t s, unsigned long long order = ~0ULL);
// state.delta of a stride-2 3x3 layer (dilation 1) as four implicit
// transposed convolutions, one per output pixel class (py, px) = parity of
// (row, column): each class's taps in scol2im's order, no col matrix.  wt =
// the weights transposed tap-major in the class order conv_tile4_dx3s2_order
// (pad) gives; form v of conv_tile4_dx3_count(); pick -1 where none applies
unsigned long long conv_tile4_dx3s2_order(int64_t pad);
int conv_tile4_dx3s2_pick(int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F, int64_t ks,
                          int64_t pad);
hipError_t launch_conv_tile4_dx3s2(int v, const float* wt, const float* delta, float* im,
                                   int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F,
                                   int64_t pad, int64_t oh, int64_t ow, hipStream_t s);
// implicit-GEMM convolution on the ping-pong schedule (conv_pp.hip): same
// operands and limits as conv_tile; conv_pp_pick = -1 where not measured faster
int conv_pp_count();
const char* conv_pp_name(int v);
int conv_pp_pick(const GemmArgs& a, int ks);
hipError_t launch_conv_pp(int v, const GemmArgs& a, int ks, int dil, hipStream_t s);
// implicit-GEMM convolution fed by an LDS-DMA ring (conv_dma.hip): same
// operands and limits as conv_tile
int conv_dma_count();
const char* conv_dma_name(int v);
int conv_dma_pick(const GemmArgs& a, int ks);
hipError_t launch_conv_dma(int v, const GemmArgs& a, int ks, int dil, hipStream_t s);
// 3x3 stride-1 pad-1 convolution reading B from a staged input patch
// (conv_patch.hip): whole output rows per tile
int conv_patch_count();
const char* conv_patch_name(int v);
int conv_patch_pick(const GemmArgs& a);
hipError_t launch_conv_patch(int v, const GemmArgs& a, hipStream_t s);
// conv backward dW in the sdot order with the im2col matrix generated in the
// staging (dw_tile.hip): part[b][m][n] = alpha * sdot over the pixels of
// delta_b[m][.] and the im2col row n of image b (BETA_STORE; the caller adds
// the images in order); M % tile rows == 0, N % tile columns == 0
struct DwArgs {
  const float* delta;  // [batch][M][HW]
  const float* x;      // [batch][C][H][W]
  float* part;         // [batch][M][N]
  int M, N, HW, C, H, W, oW, stride, pad, dil;
  int va;              // delta rows float4-loadable (HW % 4 == 0, 16-byte aligned)
  float alpha;
  int64_t strideA, strideX, strideP, batch;
};
int dw_tile_count();
const char* dw_tile_name(int v);
int dw_tile_pick(const DwArgs& a, int ks);
hipError_t launch_dw_tile(int v, const DwArgs& a, int ks, hipStream_t s);
// direct convolution (conv_direct.hip) for 3-channel 3x3 layers with 16 or
// 32 filters: bias (nullable: raw output) + activation fused
bool conv_direct_applies(int64_t C, int64_t ks, int64_t filters);
hipError_t launch_conv_direct(const float* in, const float* w, const float* bias, float* out,
                              int64_t batch, int64_t C, int64_t H, int64_t W, int64_t filters,
                              int64_t ks, int64_t stride, int64_t pad, int64_t dil, int64_t oh,
                              int64_t ow, int act, hipStream_t s);
// conv backward state.delta for stride-1, dilation-1 layers (conv_dx.hip):
// TN GEMM col = W^T . delta fused with scol2im's accumulation into im; wt is
// scratch for the [k^2][F][C] copy of the weights (F*C*k^2 floats)
bool conv_dx_fused_applies(int64_t C, int64_t H, int64_t W, int64_t ks, int64_t stride, int64_t F,
                           int64_t oh, int64_t ow);  // where measured faster
bool conv_dx_fused_fits(int64_t C, int64_t H, int64_t W, int64_t stride, int64_t F, int64_t oh,
                        int64_t ow);  // where the kernel can run (forced: TNS_OPT_DX_FUSED = 2)
hipError_t launch_conv_dx_col2im(const float* w, float* wt, const float* delta, float* im,
                                 int64_t batch, int64_t C, int64_t H, int64_t W, int64_t F,
                                 int64_t ks, int64_t pad, int64_t dil, int64_t oh, int64_t ow,
                                 hipStream_t s);
// k-table of an implicit-GEMM convolution over stored Hs x Ws images (padded
// or not): K = C*kH*kW entries plus KTAB_PAD sentinels
constexpr int KTAB_PAD = 256;
hipError_t launch_build_ktab(int* ktab, int C, int Hs, int Ws, int kH, int kW, int dY, int dX,
                             hipStream_t s);
// zero-padded copy of a batch of images: [batch][C][H+2pH][W+2pW]
hipError_t launch_pad_images(const float* im, int64_t batch, int64_t C, int64_t H, int64_t W,
                             int64_t pH, int64_t pW, float* out, hipStream_t s);
// variant < 0 picks the tile shape by heuristic; otherwise forces one (tuning)
hipError_t launch_sgemm_variant(int variant, const GemmArgs& a, bool transA, bool transB,
                                hipStream_t s);
int sgemm_variant_count();
const char* sgemm_variant_name(int v);

// ---- im2col / col2im -------------------------------------------------------
struct ConvGeom {
  int64_t C, H, W, kH, kW, padH, padW, sY, sX, dY, dX;
  int64_t oh, ow;
};
int64_t out_dim(int64_t in, int64_t pad, int64_t k, int64_t dil, int64_t stride);
hipError_t launch_im2col(const ConvGeom& g, const float* im, int64_t imStride, float* col,
                         int64_t colStride, int64_t batch, hipStream_t s);
hipError_t launch_col2im(const ConvGeom& g, const float* col, int64_t colStride, float* im,
                         int64_t imStride, int64_t batch, hipStream_t s);
// the same product as residue chains run in sequence over residue-major
// copies of delta and the im2col matrix (dw_res.hip), then added to
// weight_updates image by image; scratch: dA batch*M*8*K4 (+32), dB
// batch*dw_res_b_rows(v, N)*8*K4 (+32), part batch*groups*M*N floats
// (K4 = dw_res_k4(K))
struct DwResArgs {
  ConvGeom g;
  const float* x;        // input images, xStride floats apart
  int64_t xStride;
  const float* delta;    // [batch][M][K]
  float* weight_updates; // [M][N]
  float *dA, *dB, *part;
  int64_t M, N, K, batch;
  bool direct;           // 1x1 / stride 1 / pad 0: the input planes are the col rows
  float alpha;
};
int dw_res_count();
const char* dw_res_name(int v);
int64_t dw_res_k4(int64_t K);
int64_t dw_res_groups(int v);
int64_t dw_res_b_rows(int v, int64_t N);  // dB rows per image
int dw_res_pick(int64_t M, int64_t N, int64_t K, int64_t batch);
hipError_t launch_dw_res(int v, const DwResArgs& d, hipStream_t s);

// ---- elementwise -------------------------------------------------------------
bool act_supported(int act);
hipError_t launch_forward_bias(float* dst, int64_t nFilters, int64_t blockSize,
                               const float* bias, int64_t incb, int64_t batch, hipStream_t s);
hipError_t launch_backward_bias(float* dst, int64_t nDst, const float* src, int64_t blockSize,
                                int64_t batch, int64_t incb, hipStream_t s);
hipError_t launch_activate(float* x, int64_t n, int act, hipStream_t s);
// darknet_layers.hip: shortcut / upsample / yolo forward
hipError_t launch_shortcut(int64_t n, const float* a, const float* b, float* out, int act,
                           hipStream_t s);
hipError_t launch_upsample(int64_t planes, int H, int W, int stride, float scale, const float* in,
                           float* out, hipStream_t s);
hipError_t launch_upsample_backward(int64_t planes, int H, int W, int stride, float scale,
                                   float* in, const float* out, int zero, hipStream_t s);
// TNNCuda addvv/subvv/mulvv/fmavv (op 0..3), fmavss, inverseSqrt
hipError_t launch_vv(int op, int64_t n, const float* a, int64_t inca, const float* b, int64_t incb,
                     const float* c, int64_t incc, float* d, int64_t incd, hipStream_t s);
hipError_t launch_fmavss(int64_t n, const float* src, float scalar, float bias, float* dst,
                         hipStream_t s);
hipError_t launch_inverse_sqrt(int64_t n, const float* src, float* dst, int64_t stride,
                               hipStream_t s);
hipError_t launch_yolo(int64_t batch, int anchors, int classes, int64_t hw, const float* in,
                       float* out, hipStream_t s);
hipError_t launch_bias_activate(float* dst, int64_t nFilters, int64_t blockSize,
                                const float* bias, int64_t batch, int act, hipStream_t s);
hipError_t launch_derive(const float* x, int64_t n, int act, float* delta, hipStream_t s);
// TConnectedLayer/TConvolutionalLayer.update fused (elementwise.hip)
hipError_t launch_sgd_update(int64_t nw, float* w, float* dw, int64_t n, float* b, float* db,
                             float* sc, float* dsc, float lrb, float ndb, float mom,
                             hipStream_t s);
hipError_t launch_axpy(int64_t n, float a, const float* x, int64_t incx, float* y, int64_t incy,
                       hipStream_t s);
hipError_t launch_scale(int64_t n, float a, float* x, int64_t stride, hipStream_t s);
hipError_t launch_fill(int64_t n, float* x, float v, int64_t stride, hipStream_t s);
hipError_t launch_copy(int64_t n, const float* src, int64_t inca, float* dst, int64_t incb,
                       hipStream_t s);
hipError_t launch_clamp(int64_t n, float alpha, const float* src, float* dst, int64_t stride,
                        hipStream_t s);

// ---- batch-norm / softmax (batchnorm.hip) ----------------------------------
// x laid out [groups][N][bs]; one statistic per channel i in [0, N)
// quirk != 0: srss drops lanes 4..7 of tail-less blocks, as the reference
// part: device scratch of >= 2*groups*N floats for per-block results (conv
// blocks, bs >= 64, take the lane-chain kernels with it); nullptr = the
// one-thread-per-channel kernels only
// what: 1 the means, 2 the variances about the given means (TNNCuda.means /
// .variances, nncuda.pas:1330-1369), 3 both (meansAndVars)
hipError_t launch_means_vars(const float* x, int64_t groups, int64_t N, int64_t bs, float* means,
                             float* vars, int quirk, float* part, hipStream_t s, int what = 3);
hipError_t launch_normalize(float* x, int64_t groups, int64_t N, int64_t bs, const float* means,
                            int64_t mstride, const float* vars, int64_t vstride, hipStream_t s);
hipError_t launch_scale_add(float* x, int64_t groups, int64_t N, int64_t bs, const float* scales,
                            const float* biases, int64_t incb, hipStream_t s);
hipError_t launch_add_dots(float* dst, const float* a, const float* b, int64_t groups, int64_t N,
                           int64_t bs, float* part, hipStream_t s);
hipError_t launch_add_sums(float* dst, const float* src, int64_t groups, int64_t N, int64_t bs,
                           float* part, hipStream_t s);
// Derivative (delta *= f'(output)) fused into addSums' chains (same bits)
hipError_t launch_derive_add_sums(float* dst, float* delta, const float* output, int act,
                                  int64_t groups, int64_t N, int64_t bs, float* part,
                                  hipStream_t s);
hipError_t launch_mean_var_delta(const float* delta, const float* x, const float* mean,
                                 const float* var, int64_t groups, int64_t N, int64_t bs,
                                 float* mean_delta, float* var_delta, int quirk, float* part,
                                 hipStream_t s, const float* scales = nullptr);
hipError_t launch_normalize_delta(const float* x, const float* mean, const float* var,
                                  const float* mean_delta, const float* var_delta, float* delta,
                                  int64_t groups, int64_t N, int64_t bs, hipStream_t s, const float* scales = nullptr); 
// whether launch_mean_var_delta / launch_normalize_delta can fold the BN
// scales into their loads for planes of bs pixels (else forwardScale first)
bool bn_folds_scale(int64_t bs);
// the BN conv backward in one chain pass + normalizeDelta (CH_BNB);
// hipErrorNotSupported where it does not apply (run the separate passes).
// part: 3 * groups * N floats
hipError_t launch_bn_backward_fused(float* scale_updates, const float* x_norm, float* delta,
                                    const float* output, int act, const float* x,
                                    const float* mean, const float* var, const float* scales,
                                    float* mean_delta, float* var_delta, int64_t groups,
                                    int64_t N, int64_t bs, int quirk, float* part, hipStream_t s);
// the BN conv backward's Derivative + addDots in one pass where the chain
// kernels allow (else the two passes)
hipError_t launch_add_dots_derive(float* dst, const float* x_norm, float* delta,
                                  const float* output, int act, int64_t groups, int64_t N,
                                  int64_t bs, float* part, hipStream_t s);
// fused conv-layer BN forward: x := y, xn := normalize(y), out :=
// act(xn*scale + bias); x / xn may be nullptr (inference); out may alias y
hipError_t launch_bn_apply(const float* y, float* x, float* xn, float* out, int64_t groups,
                           int64_t N, int64_t bs, const float* means, const float* vars,
                           const float* scales, const float* biases, int act, hipStream_t s);
hipError_t launch_rolling_update(int64_t n, float* rm, float* rv, const float* mean,
                                 const float* var, float momentum, hipStream_t s);
hipError_t launch_softmax_batch(int64_t n, const float* in, int64_t batch, int64_t batch_size,
                                int64_t groups, int64_t group_size, int64_t stride, float temp,
                                float* out, hipStream_t s);
hipError_t launch_xent_softmax(int64_t n, const float* pred, const float* truth, float* delta,
                               float* error, hipStream_t s);
hipError_t launch_vssum(int64_t n, const float* a, float* out, hipStream_t s);

// ---- fused connected-network train step (mlp_train.hip) ---------------------
constexpr int MLP_MAX_LAYERS = 16;
struct MlpArgs {
  int nlayers;
  int64_t widths[MLP_MAX_LAYERS + 1];
  int acts[MLP_MAX_LAYERS];
  int bn;
  int64_t batch;
  const float* X;
  const float* truth;
  float lr, momentum, decay;
  float* buf;   // packed parameters / state, layout of ora_mlp_train_step
  float* cost;  // one float
  // filled by launch_mlp_train_step: element offsets of each layer's arrays
  int64_t off[MLP_MAX_LAYERS][16];
  int64_t softmax_off;
  int64_t stamp_off;  // end of the packed buffer (diagnostic stamp builds only)
  int lds_chunks;     // forward gemm operands staged through LDS in k-chunks
  int64_t act_off;    // LDS float offset of the stage-to-stage [B][O_max] block
  float* l0part;      // layer 0's residue partials [8][B][O0] (mlp_l0_forward_kernel)
};
int64_t mlp_buffer_floats(int nlayers, const int64_t* widths, int bn, int64_t batch);
hipError_t launch_mlp_train_step(const MlpArgs& a, hipStream_t s);

}  // namespace tns
