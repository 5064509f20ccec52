"""TNNHip — the device-resident HIP backend, shaped like the reference's
TNNCuda<T> (source/nncuda.pas:35-157) / TNNOpenCL<T> (nnopencl.pas:222-319).

Method names, argument order and meaning follow TNNCuda: device buffers plus
ELEMENT offsets, calls asynchronous on the backend's stream, ``finish()``
synchronises.  Device buffers are torch CUDA tensors (fp32, contiguous) or raw
integer device pointers; torch is only plumbing for memory and streams — all
compute runs in libtensorium_hip.so.  Errors raise ``TnsError`` the way the
reference's SAFE_CALL raises (nncuda.pas:216-275).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._abi import TnsError, check, load

try:  # torch is optional plumbing
    import torch
except Exception:  # pragma: no cover
    torch = None


CONV_UNFUSED, CONV_FUSED, CONV_IM2COL, CONV_IMPLICIT = 0, 1, 2, 3


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if torch is not None and isinstance(x, torch.Tensor):
        if not x.is_cuda:
            raise TnsError("TNNHip expects device (cuda) tensors")
        if x.dtype != torch.float32:
            raise TnsError(f"TNNHip expects float32 tensors, got {x.dtype}")
        if not x.is_contiguous():
            raise TnsError("TNNHip expects contiguous tensors")
        return x.data_ptr()
    raise TnsError(f"unsupported buffer type {type(x)!r}")


class TNNHip:
    """HIP twin of TNNCuda<single> (one context = one device + one stream)."""

    def __init__(self, deviceIndex: int = 0, stream=None, use_torch_stream: bool = True):
        self.lib = load()
        h = C.c_void_p()
        check(self.lib.tns_hip_create(int(deviceIndex), C.byref(h)))
        self.ctx = h
        self.device = int(deviceIndex)
        if stream is not None:
            check(self.lib.tns_hip_set_stream(self.ctx, C.c_void_p(int(stream))))
        elif use_torch_stream and torch is not None and torch.cuda.is_available():
            s = torch.cuda.current_stream(self.device).cuda_stream
            check(self.lib.tns_hip_set_stream(self.ctx, C.c_void_p(s)))

    # -- lifecycle --------------------------------------------------------
    def close(self):
        if getattr(self, "ctx", None):
            self.lib.tns_hip_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        # (NULL with an error set: the join of pending dW products failed —
        # handing out 0, the null stream, would order nothing after them;
        # NULL without one is the legacy default stream the context runs on)
        self.lib.tns_clear_error()
        s = self.lib.tns_hip_get_stream(self.ctx)
        if not s:
            msg = self.lib.tns_last_error().decode(errors="replace")
            if msg:
                self.lib.tns_clear_error()
                raise TnsError(f"tns_hip_get_stream: {msg}")
        return int(s or 0)

    def pendingDw(self) -> int:
        """dW products of a pipelined conv backward still on the side stream
        (tns_hip_pending_dw; 0 once joined)."""
        return int(self.lib.tns_hip_pending_dw(self.ctx))

    def finish(self):  # TNNCuda.finish, nncuda.pas:1575
        check(self.lib.tns_hip_finish(self.ctx))

    def setTelemetry(self, on: bool):
        check(self.lib.tns_hip_set_telemetry(self.ctx, 1 if on else 0))

    def opMs(self, op: int) -> float:
        return float(self.lib.tns_hip_op_ms(self.ctx, op))

    # -- GEMM ----------------------------------------------------------------
    def gemm(self, transA, transB, M, N, K, ALPHA, A, aOffset, lda, B, bOffset, ldb, BETA, C_,
             cOffset, ldc):
        check(self.lib.tns_hip_gemm(self.ctx, int(bool(transA)), int(bool(transB)), M, N, K,
                                    float(ALPHA), _ptr(A), aOffset, lda, _ptr(B), bOffset, ldb,
                                    float(BETA), _ptr(C_), cOffset, ldc))

    def gemmStridedBatched(self, transA, transB, M, N, K, ALPHA, A, aOffset, lda, strideA, B,
                           bOffset, ldb, strideB, BETA, C_, cOffset, ldc, strideC, batchCount):
        check(self.lib.tns_hip_gemm_strided_batched(
            self.ctx, int(bool(transA)), int(bool(transB)), M, N, K, float(ALPHA), _ptr(A),
            aOffset, lda, strideA, _ptr(B), bOffset, ldb, strideB, float(BETA), _ptr(C_), cOffset,
            ldc, strideC, batchCount))

    def gemmBatched(self, transA, transB, M, N, K, ALPHA, A, aOffset, lda, B, bOffset, ldb,
                    BETA, C_, cOffset, ldc, batchCount):
        """TNNCuda.gemmBatched (nncuda.pas:727): A, B, C are arrays of matrix
        pointers — device buffers holding them (int64 tensors, as the
        reference's writeBuffer-built arrays) or raw addresses."""
        def arr(x):
            if torch is not None and isinstance(x, torch.Tensor):
                if x.dtype != torch.int64 or not x.is_contiguous():
                    raise TnsError("gemmBatched pointer arrays are contiguous int64 tensors")
                return x.data_ptr()
            return int(x)
        check(self.lib.tns_hip_gemm_batched(
            self.ctx, int(bool(transA)), int(bool(transB)), M, N, K, float(ALPHA), arr(A),
            aOffset, lda, arr(B), bOffset, ldb, float(BETA), arr(C_), cOffset, ldc, batchCount))

    def gemmVariant(self, variant, transA, transB, M, N, K, ALPHA, A, aOffset, lda, strideA, B,
                    bOffset, ldb, strideB, BETA, C_, cOffset, ldc, strideC, batchCount=1):
        """Force one SGEMM tile shape (tuning sweeps); variant < 0 = heuristic."""
        check(self.lib.tns_hip_gemm_variant(
            self.ctx, int(variant), int(bool(transA)), int(bool(transB)), M, N, K, float(ALPHA),
            _ptr(A), aOffset, lda, strideA, _ptr(B), bOffset, ldb, strideB, float(BETA), _ptr(C_),
            cOffset, ldc, strideC, batchCount))

    @staticmethod
    def gemmVariants() -> list[str]:
        lib = load()
        return [lib.tns_gemm_variant_name(i).decode() for i in range(lib.tns_gemm_variant_count())]

    # -- im2col / col2im --------------------------------------------------------
    def im2col(self, aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth,
               strideY, strideX, dilationY, dilationX, im, imOffset, col, colOffset):
        check(self.lib.tns_hip_im2col(self.ctx, aChannels, aHeight, aWidth, kernelHeight,
                                      kernelWidth, padHeight, padWidth, strideY, strideX,
                                      dilationY, dilationX, _ptr(im), imOffset, _ptr(col),
                                      colOffset))

    def im2colStridedBatched(self, aChannels, aHeight, aWidth, kernelHeight, kernelWidth,
                             padHeight, padWidth, strideY, strideX, dilationY, dilationX, im,
                             imStride, imOffset, col, colStride, colOffset, batchCount):
        check(self.lib.tns_hip_im2col_strided_batched(
            self.ctx, aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth,
            strideY, strideX, dilationY, dilationX, _ptr(im), imStride, imOffset, _ptr(col),
            colStride, colOffset, batchCount))

    def col2im(self, aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth,
               strideY, strideX, dilationY, dilationX, col, colOffset, im, imOffset):
        check(self.lib.tns_hip_col2im(self.ctx, aChannels, aHeight, aWidth, kernelHeight,
                                      kernelWidth, padHeight, padWidth, strideY, strideX,
                                      dilationY, dilationX, _ptr(col), colOffset, _ptr(im),
                                      imOffset))

    def col2imStridedBatched(self, aChannels, aHeight, aWidth, kernelHeight, kernelWidth,
                             padHeight, padWidth, strideY, strideX, dilationY, dilationX, col,
                             colStride, colOffset, im, imStride, imOffset, batchCount):
        check(self.lib.tns_hip_col2im_strided_batched(
            self.ctx, aChannels, aHeight, aWidth, kernelHeight, kernelWidth, padHeight, padWidth,
            strideY, strideX, dilationY, dilationX, _ptr(col), colStride, colOffset, _ptr(im),
            imStride, imOffset, batchCount))

    # -- elementwise -------------------------------------------------------------
    def forwardBias(self, dstSize, dst, offset, srcSize, src, incb, batch):
        check(self.lib.tns_hip_forward_bias(self.ctx, dstSize, _ptr(dst), offset, srcSize,
                                            _ptr(src), incb, batch))

    def backwardBias(self, dstSize, dst, srcSize, src, srcOffset, incb, batch):
        check(self.lib.tns_hip_backward_bias(self.ctx, dstSize, _ptr(dst), srcSize, _ptr(src),
                                             srcOffset, incb, batch))

    def ActivateArray(self, N, x, offset, activation):
        check(self.lib.tns_hip_activate_array(self.ctx, N, _ptr(x), offset, int(activation)))

    def DeriveArray(self, N, x, offset, activation, delta):
        check(self.lib.tns_hip_derive_array(self.ctx, N, _ptr(x), offset, int(activation),
                                            _ptr(delta)))

    def axpy(self, N, a, x, xOffset, incx, y, yOffset, incy):
        check(self.lib.tns_hip_axpy(self.ctx, N, float(a), _ptr(x), xOffset, incx, _ptr(y),
                                    yOffset, incy))

    def sgdUpdate(self, weights, weight_updates, biases, bias_updates, learningRate, batch,
                  decay, momentum, scales=None, scale_updates=None):
        """TConnectedLayer.update / TConvolutionalLayer.update (learningRate
        already multiplied by learningRateScale for conv layers), fused."""
        f32 = np.float32
        lrb = f32(f32(learningRate) / f32(batch))
        ndb = f32(-f32(decay) * f32(batch))
        check(self.lib.tns_hip_sgd_update(
            self.ctx, weights.numel(), _ptr(weights), _ptr(weight_updates), biases.numel(),
            _ptr(biases), _ptr(bias_updates), _ptr(scales), _ptr(scale_updates), float(lrb),
            float(ndb), float(momentum)))

    def scale(self, N, a, x, stride):
        check(self.lib.tns_hip_scale(self.ctx, N, float(a), _ptr(x), stride))

    def fill(self, N, x, offset, val, stride):
        check(self.lib.tns_hip_fill(self.ctx, N, _ptr(x), offset, float(val), stride))

    def copy(self, N, src, srcOffset, inca, dst, dstOffset, incb):
        check(self.lib.tns_hip_copy(self.ctx, N, _ptr(src), srcOffset, inca, _ptr(dst), dstOffset,
                                    incb))

    def clamp(self, N, alpha, src, dst, stride=1, offset=0):
        check(self.lib.tns_hip_clamp(self.ctx, N, float(alpha), _ptr(src), _ptr(dst), stride,
                                     offset))

    # -- non-convolutional YOLOv3 layers ----------------------------------------
    def shortcut(self, N, a, aOffset, b, bOffset, out, outOffset=0, activation=4):
        """TAddLayer.forward: out = activate(a + b)."""
        check(self.lib.tns_hip_shortcut(self.ctx, N, _ptr(a), aOffset, _ptr(b), bOffset, _ptr(out),
                                        outOffset, int(activation)))

    def upSample(self, aBatch, aChannels, outHeight, outWidth, in_, stride, isForward, scale,
                 out, zeroIn=0):
        """TNNCuda.upSample (nncuda.pas:136): outHeight/outWidth are the small
        tensor's; isForward=1 writes out, isForward=0 accumulates into in_."""
        check(self.lib.tns_hip_upsample(self.ctx, aBatch, aChannels, outHeight, outWidth,
                                        _ptr(in_), stride, int(isForward), float(scale),
                                        _ptr(out), int(zeroIn)))

    def addvv(self, N, src1, src1Offset, inca, src2, src2Offset, incb, dst, dstOffset, incc):
        check(self.lib.tns_hip_addvv(self.ctx, N, _ptr(src1), src1Offset, inca, _ptr(src2),
                                     src2Offset, incb, _ptr(dst), dstOffset, incc))

    def subvv(self, N, src1, src1Offset, inca, src2, src2Offset, incb, dst, dstOffset, incc):
        check(self.lib.tns_hip_subvv(self.ctx, N, _ptr(src1), src1Offset, inca, _ptr(src2),
                                     src2Offset, incb, _ptr(dst), dstOffset, incc))

    def mulvv(self, N, src1, src1Offset, inca, src2, src2Offset, incb, dst, dstOffset, incc):
        check(self.lib.tns_hip_mulvv(self.ctx, N, _ptr(src1), src1Offset, inca, _ptr(src2),
                                     src2Offset, incb, _ptr(dst), dstOffset, incc))

    def fmavv(self, N, src1, src1Offset, inca, src2, src2Offset, incb, src3, src3Offset, incc,
              dst, dstOffset, incd):
        check(self.lib.tns_hip_fmavv(self.ctx, N, _ptr(src1), src1Offset, inca, _ptr(src2),
                                     src2Offset, incb, _ptr(src3), src3Offset, incc, _ptr(dst),
                                     dstOffset, incd))

    def fmavss(self, N, src, offset, scalar, bias, dst):
        check(self.lib.tns_hip_fmavss(self.ctx, N, _ptr(src), offset, float(scalar), float(bias),
                                      _ptr(dst)))

    def inverseSqrt(self, N, alpha, src, dst, stride=1, offset=0):
        check(self.lib.tns_hip_inverse_sqrt(self.ctx, N, float(alpha), _ptr(src), _ptr(dst),
                                            stride, offset))

    def yoloForward(self, batch, anchors, classes, hw, inp, out):
        check(self.lib.tns_hip_yolo_forward(self.ctx, batch, anchors, classes, hw, _ptr(inp),
                                            _ptr(out)))

    # -- layer drivers ------------------------------------------------------------
    def conv2d(self, batch, C_, H, W, input, weights, filters, kH, kW, wPadding, hPadding,
               xStride, yStride, xDilation, yDilation, workspace, out):
        check(self.lib.tns_hip_conv2d(self.ctx, batch, C_, H, W, _ptr(input), _ptr(weights),
                                      filters, kH, kW, wPadding, hPadding, xStride, yStride,
                                      xDilation, yDilation, _ptr(workspace), _ptr(out)))

    def convForward(self, batch, C_, H, W, input, weights, biases, filters, kSize, stride,
                    padding, dilation, activation, workspace, out, fused=True):
        """fused: False/0 reference stages, True/1 library choice, 2 im2col +
        fused epilogue, 3 implicit GEMM (CONV_* constants)."""
        mode = int(fused) if not isinstance(fused, bool) else (CONV_FUSED if fused else 0)
        check(self.lib.tns_hip_conv_forward(self.ctx, batch, C_, H, W, _ptr(input),
                                            _ptr(weights), _ptr(biases), filters, kSize, stride,
                                            padding, dilation, int(activation), _ptr(workspace),
                                            _ptr(out), mode))

    def convBackward(self, batch, C_, H, W, input, weights, filters, kSize, stride, padding,
                     dilation, activation, output, delta, bias_updates, weight_updates,
                     workspace=None, state_delta=None):
        """TConvolutionalLayer.backward (no BN); delta is updated in place."""
        check(self.lib.tns_hip_conv_backward(
            self.ctx, batch, C_, H, W, _ptr(input), _ptr(weights), filters, kSize, stride,
            padding, dilation, int(activation), _ptr(output), _ptr(delta), _ptr(bias_updates),
            _ptr(weight_updates), _ptr(workspace), _ptr(state_delta)))

    def convForwardTrain(self, batch, C_, H, W, input, weights, filters, kSize, stride, padding,
                         dilation, activation, scales, biases, rolling_mean, rolling_variance,
                         bnMomentum, training, mean, variance, x, x_norm, workspace, out):
        """TConvolutionalLayer.forward with batch norm (training or not)."""
        check(self.lib.tns_hip_conv_forward_train(
            self.ctx, batch, C_, H, W, _ptr(input), _ptr(weights), filters, kSize, stride, padding,
            dilation, int(activation), _ptr(scales), _ptr(biases), _ptr(rolling_mean),
            _ptr(rolling_variance), float(bnMomentum), int(bool(training)), _ptr(mean),
            _ptr(variance), _ptr(x), _ptr(x_norm), _ptr(workspace), _ptr(out)))

    def convBackwardBN(self, batch, C_, H, W, input, weights, filters, kSize, stride, padding,
                       dilation, activation, output, delta, scales, x, x_norm, mean, variance,
                       scale_updates, mean_delta, variance_delta, weight_updates, workspace=None,
                       state_delta=None):
        """TConvolutionalLayer.backward with batchNormBack; delta in place."""
        check(self.lib.tns_hip_conv_backward_bn(
            self.ctx, batch, C_, H, W, _ptr(input), _ptr(weights), filters, kSize, stride, padding,
            dilation, int(activation), _ptr(output), _ptr(delta), _ptr(scales), _ptr(x),
            _ptr(x_norm), _ptr(mean), _ptr(variance), _ptr(scale_updates), _ptr(mean_delta),
            _ptr(variance_delta), _ptr(weight_updates), _ptr(workspace), _ptr(state_delta)))

    def setConvVariant(self, variant: int = -1):
        """Force the implicit-GEMM tile shape (-1 = heuristic); process-wide."""
        check(self.lib.tns_set_option(1, int(variant)))

    def setConvPad(self, mode: int = -1):
        """Implicit-GEMM gather: 1 padded copy, 0 bounds-checked, -1 by cost."""
        check(self.lib.tns_set_option(2, int(mode)))

    def setSrssQuirk(self, on: bool = False):
        """Reproduce the reference's srss lane drop in meansAndVars (blocks a
        multiple of 8 long); process-wide."""
        check(self.lib.tns_set_option(4, 1 if on else 0))

    def setNtSdot(self, on: bool = True):
        """gemm(NoTrans, Trans) in the reference's sdot order (default) or as
        one ascending-k chain per element; process-wide."""
        check(self.lib.tns_set_option(3, 1 if on else 0))

    def setSdotForm(self, form: int = -1):
        """Kernel of the sdot-order NT product: -1 by shape, 0 the MFMA
        kernel, 1 + v VALU chain variant v, 64 + v residue-register form v
        (bit-identical); process-wide."""
        check(self.lib.tns_set_option(6, int(form)))

    def setDxFused(self, mode: int = 1):
        """Conv backward state.delta of stride-1 layers: 1 one kernel (each
        tap's filter chain added to the pixel in scol2im's order, no col
        matrix) on the large planes where it is faster, 2 on every layer it
        fits, 0 the reference's TN GEMM + col2im (bit-identical); process-wide."""
        check(self.lib.tns_set_option(7, int(mode)))

    def setDxTile(self, form: int = -1):
        """Conv backward col = W^T . delta: -1 a k-major-A conv tile where one
        applies, -2 the TN GEMM, v >= 0 form v of convDxTiles() (all
        bit-identical); process-wide."""
        check(self.lib.tns_set_option(8, int(form)))

    def setDwTile(self, form: int = -1):
        """Conv backward dW: -1 the implicit-im2col sdot kernel where measured
        faster, -2 im2col + the sdot kernels, v >= 0 form v of convDwTiles()
        (all bit-identical); process-wide."""
        check(self.lib.tns_set_option(9, int(form)))

    def setDxConv(self, form: int = -1):
        """Conv backward state.delta of stride-1 3x3 layers: -1 one implicit
        transposed convolution (each tap's filter chain added to the pixel in
        scol2im's order, no col matrix) where a form applies, -2 off, v >= 0
        form v of convDxConvs() (all bit-identical); process-wide."""
        check(self.lib.tns_set_option(11, int(form)))

    def setDwRes(self, form: int = -1):
        """Conv backward dW: -1 the residue-sequential kernel where picked
        by shape, -2 off, v >= 0 form v of convDwRes() (all bit-identical);
        process-wide."""
        check(self.lib.tns_set_option(12, int(form)))

    def convDwRes(self) -> int:
        """Residue-sequential dW forms of the conv backward."""
        return int(self.lib.tns_conv_dw_res_count())

    def convDxConvs(self) -> int:
        """Implicit transposed-convolution forms of the backward's state.delta."""
        return int(self.lib.tns_conv_dx_conv_count())

    def setBwdOverlap(self, mode=True):
        """Conv backward: dW and state.delta concurrently on two streams,
        joined before the call returns (1 / True), in sequence (0 / False), or
        pipelined (2: each call's dW left running on the side stream behind
        the earlier ones, joined by a later call whose operands meet a pending
        dW's, by finish() or by the stream property); same results;
        process-wide."""
        m = int(mode) if not isinstance(mode, bool) else (1 if mode else 0)
        check(self.lib.tns_set_option(10, m))

    def setScratchCap(self, floats: int = 0):
        """Largest context scratch buffer in floats (0 = none); a larger
        request fails as a failed allocation does; process-wide."""
        check(self.lib.tns_set_option(14, int(floats)))

    def setDeriveSums(self, on: bool = False):
        """Conv backward (no batch norm): Derivative fused into addSums'
        chain pass (True, where it applies) or two passes (False, the
        default); same results; process-wide."""
        check(self.lib.tns_set_option(13, 1 if on else 0))

    def convDwTiles(self) -> int:
        """Implicit-im2col dW tiles of the conv backward."""
        return int(self.lib.tns_conv_dw_tile_count())

    def convDxTiles(self) -> int:
        """k-major-A conv tiles of the backward's col = W^T . delta."""
        return int(self.lib.tns_conv_dx_tile_count())

    def conv1x1Forms(self) -> int:
        """1x1 conv forms reading the input planes by DMA (setConvVariant(600 + v))."""
        return int(self.lib.tns_conv1x1_count())

    def convSlabForms(self) -> int:
        """Two-pass slab conv forms (setConvVariant(500 + v))."""
        return int(self.lib.tns_conv_slab_count())

    def convTileVariants(self) -> int:
        """Plane-sized implicit-conv tiles (setConvVariant(100 + v))."""
        return int(self.lib.tns_conv_tile_variant_count())

    def convPPVariants(self) -> int:
        """Ping-pong implicit-conv tiles (setConvVariant(200 + v))."""
        return int(self.lib.tns_conv_pp_variant_count())

    def convPatchVariants(self) -> int:
        """Input-patch 3x3 stride-1 conv tiles (setConvVariant(400 + v))."""
        return int(self.lib.tns_conv_patch_variant_count())

    def convDMAVariants(self) -> int:
        """LDS-DMA-ring implicit-conv tiles (setConvVariant(300 + v))."""
        return int(self.lib.tns_conv_dma_variant_count())

    def sdotChainsVariants(self) -> int:
        return int(self.lib.tns_sdot_chains_variant_count())

    def sdotRcVariants(self) -> int:
        """Residue-register sdot forms (setSdotForm(64 + v))."""
        return int(self.lib.tns_sdot_rc_variant_count())

    def setTtExact(self, on: bool = True):
        """gemm(Trans, Trans) in the reference's scalar s_tt order on the VALU
        (default) or on the fp32 MFMA kernel; process-wide."""
        check(self.lib.tns_set_option(5, 1 if on else 0))

    # -- batch norm / softmax (TNNCuda.meansAndVars ... crossEntropySoftmax) ----
    def meansAndVars(self, srcSize, dstSize, groups, src, offset, means, vars_):
        check(self.lib.tns_hip_means_and_vars(self.ctx, srcSize, dstSize, groups, _ptr(src),
                                              offset, _ptr(means), _ptr(vars_)))

    def means(self, srcSize, dstSize, groups, src, offset, means):
        """TNNCuda.means (nncuda.pas:1330): the first half of meansAndVars."""
        check(self.lib.tns_hip_means(self.ctx, srcSize, dstSize, groups, _ptr(src), offset,
                                     _ptr(means)))

    def variances(self, srcSize, dstSize, groups, src, offset, means, vars_):
        """TNNCuda.variances (nncuda.pas:1350): the unbiased variance about the
        given means, in MeansAndVars' srss order."""
        check(self.lib.tns_hip_variances(self.ctx, srcSize, dstSize, groups, _ptr(src), offset,
                                         _ptr(means), _ptr(vars_)))

    def normalize(self, srcSize, dstSize, groups, means, meansStride, vars_, varsStride, dst,
                  dstOffset):
        check(self.lib.tns_hip_normalize(self.ctx, srcSize, dstSize, groups, _ptr(means),
                                         meansStride, _ptr(vars_), varsStride, _ptr(dst),
                                         dstOffset))

    def forwardScale(self, dstSize, dst, offset, scaleSize, scale, incb, batch):
        check(self.lib.tns_hip_forward_scale(self.ctx, dstSize, _ptr(dst), offset, scaleSize,
                                             _ptr(scale), incb, batch))

    def forwardScaleAdd(self, dstSize, dst, offset, scaleSize, scales, biases, incb, batch):
        check(self.lib.tns_hip_forward_scale_add(self.ctx, dstSize, _ptr(dst), offset, scaleSize,
                                                 _ptr(scales), _ptr(biases), incb, batch))

    def meansAndVarsDelta(self, srcSize, dstSize, groups, delta, x, offset, mean, variance,
                          mean_delta, variance_delta):
        check(self.lib.tns_hip_means_and_vars_delta(
            self.ctx, srcSize, dstSize, groups, _ptr(delta), _ptr(x), offset, _ptr(mean),
            _ptr(variance), _ptr(mean_delta), _ptr(variance_delta)))

    def normalizeDelta(self, deltaSize, meanSize, groups, delta, x, offset, mean, variance,
                       mean_delta, variance_delta):
        check(self.lib.tns_hip_normalize_delta(
            self.ctx, deltaSize, meanSize, groups, _ptr(delta), _ptr(x), offset, _ptr(mean),
            _ptr(variance), _ptr(mean_delta), _ptr(variance_delta)))

    def addDots(self, N, dstSize, groups, src1, src2, srcOffset, dst):
        check(self.lib.tns_hip_add_dots(self.ctx, N, dstSize, groups, _ptr(src1), _ptr(src2),
                                        srcOffset, _ptr(dst)))

    def softmaxBatch(self, N, input, iOffset, batch, batch_size, groups, group_size, stride, temp,
                     output, oOffset):
        check(self.lib.tns_hip_softmax_batch(self.ctx, N, _ptr(input), iOffset, batch,
                                             batch_size, groups, group_size, stride, float(temp),
                                             _ptr(output), oOffset))

    def crossEntropySoftmax(self, N, pred, truth, delta, error):
        check(self.lib.tns_hip_cross_entropy_softmax(self.ctx, N, _ptr(pred), _ptr(truth),
                                                     _ptr(delta), _ptr(error)))

    def sum(self, N, src, offset, out):
        check(self.lib.tns_hip_sum(self.ctx, N, _ptr(src), offset, _ptr(out)))

    # -- fused connected-network train step (config 5) ---------------------------
    @staticmethod
    def mlpBufferFloats(widths, bn, batch) -> int:
        w = (C.c_int64 * len(widths))(*widths)
        return int(load().tns_mlp_buffer_floats(len(widths) - 1, w, 1 if bn else 0, batch))

    def mlpTrainStep(self, widths, acts, bn, batch, X, truth, lr, momentum, decay, buf, cost):
        w = (C.c_int64 * len(widths))(*widths)
        a = (C.c_int32 * len(acts))(*acts)
        check(self.lib.tns_hip_mlp_train_step(self.ctx, len(widths) - 1, w, a, 1 if bn else 0,
                                              batch, _ptr(X), _ptr(truth), float(lr),
                                              float(momentum), float(decay), _ptr(buf),
                                              _ptr(cost)))


def initHIP(deviceIndex: int = 0, srssQuirk: bool = True) -> TNNHip:
    """initHIP twin of pascal/nnHip.pas (initCUDART, ntensors.pas:6191-6210):
    one backend context for the process, with the reference's configured
    USE_AVX2 BN lane order selected (TNS_OPT_SRSS_QUIRK = 1: srss /
    sVarinceDelta_avx drop lanes 4..7 of blocks a multiple of 8 long,
    ntensors.pas:1509-1511, 8739-8741), so a forwardGPU / backwardGPU caller
    reproduces the CPU build's statistics by default."""
    global hip
    lib = load()
    check(lib.tns_set_option(4, 1 if srssQuirk else 0))
    if hip is None:
        hip = TNNHip(deviceIndex)
    return hip


hip: TNNHip | None = None
