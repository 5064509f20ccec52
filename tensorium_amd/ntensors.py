"""Host-pointer op table — the drop-in for TTensor<Single>'s class-var
procedure pointers (source/ntensors.pas:345-385, bound in
TTensorOps.initSingle, 12651-12758).

``bind_hip_op_table()`` returns the table a Pascal maintainer would assign
after initSingle (``TSingleTensor.gemm := @tns_cblas_sgemm`` …, see
INTEGRATION.md).  ``matMul`` / ``conv2D`` restate the two reference callers
on numpy host arrays so tests read like the reference's own call sites.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ._abi import CblasNoTrans, CblasRowMajor, CblasTrans, TnsError, load


@dataclass
class SingleOpTable:
    gemm: object
    gemmStridedBatched: object
    im2colvv: object
    col2imvv: object
    im2colStridedBatchedvv: object
    col2imStridedBatchedvv: object


def bind_hip_op_table() -> SingleOpTable:
    lib = load()
    return SingleOpTable(
        gemm=lib.tns_cblas_sgemm,
        gemmStridedBatched=lib.tns_cblas_sgemm_batch_strided,
        im2colvv=lib.tns_im2col,
        col2imvv=lib.tns_col2im,
        im2colStridedBatchedvv=lib.tns_im2col_strided_batched,
        col2imStridedBatchedvv=lib.tns_col2im_strided_batched,
    )


def _p(a: np.ndarray):
    if a.dtype != np.float32 or not a.flags["C_CONTIGUOUS"]:
        raise TnsError("host arrays must be C-contiguous float32")
    return a.ctypes.data


def _raise_if_error():
    lib = load()
    msg = lib.tns_last_error()
    if msg:
        lib.tns_clear_error()
        raise TnsError(msg.decode(errors="replace"))


def matMul(a: np.ndarray, b: np.ndarray, c: np.ndarray, transA=False, transB=False,
           ops: SingleOpTable | None = None) -> np.ndarray:
    """TTensor<T>.matMul (ntensors.pas:8059-8140): c += op(a)·op(b) with
    beta = One (accumulates), M = c rows, N = c cols, K = a's inner dim."""
    ops = ops or bind_hip_op_table()
    M, N = c.shape
    K = a.shape[0] if transA else a.shape[1]
    lda = M if transA else K
    ldb = K if transB else N
    ops.gemm(CblasRowMajor, CblasTrans if transA else CblasNoTrans,
             CblasTrans if transB else CblasNoTrans, M, N, K, 1.0, _p(a), lda, _p(b), ldb, 1.0,
             _p(c), N)
    _raise_if_error()
    return c


def conv2D(x: np.ndarray, kernels: np.ndarray, padding: int, stride: int, dilation: int = 1,
           ops: SingleOpTable | None = None) -> np.ndarray:
    """TTensor.Conv2D (ntensors.pas:8252-8349) through the op table:
    im2colStridedBatchedvv then per-image gemm(NN, .., beta=0).
    x: [batch, C, H, W]; kernels: [filters, C, k, k]."""
    ops = ops or bind_hip_op_table()
    batch, C, H, W = x.shape
    F, C2, kH, kW = kernels.shape
    assert C2 == C
    oh = (H + 2 * padding - (dilation * (kH - 1) + 1)) // stride + 1
    ow = (W + 2 * padding - (dilation * (kW - 1) + 1)) // stride + 1
    k = C * kH * kW
    out = np.zeros((batch, F, oh, ow), np.float32)
    if kH * kW != 1 or stride != 1 or dilation != 1:
        ws = np.empty((batch, k, oh * ow), np.float32)
        ops.im2colStridedBatchedvv(C, H, W, kH, kW, padding, padding, stride, stride, dilation,
                                   dilation, _p(x), C * H * W, 0, _p(ws), k * oh * ow, 0, batch)
        _raise_if_error()
        B = ws
    else:
        B = x.reshape(batch, C, H * W)
    w = np.ascontiguousarray(kernels.reshape(F, k))
    for b in range(batch):
        Bb = np.ascontiguousarray(B[b])
        Cb = out[b].reshape(F, oh * ow)
        ops.gemm(CblasRowMajor, CblasNoTrans, CblasNoTrans, F, oh * ow, k, 1.0, _p(w), k, _p(Bb),
                 oh * ow, 0.0, _p(Cb), oh * ow)
        _raise_if_error()
    return out
