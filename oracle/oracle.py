"""TEST INFRASTRUCTURE ONLY — ctypes binding of oracle/libtns_oracle.so.

The CPU restatement of the reference hot path (see tns_oracle.h).  Imported
only by tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg,
as the checker / baseline; the product (tensorium_amd, libtensorium_hip.so)
never imports it.  PARITY UNPINNED by reference artefacts — see DESIGN.md.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "libtns_oracle.so"

i32, i64, f32, fp = C.c_int32, C.c_int64, C.c_float, C.c_void_p
_CONV = [i64] * 11

_PROTO = {
    "ora_set_threads": (None, [C.c_int]),
    "ora_get_threads": (C.c_int, []),
    "ora_saxpy": (None, [i64, f32, fp, fp]),
    "ora_sdot": (f32, [i64, fp, fp]),
    "ora_sgemm": (None, [i32, i32, i32, i64, i64, i64, f32, fp, i64, fp, i64, f32, fp, i64]),
    "ora_sgemm_rows": (None, [i32, i32, i64, i64, i64, i64, i64, f32, fp, i64, fp, i64, f32, fp,
                              i64]),
    "ora_sgemm_batch_strided": (None, [i32, i32, i32, i64, i64, i64, f32, fp, i64, i64, fp, i64,
                                       i64, f32, fp, i64, i64, i64]),
    "ora_im2col": (None, [*_CONV, fp, i64, fp, i64]),
    "ora_im2col_strided_batched": (None, [*_CONV, fp, i64, i64, fp, i64, i64, i64]),
    "ora_col2im": (None, [*_CONV, fp, i64, fp, i64]),
    "ora_col2im_strided_batched": (None, [*_CONV, fp, i64, i64, fp, i64, i64, i64]),
    "ora_add_bias": (None, [i64, fp, i64, fp, i64, i64]),
    "ora_backward_bias": (None, [i64, fp, i64, i64, fp]),
    "ora_activate": (C.c_int, [fp, i64, i32]),
    "ora_gradient": (C.c_int, [fp, i64, i32, fp]),
    "ora_conv2d": (None, [i64, i64, i64, i64, fp, fp, i64, i64, i64, i64, i64, i64, i64, i64, i64,
                          fp, fp]),
    "ora_conv_forward": (None, [i64, i64, i64, i64, fp, fp, fp, i64, i64, i64, i64, i64, i32, fp,
                                fp]),
    "ora_fuse_batchnorm": (None, [i64, i64, fp, fp, fp, fp, fp]),
    "ora_fill_uniform": (None, [fp, i64, C.c_uint64, C.c_uint64, f32, f32]),
}

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} not built (make -C oracle)")
        _lib = C.CDLL(str(LIB_PATH))
        for n, (r, a) in _PROTO.items():
            f = getattr(_lib, n)
            f.restype = r
            f.argtypes = a
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data


def set_threads(n: int) -> None:
    lib().ora_set_threads(int(n))


def uniform(shape, seed: int, stream: int, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    x = np.empty(shape, np.float32)
    lib().ora_fill_uniform(_p(x), x.size, seed, stream, lo, hi)
    return x


def sdot(a: np.ndarray, b: np.ndarray) -> float:
    return float(lib().ora_sdot(a.size, _p(a), _p(b)))


def sgemm(transA: bool, transB: bool, M, N, K, alpha, A, lda, B, ldb, beta, C_, ldc):
    lib().ora_sgemm(101, 112 if transA else 111, 112 if transB else 111, M, N, K, alpha, _p(A),
                    lda, _p(B), ldb, beta, _p(C_), ldc)
    return C_


def sgemm_rows(transA, transB, row0, row1, M, N, K, alpha, A, lda, B, ldb, beta, C_, ldc):
    lib().ora_sgemm_rows(112 if transA else 111, 112 if transB else 111, row0, row1, M, N, K,
                         alpha, _p(A), lda, _p(B), ldb, beta, _p(C_), ldc)
    return C_


def sgemm_batch_strided(transA, transB, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C_, ldc,
                        sC, batch):
    lib().ora_sgemm_batch_strided(101, 112 if transA else 111, 112 if transB else 111, M, N, K,
                                  alpha, _p(A), lda, sA, _p(B), ldb, sB, beta, _p(C_), ldc, sC,
                                  batch)
    return C_


def out_dim(inp, pad, k, dil, stride):
    v = inp + 2 * pad - (dil * (k - 1) + 1)
    q = abs(v) // stride
    return (q if v >= 0 else -q) + 1   # Pascal div truncates toward zero


def im2col(C_, H, W, kH, kW, pH, pW, sY, sX, dY, dX, im: np.ndarray, batch=1) -> np.ndarray:
    oh, ow = out_dim(H, pH, kH, dY, sY), out_dim(W, pW, kW, dX, sX)
    col = np.full((batch, C_ * kH * kW, max(oh, 0) * max(ow, 0)), np.nan, np.float32)
    lib().ora_im2col_strided_batched(C_, H, W, kH, kW, pH, pW, sY, sX, dY, dX, _p(im),
                                     C_ * H * W, 0, _p(col), col[0].size, 0, batch)
    return col


def col2im(C_, H, W, kH, kW, pH, pW, sY, sX, dY, dX, col: np.ndarray, im: np.ndarray,
           batch=1) -> np.ndarray:
    lib().ora_col2im_strided_batched(C_, H, W, kH, kW, pH, pW, sY, sX, dY, dX, _p(col),
                                     col.size // batch, 0, _p(im), C_ * H * W, 0, batch)
    return im


def add_bias(x: np.ndarray, bias: np.ndarray, filters: int, block: int, batch: int):
    lib().ora_add_bias(filters, _p(x), block, _p(bias), 1, batch)
    return x


def activate(x: np.ndarray, act: int) -> np.ndarray:
    rc = lib().ora_activate(_p(x), x.size, act)
    if rc:
        raise ValueError(f"activation {act} not in oracle")
    return x


def gradient(y: np.ndarray, act: int, delta: np.ndarray) -> np.ndarray:
    rc = lib().ora_gradient(_p(y), y.size, act, _p(delta))
    if rc:
        raise ValueError(f"gradient {act} not in oracle")
    return delta


def conv2d(x, w, filters, k, pad, stride, dil=1):
    batch, C_, H, W = x.shape
    oh, ow = out_dim(H, pad, k, dil, stride), out_dim(W, pad, k, dil, stride)
    ws = np.zeros(max(batch * C_ * k * k * oh * ow, 1), np.float32)
    out = np.zeros((batch, filters, oh, ow), np.float32)
    lib().ora_conv2d(batch, C_, H, W, _p(x), _p(w), filters, k, k, pad, pad, stride, stride, dil,
                     dil, _p(ws), _p(out))
    return out


def conv_forward(x, w, b, filters, k, stride, pad, act, dil=1):
    batch, C_, H, W = x.shape
    oh, ow = out_dim(H, pad, k, dil, stride), out_dim(W, pad, k, dil, stride)
    ws = np.zeros(max(batch * C_ * k * k * oh * ow, 1), np.float32)
    out = np.zeros((batch, filters, oh, ow), np.float32)
    lib().ora_conv_forward(batch, C_, H, W, _p(x), _p(w), _p(b), filters, k, stride, pad, dil,
                           act, _p(ws), _p(out))
    return out
