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
    "ora_shortcut": (C.c_int, [i64, fp, fp, fp, i32]),
    "ora_upsample": (None, [i64, i64, i64, i64, f32, fp, fp]),
    "ora_yolo_forward": (None, [i64, i64, i64, i64, fp, fp]),
    "ora_gradient": (C.c_int, [fp, i64, i32, fp]),
    "ora_conv2d": (None, [i64, i64, i64, i64, fp, fp, i64, i64, i64, i64, i64, i64, i64, i64, i64,
                          fp, fp]),
    "ora_conv_forward": (None, [i64, i64, i64, i64, fp, fp, fp, i64, i64, i64, i64, i64, i32, fp,
                                fp]),
    "ora_fuse_batchnorm": (None, [i64, i64, fp, fp, fp, fp, fp]),
    "ora_conv_backward": (C.c_int, [i64, i64, i64, i64, fp, fp, i64, i64, i64, i64, i64, i32,
                                    fp, fp, fp, fp, fp, fp]),
    "ora_fill_uniform": (None, [fp, i64, C.c_uint64, C.c_uint64, f32, f32]),
    "ora_conv_backward_oh": (i64, [i64, i64, i64, i64, i64]),
    "ora_conv_forward_train": (None, [i64, i64, i64, i64, fp, fp, i64, i64, i64, i64, i64, i32,
                                      fp, fp, fp, fp, f32, i32, fp, fp, fp, fp, fp, fp, i32]),
    "ora_conv_backward_bn": (C.c_int, [i64, i64, i64, i64, fp, fp, i64, i64, i64, i64, i64, i32,
                                       fp, fp, fp, fp, fp, fp, fp, fp, fp, fp, fp, fp, fp, i32]),
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


def shortcut(a: np.ndarray, b: np.ndarray, act: int) -> np.ndarray:
    out = np.empty_like(a)
    rc = lib().ora_shortcut(a.size, _p(a), _p(b), _p(out), act)
    assert rc == 0, act
    return out


def upsample(x: np.ndarray, planes: int, h: int, w: int, stride: int, scale: float = 1.0):
    out = np.empty(planes * h * stride * w * stride, np.float32)
    lib().ora_upsample(planes, h, w, stride, scale, _p(x), _p(out))
    return out


def yolo_forward(x: np.ndarray, batch: int, anchors: int, classes: int, hw: int) -> np.ndarray:
    out = np.empty_like(x)
    lib().ora_yolo_forward(batch, anchors, classes, hw, _p(x), _p(out))
    return out


def concat(tensors) -> np.ndarray:
    """TTensor.concat (ntensors.pas:12045-12061): whole tensors, in order."""
    return np.concatenate([np.ascontiguousarray(t).ravel() for t in tensors])


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


def conv_backward(x, w, filters, k, stride, pad, act, output, delta, bias_updates,
                  weight_updates, state_delta=None, dil=1):
    """Restated TConvolutionalLayer.backward; updates delta, bias_updates,
    weight_updates (and state_delta if given) in place."""
    batch, C_, H, W = x.shape
    oh, ow = out_dim(H, pad * dil, k, dil, stride), out_dim(W, pad * dil, k, dil, stride)
    ws = np.zeros(max(batch * C_ * k * k * oh * ow, 1), np.float32)
    rc = lib().ora_conv_backward(batch, C_, H, W, _p(x), _p(w), filters, k, stride, pad, dil,
                                 act, _p(output), _p(delta), _p(bias_updates),
                                 _p(weight_updates), _p(ws),
                                 _p(state_delta) if state_delta is not None else None)
    assert rc == 0, rc


def conv_forward_train(x, w, filters, k, stride, pad, act, scales, biases, rmean, rvar,
                       momentum, training, dil=1, quirk=0):
    """Restated TConvolutionalLayer.forward with batch norm.  Updates
    rmean / rvar in place; returns (out, mean, var, x, x_norm)."""
    batch, C_, H, W = x.shape
    oh, ow = out_dim(H, pad, k, dil, stride), out_dim(W, pad, k, dil, stride)
    ws = np.zeros(max(batch * C_ * k * k * oh * ow, 1), np.float32)
    out = np.zeros((batch, filters, oh, ow), np.float32)
    m, v = np.zeros(filters, np.float32), np.zeros(filters, np.float32)
    xs, xn = np.zeros_like(out), np.zeros_like(out)
    lib().ora_conv_forward_train(batch, C_, H, W, _p(x), _p(w), filters, k, stride, pad, dil, act,
                                 _p(scales), _p(biases), _p(rmean), _p(rvar), momentum,
                                 int(training), _p(m), _p(v), _p(xs), _p(xn), _p(ws), _p(out),
                                 int(quirk))
    return out, m, v, xs, xn


def conv_backward_bn(x, w, filters, k, stride, pad, act, output, delta, scales, xs, xn, mean,
                     var, scale_updates, weight_updates, state_delta=None, dil=1, quirk=0):
    """Restated TConvolutionalLayer.backward with batchNormBack; updates delta,
    scale_updates, weight_updates (and state_delta) in place; returns
    (mean_delta, variance_delta)."""
    batch, C_, H, W = x.shape
    oh, ow = out_dim(H, pad * dil, k, dil, stride), out_dim(W, pad * dil, k, dil, stride)
    ws = np.zeros(max(batch * C_ * k * k * oh * ow, 1), np.float32)
    md, vd = np.zeros(filters, np.float32), np.zeros(filters, np.float32)
    rc = lib().ora_conv_backward_bn(batch, C_, H, W, _p(x), _p(w), filters, k, stride, pad, dil,
                                    act, _p(output), _p(delta), _p(scales), _p(xs), _p(xn),
                                    _p(mean), _p(var), _p(scale_updates), _p(md), _p(vd),
                                    _p(weight_updates), _p(ws),
                                    _p(state_delta) if state_delta is not None else None,
                                    int(quirk))
    assert rc == 0, rc
    return md, vd


_PROTO2 = {
    "ora_vssum": (f32, [i64, fp]),
    "ora_sgd_update": (None, [i64, fp, fp, i64, fp, fp, fp, fp, f32, f32, f32]),
    "ora_means_and_vars": (None, [fp, i64, i64, i64, fp, fp]),
    "ora_means_and_vars_q": (None, [fp, i64, i64, i64, fp, fp, i32]),
    "ora_normalize": (None, [fp, i64, i64, i64, fp, fp]),
    "ora_batch_norm": (None, [fp, i64, i64, i64, fp, fp, fp, fp, f32, i32, fp, fp, fp, fp, i32]),
    "ora_forward_scale": (None, [fp, i64, i64, i64, fp]),
    "ora_add_dots": (None, [fp, fp, fp, i64, i64, i64]),
    "ora_add_sums": (None, [fp, fp, i64, i64, i64]),
    "ora_mean_var_delta": (None, [fp, fp, fp, fp, i64, i64, i64, fp, fp]),
    "ora_mean_var_delta_q": (None, [fp, fp, fp, fp, i64, i64, i64, fp, fp, i32]),
    "ora_var_delta_avx": (f32, [i64, f32, fp, fp, i32]),
    "ora_srss": (f32, [i64, f32, fp, i32]),
    "ora_normalize_delta": (None, [fp, fp, fp, fp, fp, fp, i64, i64, i64]),
    "ora_softmax": (None, [i64, fp, f32, i64, fp]),
    "ora_softmax_xent": (None, [i64, fp, fp, fp, fp]),
    "ora_clamp": (None, [fp, i64, f32, f32]),
    "ora_mlp_train_step": (f32, [i32, C.POINTER(i64), C.POINTER(i32), i32, i64, fp, fp, f32, f32,
                                 f32, fp]),
    "ora_mlp_buffer_floats": (i64, [i32, C.POINTER(i64), i32, i64]),
}


def _lib2():
    L = lib()
    if not getattr(L, "_tns_p2", False):
        for n, (r, a) in _PROTO2.items():
            f = getattr(L, n)
            f.restype = r
            f.argtypes = a
        L._tns_p2 = True
    return L


def vssum(a):
    return float(_lib2().ora_vssum(a.size, _p(a)))


def means_and_vars(x, groups, N, bs, quirk=0):
    m = np.zeros(N, np.float32)
    v = np.zeros(N, np.float32)
    _lib2().ora_means_and_vars_q(_p(x), groups, N, bs, _p(m), _p(v), int(quirk))
    return m, v


def normalize(x, groups, N, bs, m, v):
    _lib2().ora_normalize(_p(x), groups, N, bs, _p(m), _p(v))
    return x


def batch_norm(out, groups, N, bs, scales, biases, rmean, rvar, momentum, training, quirk=0):
    """Restated TBaseLayer.batchNorm (nbaselayer.pas:336-370) on out in place;
    rmean / rvar updated in place; returns (mean, var, x, x_norm)."""
    m, v = np.zeros(N, np.float32), np.zeros(N, np.float32)
    x, xn = np.zeros_like(out), np.zeros_like(out)
    _lib2().ora_batch_norm(_p(out), groups, N, bs, _p(scales), _p(biases), _p(rmean), _p(rvar),
                           float(momentum), int(bool(training)), _p(m), _p(v), _p(x), _p(xn),
                           int(quirk))
    return m, v, x, xn


def forward_scale(x, groups, N, bs, s):
    _lib2().ora_forward_scale(_p(x), groups, N, bs, _p(s))
    return x


def add_dots(dst, a, b, groups, N, bs):
    _lib2().ora_add_dots(_p(dst), _p(a), _p(b), groups, N, bs)
    return dst


def add_sums(dst, src, groups, N, bs):
    _lib2().ora_add_sums(_p(dst), _p(src), groups, N, bs)
    return dst


def sgd_update(W, dW, b, db, scales, dscales, lrb, ndb, momentum):
    """TConnectedLayer/TConvolutionalLayer.update in place (ora_sgd_update)."""
    _lib2().ora_sgd_update(W.size, _p(W), _p(dW), b.size, _p(b), _p(db),
                           _p(scales) if scales is not None else None,
                           _p(dscales) if dscales is not None else None,
                           lrb, ndb, momentum)


def mean_var_delta(delta, x, mean, var, groups, N, bs, quirk=0):
    md = np.zeros(N, np.float32)
    vd = np.zeros(N, np.float32)
    _lib2().ora_mean_var_delta_q(_p(delta), _p(x), _p(mean), _p(var), groups, N, bs, _p(md),
                                 _p(vd), int(quirk))
    return md, vd


def var_delta_avx(mean, delta, x, quirk=0):
    """sVarinceDelta_avx over one block (ntensors.pas:8721-8757)."""
    return float(_lib2().ora_var_delta_avx(delta.size, mean, _p(delta), _p(x), int(quirk)))


def srss(mean, a, quirk=0):
    """srss over one block (ntensors.pas:1493-1523)."""
    return float(_lib2().ora_srss(a.size, mean, _p(a), int(quirk)))


def normalize_delta(x, mean, var, md, vd, delta, groups, N, bs):
    _lib2().ora_normalize_delta(_p(x), _p(mean), _p(var), _p(md), _p(vd), _p(delta), groups, N,
                                bs)
    return delta


def softmax_rows(x, n, temp=1.0):
    out = np.zeros_like(x)
    rows = x.size // n
    L = _lib2()
    for r in range(rows):
        L.ora_softmax(n, x.ctypes.data + 4 * r * n, temp, 1, out.ctypes.data + 4 * r * n)
    return out


def softmax_xent(pred, truth):
    d = np.zeros_like(pred)
    e = np.zeros_like(pred)
    _lib2().ora_softmax_xent(pred.size, _p(pred), _p(truth), _p(d), _p(e))
    return d, e


def mlp_buffer_floats(widths, bn, batch):
    w = (C.c_int64 * len(widths))(*widths)
    return int(_lib2().ora_mlp_buffer_floats(len(widths) - 1, w, 1 if bn else 0, batch))


def mlp_train_step(widths, acts, bn, batch, X, truth, lr, momentum, decay, buf):
    w = (C.c_int64 * len(widths))(*widths)
    a = (C.c_int32 * len(acts))(*acts)
    return float(_lib2().ora_mlp_train_step(len(widths) - 1, w, a, 1 if bn else 0, batch, _p(X),
                                            _p(truth), lr, momentum, decay, _p(buf)))


def mlp_init(widths, bn, batch, seed=5):
    """Buffer with parameters initialised like TConnectedLayer.Create
    (W ~ U[-sqrt(2/inputs), sqrt(2/inputs)], biases 0, scales 1)."""
    buf = np.zeros(mlp_buffer_floats(widths, bn, batch), np.float32)
    off = 0
    for l in range(len(widths) - 1):
        I, O = widths[l], widths[l + 1]
        r = float(np.sqrt(2.0 / I))
        buf[off:off + I * O] = uniform(I * O, seed, 100 + l, -r, r)
        off += I * O          # W
        off += O              # b (zeros)
        off += I * O + O      # dW, db
        if bn:
            buf[off:off + O] = 1.0   # scales
            off += 4 * O
        off += 2 * batch * O  # out, delta
        if bn:
            off += 2 * batch * O + 4 * O
    return buf


def mnist_batch(batch, seed=5, classes=10, inputs=784):
    X = uniform(batch * inputs, seed, 1, 0.0, 1.0)
    lab = (uniform(batch, seed, 2, 0.0, 1.0) * classes).astype(np.int64) % classes
    T = np.zeros((batch, classes), np.float32)
    T[np.arange(batch), lab] = 1.0
    return X, T.ravel()


def darknet_forward(net, params, x):
    """TNNet.forward restated over a tensorium_amd.darknet.Network: every
    layer's output (float32, flat), convolutions with BN folded first
    (ora_fuse_batchnorm = fuseBatchNorm, nConvolutionLayer.pas:102-126)."""
    B = net.batch
    outs = []
    prev = np.ascontiguousarray(x, np.float32).ravel()
    ci = 0
    for l in net.layers:
        if l.kind == "convolutional":
            p = params[ci]
            ci += 1
            w = np.ascontiguousarray(p.weights, np.float32).ravel().copy()
            b = np.ascontiguousarray(p.biases, np.float32).copy()
            if l.bn:
                sc, rm, rv = (np.ascontiguousarray(t, np.float32) for t in
                              (p.scales, p.rolling_mean, p.rolling_var))
                lib().ora_fuse_batchnorm(l.filters, l.c * l.size * l.size, _p(w), _p(b), _p(sc),
                                         _p(rm), _p(rv))
            y = conv_forward(prev.reshape(B, l.c, l.h, l.w), w, b, l.filters, l.size, l.stride,
                             l.pad, l.activation).ravel()
        elif l.kind == "shortcut":
            y = shortcut(prev, outs[l.inputs[0]], l.activation)
        elif l.kind == "route":
            y = concat([outs[s] for s in l.inputs])
        elif l.kind == "upsample":
            y = upsample(prev, B * l.c, l.h, l.w, l.stride, 1.0)
        elif l.kind == "yolo":
            y = yolo_forward(prev, B, l.anchors, l.classes, l.h * l.w)
        else:
            raise ValueError(l.kind)
        outs.append(y)
        prev = y
    return outs

