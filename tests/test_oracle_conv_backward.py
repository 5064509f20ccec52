"""Restated TConvolutionalLayer.backward (nConvolutionLayer.pas:571-671,
oracle/tns_oracle.c ora_conv_backward) against an independent float64 numpy
statement of the same maths: dW = sum_b delta_b col_b^T, dbias = sum of
delta per filter, dX = col2im(W^T delta_b), delta *= f'(output)."""
import numpy as np
import pytest


def im2col64(x, k, s, p):
    C, H, W = x.shape
    oh, ow = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    xp = np.zeros((C, H + 2 * p, W + 2 * p))
    xp[:, p:p + H, p:p + W] = x
    col = np.empty((C, k, k, oh, ow))
    for kr in range(k):
        for kc in range(k):
            col[:, kr, kc] = xp[:, kr:kr + s * oh:s, kc:kc + s * ow:s]
    return col.reshape(C * k * k, oh * ow)


def col2im64(col, C, H, W, k, s, p):
    oh, ow = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    xp = np.zeros((C, H + 2 * p, W + 2 * p))
    c = col.reshape(C, k, k, oh, ow)
    for kr in range(k):
        for kc in range(k):
            xp[:, kr:kr + s * oh:s, kc:kc + s * ow:s] += c[:, kr, kc]
    return xp[:, p:p + H, p:p + W]


def leaky_grad(y):
    return np.where(y > 0, 1.0, 0.1)


@pytest.mark.parametrize("batch,C,H,F,k,s,p", [(2, 3, 9, 4, 3, 1, 1), (3, 2, 11, 5, 3, 2, 1),
                                               (2, 4, 7, 3, 1, 1, 0)])
def test_conv_backward_vs_float64(ora, batch, C, H, F, k, s, p):
    rng = np.random.default_rng(batch * 100 + C * 10 + H)
    oh = (H + 2 * p - k) // s + 1
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.5, 0.5, F * C * k * k).astype(np.float32)
    out = rng.uniform(-1, 1, (batch, F, oh, oh)).astype(np.float32)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu0 = rng.uniform(-1, 1, F).astype(np.float32)
    wu0 = rng.uniform(-1, 1, F * C * k * k).astype(np.float32)
    sd0 = rng.uniform(-1, 1, x.shape).astype(np.float32)
    delta, bu, wu, sd = d0.copy(), bu0.copy(), wu0.copy(), sd0.copy()
    ora.conv_backward(x, w, F, k, s, p, 9, out, delta, bu, wu, sd)

    # gradient_array leaky: delta *= (y > 0 ? 1 : 0.1f), single float32 multiply
    assert np.array_equal(delta, d0 * np.where(out > 0, np.float32(1), np.float32(0.1)))
    d64 = d0.astype(np.float64) * leaky_grad(out)
    W64 = w.astype(np.float64).reshape(F, -1)
    dW, dX = np.zeros_like(W64), np.zeros(x.shape)
    for b in range(batch):
        col = im2col64(x[b].astype(np.float64), k, s, p)
        db = d64[b].reshape(F, -1)
        dW += db @ col.T
        dX[b] = col2im64(W64.T @ db, C, H, H, k, s, p)
    tol = 1e-5
    assert np.allclose(bu, bu0 + d64.sum(axis=(0, 2, 3)), rtol=tol, atol=tol)
    assert np.allclose(wu.reshape(F, -1), wu0.reshape(F, -1) + dW, rtol=tol, atol=tol)
    assert np.allclose(sd, sd0 + dX, rtol=tol, atol=tol)


def test_conv_backward_rejects_dilation(ora):
    import ctypes
    x = np.zeros((1, 1, 5, 5), np.float32)
    z = np.zeros(100, np.float32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = ora.lib().ora_conv_backward(1, 1, 5, 5, p(x), p(z), 1, 3, 1, 2, 2, 9, p(z), p(z), p(z),
                                     p(z), p(z), None)
    assert rc == -1


def _bn_case(seed, batch=3, C=4, H=9, F=6, k=3, s=1, p=1):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.3, 0.3, F * C * k * k).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, F).astype(np.float32)
    b = rng.uniform(-0.2, 0.2, F).astype(np.float32)
    return x, w, sc, b


def test_oracle_conv_forward_train_batchnorm():
    """Restated TConvolutionalLayer.forward + TBaseLayer.batchNorm (training):
    x is the raw convolution, the statistics are its per-filter mean and
    unbiased variance, x_norm / out follow in float64 within 1e-5, and the
    rolling statistics take one multiply + one FMA step with momentum 0.1."""
    from oracle import oracle as ora
    x, w, sc, b = _bn_case(1)
    F = sc.size
    rm0 = np.full(F, 0.5, np.float32)
    rv0 = np.full(F, 2.0, np.float32)
    rm, rv = rm0.copy(), rv0.copy()
    out, m, v, xs, xn = ora.conv_forward_train(x, w, F, 3, 1, 1, 4, sc, b, rm, rv, 0.1, True)
    raw = ora.conv2d(x, w, F, 3, 1, 1)
    assert np.array_equal(xs, raw)
    r64 = raw.astype(np.float64).transpose(1, 0, 2, 3).reshape(F, -1)
    assert np.allclose(m, r64.mean(1), rtol=1e-5, atol=1e-6)
    assert np.allclose(v, r64.var(1, ddof=1), rtol=1e-5)
    sd = np.maximum(np.sqrt(v.astype(np.float64)), 1e-6)
    xn64 = (raw - m[None, :, None, None]) / sd[None, :, None, None]
    assert np.allclose(xn, xn64, rtol=1e-5, atol=1e-5)
    assert np.allclose(out, xn64 * sc[None, :, None, None] + b[None, :, None, None], atol=1e-5)
    keep = np.float32(1) - np.float32(0.1)
    assert np.array_equal(rm, np.float32(np.float32(0.1) * m.astype(np.float64)
                                         + (rm0 * keep).astype(np.float64)).astype(np.float32))
    # inference: rolling statistics, no stats written
    rm2, rv2 = rm.copy(), rv.copy()
    out2, *_ = ora.conv_forward_train(x, w, F, 3, 1, 1, 4, sc, b, rm2, rv2, 0.1, False)
    assert np.array_equal(rm2, rm) and np.array_equal(rv2, rv)
    sd2 = np.maximum(np.sqrt(rv.astype(np.float64)), 1e-6)
    ref2 = (raw - rm[None, :, None, None]) / sd2[None, :, None, None] * sc[None, :, None, None] \
        + b[None, :, None, None]
    assert np.allclose(out2, ref2, atol=1e-5)


def test_oracle_conv_backward_batchnorm_float64():
    """Restated batchNormBack (+ conv gradients) against the float64 closed
    form of the same formulas (ntensors.pas:8831-8951): within 1e-4."""
    from oracle import oracle as ora
    x, w, sc, b = _bn_case(2)
    F = sc.size
    rm, rv = np.zeros(F, np.float32), np.ones(F, np.float32)
    out, m, v, xs, xn = ora.conv_forward_train(x, w, F, 3, 1, 1, 4, sc, b, rm, rv, 0.1, True)
    rng = np.random.default_rng(3)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    su0 = rng.uniform(-1, 1, F).astype(np.float32)
    wu0 = np.zeros(w.size, np.float32)
    delta, su, wu = d0.copy(), su0.copy(), wu0.copy()
    md, vd = ora.conv_backward_bn(x, w, F, 3, 1, 1, 4, out, delta, sc, xs, xn, m, v, su, wu)
    D = d0.astype(np.float64)
    ax = (0, 2, 3)
    assert np.allclose(su, su0 + (xn * D).sum(ax), rtol=1e-4, atol=1e-4)
    Ds = D * sc[None, :, None, None]
    ve = np.maximum(v.astype(np.float64), 1e-6)
    c = xs.astype(np.float64) - m[None, :, None, None]
    md64 = Ds.sum(ax) * (-1 / np.sqrt(ve))
    vd64 = (Ds * c).sum(ax) * -0.5 * ve ** -1.5
    assert np.allclose(md, md64, rtol=1e-4, atol=1e-5)
    assert np.allclose(vd, vd64, rtol=1e-4, atol=1e-5)
    Bn = out.size // F
    d64 = Ds / np.sqrt(ve)[None, :, None, None] + c * (2 * vd64 / Bn)[None, :, None, None] \
        + (md64 / Bn)[None, :, None, None]
    assert np.allclose(delta, d64, rtol=1e-4, atol=1e-5)


def test_oracle_conv_backward_dilation_same_padding():
    """The backward im2col / col2im pad with padding*dilation
    (nConvolutionLayer.pas:640, 665): with the 'same' padding k=3, p=1 the
    columns match the layer's outH at dilation 2; other paddings are refused."""
    from oracle import oracle as ora
    lib = ora.lib()
    assert lib.ora_conv_backward_oh(13, 3, 1, 1, 2) == 13
    assert lib.ora_conv_backward_oh(13, 3, 2, 1, 3) == 7
    assert lib.ora_conv_backward_oh(13, 3, 1, 2, 2) == 0
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, (2, 3, 11, 11)).astype(np.float32)
    w = rng.uniform(-0.3, 0.3, 4 * 27).astype(np.float32)
    out = rng.uniform(-1, 1, (2, 4, 11, 11)).astype(np.float32)
    d = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu, wu, sd = np.zeros(4, np.float32), np.zeros(108, np.float32), np.zeros(x.shape, np.float32)
    ora.conv_backward(x, w, 4, 3, 1, 1, 9, out, d, bu, wu, sd, dil=2)
    # dW in float64: col built with pad 2, dilation 2
    xp = np.pad(x.astype(np.float64), ((0, 0), (0, 0), (2, 2), (2, 2)))
    col = np.stack([xp[:, :, 2 * kr:2 * kr + 11, 2 * kc:2 * kc + 11]
                    for kr in range(3) for kc in range(3)], 2).reshape(2, 27, 121)
    dW = np.einsum("bfp,bkp->fk", d.reshape(2, 4, 121).astype(np.float64), col)
    assert np.allclose(wu.reshape(4, 27), dW, rtol=1e-4, atol=1e-4)
