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
