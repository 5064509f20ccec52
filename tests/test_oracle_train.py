"""CPU checks of the oracle's batch-norm / softmax / train-step restatement
(oracle/tns_oracle_train.c) against an independent float64 numpy statement of
the same reference formulas (ntensors.pas:8821-8951, 9102-9177;
nconnectedlayer.pas:157-359; nsoftmaxlayer.pas:83-137)."""
import numpy as np
import pytest

EPS = 1e-6


def test_means_vars_normalize(ora):
    rng = np.random.default_rng(0)
    for groups, N, bs in [(32, 64, 1), (4, 8, 9), (2, 3, 52 * 52)]:
        x = rng.normal(0.3, 2.0, groups * N * bs).astype(np.float32)
        m, v = ora.means_and_vars(x, groups, N, bs)
        x3 = x.reshape(groups, N, bs).astype(np.float64)
        m64 = x3.mean(axis=(0, 2))
        v64 = x3.var(axis=(0, 2), ddof=1)
        assert np.allclose(m, m64, rtol=1e-5, atol=1e-5)
        assert np.allclose(v, v64, rtol=1e-4)
        y = ora.normalize(x.copy(), groups, N, bs, m, v)
        if bs == 1:
            ref = (x3 - m[None, :, None]) / np.sqrt(np.maximum(v, EPS))[None, :, None]
        else:
            ref = (x3 - m[None, :, None]) / np.maximum(np.sqrt(v), EPS)[None, :, None]
        assert np.allclose(y.reshape(groups, N, bs), ref, rtol=1e-4, atol=1e-5)


def test_softmax_and_xent(ora):
    rng = np.random.default_rng(1)
    x = rng.normal(0, 3, 7 * 10).astype(np.float32)
    p = ora.softmax_rows(x, 10)
    e = np.exp(x.reshape(7, 10).astype(np.float64) - x.reshape(7, 10).max(axis=1, keepdims=True))
    ref = e / e.sum(axis=1, keepdims=True)
    assert np.allclose(p.reshape(7, 10), ref, rtol=1e-6, atol=1e-7)
    t = np.zeros(70, np.float32)
    t[::10] = 1.0
    d, err = ora.softmax_xent(p, t)
    assert np.array_equal(d, t - p)
    assert np.allclose(err[::10], -np.log(np.maximum(p[::10], EPS)), rtol=1e-6)
    assert np.all(err[1::10] == 0)


def test_vssum_order(ora):
    a = np.array([1e8, 1.0, -1e8, 1.0, 3.0, 1.0, 2.0, 1.0, 0.5], np.float32)
    # lanes: (1e8+3)+(1+1)+(-1e8+2)+(1+1), then + 0.5 sequentially
    s0, s1 = np.float32(1e8) + np.float32(3.0), np.float32(1.0) + np.float32(1.0)
    s2, s3 = np.float32(-1e8) + np.float32(2.0), np.float32(2.0)
    ref = np.float32(np.float32(np.float32(s0 + s1) + np.float32(s2 + s3)) + np.float32(0.5))
    assert np.float32(ora.vssum(a)) == ref


def mlp_step_f64(widths, acts, bn, B, X, T, buf, lr, mom, decay):
    """float64 numpy statement of one TNNet.Propagate + update (reference formulas)."""
    L = len(widths) - 1
    views = []
    off = 0

    def take(n):
        nonlocal off
        v = buf[off:off + n].astype(np.float64)
        off += n
        return v

    for l in range(L):
        I, O = widths[l], widths[l + 1]
        d = dict(W=take(I * O).reshape(O, I), b=take(O), dW=take(I * O).reshape(O, I), db=take(O))
        if bn:
            d.update(scales=take(O), rmean=take(O), rvar=take(O), dscales=take(O))
        take(2 * B * O)
        if bn:
            take(2 * B * O + 4 * O)
        views.append(d)
    x = X.reshape(B, widths[0]).astype(np.float64)
    ins, outs, xs, xns, stats = [], [], [], [], []
    for l, d in enumerate(views):
        ins.append(x)
        z = x @ d["W"].T
        if bn:
            m, v = z.mean(0), z.var(0, ddof=1)
            d["rmean"] = d["rmean"] * 0.95 + 0.05 * m
            d["rvar"] = d["rvar"] * 0.95 + 0.05 * v
            xn = (z - m) / np.sqrt(np.maximum(v, EPS))
            xs.append(z)
            xns.append(xn)
            stats.append((m, v))
            z = xn * d["scales"]
        z = z + d["b"]
        if acts[l] == 1:
            z = z * (z > 0)
        outs.append(z)
        x = z
    e = np.exp(x - x.max(1, keepdims=True))
    p = e / e.sum(1, keepdims=True)
    t = T.reshape(B, -1).astype(np.float64)
    cost = float(np.sum(np.where(t != 0, -np.log(np.maximum(p, EPS)), 0)))
    delta = t - p
    for l in range(L - 1, -1, -1):
        d = views[l]
        delta = np.clip(delta, -1, 1)
        if acts[l] == 1:
            delta = delta * (outs[l] > 0)
        d["db"] = d["db"] + delta.sum(0)
        if bn:
            m, v = stats[l]
            ve = np.maximum(v, EPS)
            d["dscales"] = d["dscales"] + (xns[l] * delta).sum(0)
            delta = delta * d["scales"]
            md = delta.sum(0) * (-1 / np.sqrt(ve))
            vd = (delta * (xs[l] - m)).sum(0) * -0.5 * ve ** -1.5
            delta = delta / np.sqrt(ve) + (xs[l] - m) * (2 * vd / B) + md / B
        d["dW"] = d["dW"] + delta.T @ ins[l]
        delta = delta @ d["W"]
    for d in views:
        d["b"] = d["b"] + lr / B * d["db"]
        d["db"] = d["db"] * mom
        if bn:
            d["scales"] = d["scales"] + lr / B * d["dscales"]
            d["dscales"] = d["dscales"] * mom
        d["dW"] = d["dW"] - decay * B * d["W"]
        d["W"] = d["W"] + lr / B * d["dW"]
        d["dW"] = d["dW"] * mom
    return cost, views


def unpack(widths, bn, B, buf):
    views = []
    off = 0
    for l in range(len(widths) - 1):
        I, O = widths[l], widths[l + 1]
        d = {}
        for name, n in [("W", I * O), ("b", O), ("dW", I * O), ("db", O)]:
            d[name] = buf[off:off + n]
            off += n
        if bn:
            for name in ("scales", "rmean", "rvar", "dscales"):
                d[name] = buf[off:off + O]
                off += O
        off += 2 * B * O
        if bn:
            off += 2 * B * O + 4 * O
        views.append(d)
    return views


@pytest.mark.parametrize("bn", [0, 1])
def test_mlp_train_step_matches_float64(ora, bn):
    widths = [784, 64, 64, 64, 64, 32, 10]
    acts = [1, 1, 1, 1, 1, 4]
    B = 32
    buf = ora.mlp_init(widths, bn, B)
    X, T = ora.mnist_batch(B)
    buf0 = buf.copy()
    cost = ora.mlp_train_step(widths, acts, bn, B, X, T, 1e-2, 0.9, 1e-4, buf)
    cost64, ref = mlp_step_f64(widths, acts, bn, B, X, T, buf0, 1e-2, 0.9, 1e-4)
    assert abs(cost - cost64) <= 1e-4 * abs(cost64)
    got = unpack(widths, bn, B, buf)
    for l, (g, r) in enumerate(zip(got, ref)):
        for name in g:
            a, b = g[name].astype(np.float64), r[name].reshape(-1)
            scale = np.abs(b).max() + 1e-12
            assert np.max(np.abs(a - b)) <= 1e-4 * scale, (l, name, np.max(np.abs(a - b)) / scale)
