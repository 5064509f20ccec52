"""Bias / activation / BLAS-1 kernels vs the oracle.
Bar: bit-exact for every supported activation.  logistic / tanh follow the
scalar Pascal forms with exp's real result rounded where the Pascal stores it
(tanh: two single exps, NaN once exp overflows); the device and the oracle
share that form, so only a last-ulp difference between the two libms' double
exp could separate them (not seen)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EXACT = [1, 4, 8, 9, 13]
TRANSC = [0, 6]


@pytest.mark.parametrize("act", EXACT + TRANSC)
@pytest.mark.parametrize("n", [1, 7, 1024, 100003])
def test_activate(hip, torch_cuda, ora, act, n):
    x = ora.uniform(n, 8, act, -6.0, 6.0)
    if n > 100:  # overflow / underflow / signed zero edges
        x[:8] = np.array([-100, 100, 0.0, -0.0, 88.8, -88.8, 1e-8, -1e-30], np.float32)
    ref = ora.activate(x.copy(), act)
    dx = torch_cuda.from_numpy(x).cuda()
    hip.ActivateArray(n, dx, 0, act)
    hip.finish()
    got = dx.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)) or \
        np.array_equal(got, ref, equal_nan=True), (act, np.abs(got - ref).max())


@pytest.mark.parametrize("n", [5001, 5004])  # scalar and float4 forms
@pytest.mark.parametrize("act", EXACT + TRANSC)
def test_derive(hip, torch_cuda, ora, act, n):
    y = ora.activate(ora.uniform(n, 9, act, -3.0, 3.0), act)
    delta = ora.uniform(n, 10, act)
    ref = ora.gradient(y, act, delta.copy())
    dy, dd = torch_cuda.from_numpy(y).cuda(), torch_cuda.from_numpy(delta.copy()).cuda()
    hip.DeriveArray(n, dy, 0, act, dd)
    hip.finish()
    assert np.array_equal(dd.cpu().numpy(), ref)


@pytest.mark.parametrize("F,bs,batch", [(3, 5, 2), (64, 2704, 2), (255, 169, 1), (10, 1, 32),
                                        (32, 173056, 1)])
def test_forward_bias(hip, torch_cuda, ora, F, bs, batch):
    x = ora.uniform(batch * F * bs, 11, F)
    b = ora.uniform(F, 12, F, -0.1, 0.1)
    ref = ora.add_bias(x.copy(), b, F, bs, batch)
    dx, db = torch_cuda.from_numpy(x).cuda(), torch_cuda.from_numpy(b).cuda()
    hip.forwardBias(x.size, dx, 0, F, db, 1, batch)
    hip.finish()
    assert np.array_equal(dx.cpu().numpy(), ref)


@pytest.mark.parametrize("F,bs,batch", [(16, 333, 4), (3, 8, 2), (5, 7, 3), (1, 1000, 40),
                                         (4, 64, 1100), (2, 43264, 8), (3, 2053, 11),
                                         (2, 4096, 3)])
def test_backward_bias_addsums_order(hip, torch_cuda, ora, F, bs, batch):
    """addSums (ntensors.pas:7729-7781): vssum_avx2 per contiguous block,
    blocks summed in order — bit-exact; also more groups than one LDS chunk."""
    src = ora.uniform(batch * F * bs, 13, 0)
    dst = ora.uniform(F, 14, 0)
    ref = ora.add_sums(dst.copy(), src, batch, F, bs)
    dsrc, ddst = torch_cuda.from_numpy(src).cuda(), torch_cuda.from_numpy(dst.copy()).cuda()
    hip.backwardBias(F, ddst, src.size, dsrc, 0, 1, batch)
    hip.finish()
    assert np.array_equal(ddst.cpu().numpy(), ref)
    scale = np.abs(src.reshape(batch, F, bs)).sum(axis=(0, 2)) + np.abs(dst)
    f64 = dst.astype(np.float64) + src.reshape(batch, F, bs).astype(np.float64).sum(axis=(0, 2))
    assert np.all(np.abs(ref - f64) <= 1e-5 * scale)


def test_blas1(hip, torch_cuda, ora):
    n = 10007
    x = ora.uniform(n, 15, 0)
    y = ora.uniform(n, 16, 0)
    dx, dy = torch_cuda.from_numpy(x).cuda(), torch_cuda.from_numpy(y.copy()).cuda()
    hip.axpy(n, 0.37, dx, 0, 1, dy, 0, 1)
    hip.finish()
    ref = y.copy()
    ora.lib().ora_saxpy(n, 0.37, x.ctypes.data, ref.ctypes.data)
    assert np.array_equal(dy.cpu().numpy(), ref)
    hip.scale(n, 2.5, dy, 1)
    hip.finish()
    assert np.array_equal(dy.cpu().numpy(), (ref * np.float32(2.5)).astype(np.float32))
    hip.fill(n, dy, 0, 3.0, 1)
    hip.clamp(n, 1.0, dx, dx, 1, 0)
    hip.copy(n // 2, dx, 0, 2, dy, 0, 1)
    hip.finish()
    got = dy.cpu().numpy()
    assert np.array_equal(got[: n // 2], np.clip(x, -1, 1)[0:2 * (n // 2):2])
    assert np.all(got[n // 2:] == 3.0)


def test_tnncuda_vector_ops(hip, torch_cuda):
    """TNNCuda addvv / subvv / mulvv / fmavv / fmavss / inverseSqrt
    (nncuda.pas:120-151): strided, offsets in elements, one rounding per
    arithmetic operation (numpy float32 arithmetic is the same IEEE op)."""
    T = torch_cuda
    rng = np.random.default_rng(9)
    n = 1000
    a = rng.uniform(-2, 2, 3 * n + 5).astype(np.float32)
    b = rng.uniform(-2, 2, 2 * n + 3).astype(np.float32)
    c = rng.uniform(-2, 2, n + 7).astype(np.float32)
    da, db, dc = (T.from_numpy(x).cuda() for x in (a, b, c))
    A, B, Cc = a[5::3][:n], b[3::2][:n], c[7:][:n]
    for name, ref in (("addvv", A + B), ("subvv", A - B), ("mulvv", A * B)):
        out = T.zeros(2 * n + 1, device="cuda")
        getattr(hip, name)(n, da, 5, 3, db, 3, 2, out, 1, 2)
        hip.finish()
        assert np.array_equal(out.cpu().numpy()[1::2][:n], ref.astype(np.float32)), name
    out = T.zeros(n, device="cuda")
    hip.fmavv(n, da, 5, 3, db, 3, 2, dc, 7, 1, out, 0, 1)
    hip.finish()
    assert np.array_equal(out.cpu().numpy(), ((A * B).astype(np.float32) + Cc).astype(np.float32))
    out = T.zeros(c.size, device="cuda")
    hip.fmavss(n, dc, 7, 1.5, -0.25, out)
    hip.finish()
    ref = ((Cc * np.float32(1.5)).astype(np.float32) + np.float32(-0.25)).astype(np.float32)
    assert np.array_equal(out.cpu().numpy()[7:7 + n], ref)
    v = np.abs(rng.uniform(-1e-5, 4, 2 * n)).astype(np.float32)
    v[::50] = 0.0
    dv, out = T.from_numpy(v).cuda(), T.zeros(2 * n, device="cuda")
    hip.inverseSqrt(n, 0.0, dv, out, 2, 1)
    hip.finish()
    ref = (np.float32(1) / np.sqrt(np.maximum(v[1::2], np.float32(1e-6)))).astype(np.float32)
    assert np.array_equal(out.cpu().numpy()[1::2], ref)
