"""Batch-norm, softmax / cross-entropy device ops and the fused connected-
network train step (BASELINE config 5) vs the oracle.

Bar: bit-exact.  Sums follow the reference's orders (sequential strided
sums, vssum_avx2 / srss / sdot_avx2 lanes for contiguous blocks); exp / ln /
pow are evaluated in double and rounded once on both sides; the whole train
step's parameters after 1 and 5 steps and its cost match the oracle bit for
bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def dev(torch, x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


@pytest.mark.parametrize("groups,N,bs", [(32, 64, 1), (32, 10, 1), (4, 8, 9), (2, 3, 2704),
                                         (8, 16, 2704), (3, 4, 1029), (1100, 2, 9),
                                         (8, 4, 173056), (8, 5, 169), (6, 3, 64),
                                         (2, 3, 20011), (1, 3, 16392)])
def test_means_vars_normalize_scale(hip, torch_cuda, ora, groups, N, bs):
    x = ora.uniform(groups * N * bs, 21, N, -2.0, 3.0)
    m, v = ora.means_and_vars(x, groups, N, bs)
    dx = dev(torch_cuda, x)
    dm, dv = torch_cuda.zeros(N, device="cuda"), torch_cuda.zeros(N, device="cuda")
    hip.meansAndVars(x.size, N, groups, dx, 0, dm, dv)
    hip.finish()
    assert np.array_equal(dm.cpu().numpy(), m), "mean"
    assert np.array_equal(dv.cpu().numpy(), v), "var"
    y = ora.normalize(x.copy(), groups, N, bs, m, v)
    hip.normalize(N, x.size, groups, dev(torch_cuda, m), 1, dev(torch_cuda, v), 1, dx, 0)
    hip.finish()
    assert np.array_equal(dx.cpu().numpy(), y)
    s = ora.uniform(N, 22, N, 0.5, 1.5)
    b = ora.uniform(N, 23, N, -0.2, 0.2)
    y2 = ora.forward_scale(y.copy(), groups, N, bs, s)
    y2 = ora.add_bias(y2, b, N, bs, groups)
    hip.forwardScaleAdd(x.size, dx, 0, N, dev(torch_cuda, s), dev(torch_cuda, b), 1, groups)
    hip.finish()
    assert np.array_equal(dx.cpu().numpy(), y2)


@pytest.mark.parametrize("groups,N,bs", [(4, 8, 16), (8, 16, 2704), (3, 5, 24), (8, 2, 173056)])
def test_means_vars_srss_quirk(hip, torch_cuda, ora, groups, N, bs):
    """TNS_OPT_SRSS_QUIRK: blocks a multiple of 8 long lose lanes 4..7 of the
    variance sum, as the reference's srss does; off by default."""
    x = ora.uniform(groups * N * bs, 24, N, -2.0, 3.0)
    m0, v0 = ora.means_and_vars(x, groups, N, bs)
    m1, v1 = ora.means_and_vars(x, groups, N, bs, quirk=1)
    assert np.array_equal(m0, m1) and not np.array_equal(v0, v1)
    dx = dev(torch_cuda, x)
    for quirk, (m, v) in ((1, (m1, v1)), (0, (m0, v0))):
        hip.setSrssQuirk(bool(quirk))
        dm, dv = torch_cuda.zeros(N, device="cuda"), torch_cuda.zeros(N, device="cuda")
        try:
            hip.meansAndVars(x.size, N, groups, dx, 0, dm, dv)
            hip.finish()
        finally:
            hip.setSrssQuirk(False)
        assert np.array_equal(dm.cpu().numpy(), m) and np.array_equal(dv.cpu().numpy(), v)


BN_REPLAY = [(32, 64, 1), (32, 10, 1), (3, 5, 24), (2, 7, 65), (8, 32, 173056), (8, 64, 43264),
             (8, 256, 2704), (8, 1024, 169)]


@pytest.mark.parametrize("quirk", [0, 1])
@pytest.mark.parametrize("groups,N,bs", BN_REPLAY)
def test_batchnorm_gpu_call_sequence(hip, torch_cuda, ora, groups, N, bs, quirk):
    """The reference's BN forward on the GPU, call for call: batchNormGPU
    (nbaselayer.pas:583-643; blocks > 1, conv layers) and TConnectedLayer.
    forwardGPU (nconnectedlayer.pas:664-714; blockSize 1, forwardScaleAdd) —
    means, variances, scale/axpy rolling updates, copy to x, normalize, copy
    to x_norm, scale + bias — through TNNHip at state.step = 1 (element
    offset = outputStep), bit-exact against the CPU batchNorm restated
    (ora_batch_norm, nbaselayer.pas:336-370) in both srss lane modes."""
    T = torch_cuda
    n = groups * N * bs
    fc = bs == 1
    mom = np.float32(0.05 if fc else 0.1)
    y = ora.uniform(n, 61, N, -2.0, 3.0)
    sc = ora.uniform(N, 62, N, 0.5, 1.5)
    bi = ora.uniform(N, 63, N, -0.2, 0.2)
    rm = ora.uniform(N, 64, N, -0.5, 0.5)
    rv = ora.uniform(N, 65, N, 0.5, 1.5)
    ref, rm_ref, rv_ref = y.copy(), rm.copy(), rv.copy()
    m, v, xr, xnr = ora.batch_norm(ref, groups, N, bs, sc, bi, rm_ref, rv_ref, mom, True, quirk)

    off = n  # state.step = 1
    out = T.zeros(2 * n, device="cuda")
    out[off:] = dev(T, y)
    x, xn = T.zeros(2 * n, device="cuda"), T.zeros(2 * n, device="cuda")
    mean, var = T.zeros(N, device="cuda"), T.zeros(N, device="cuda")
    drm, drv, dsc, dbi = dev(T, rm), dev(T, rv), dev(T, sc), dev(T, bi)
    keep = float(np.float32(1) - mom)
    hip.setSrssQuirk(bool(quirk))
    try:
        hip.means(n, N, groups, out, off, mean)
        hip.variances(n, N, groups, out, off, mean, var)
        hip.scale(N, keep, drm, 1)
        hip.axpy(N, float(mom), mean, 0, 1, drm, 0, 1)
        hip.scale(N, keep, drv, 1)
        hip.axpy(N, float(mom), var, 0, 1, drv, 0, 1)
        hip.copy(n, out, off, 1, x, off, 1)
        hip.normalize(N, n, groups, mean, 1, var, 1, out, off)
        hip.copy(n, out, off, 1, xn, off, 1)
        if fc:
            hip.forwardScaleAdd(n, out, off, N, dsc, dbi, 1, groups)
        else:
            hip.forwardScale(n, out, off, N, dsc, 1, groups)
            hip.forwardBias(n, out, off, N, dbi, 1, groups)
        hip.finish()
    finally:
        hip.setSrssQuirk(False)
    assert np.array_equal(mean.cpu().numpy(), m), "mean"
    assert np.array_equal(var.cpu().numpy(), v), "variance"
    assert np.array_equal(drm.cpu().numpy(), rm_ref), "rolling_mean"
    assert np.array_equal(drv.cpu().numpy(), rv_ref), "rolling_variance"
    assert np.array_equal(x.cpu().numpy()[off:], xr), "x"
    assert np.array_equal(xn.cpu().numpy()[off:], xnr), "x_norm"
    assert np.array_equal(out.cpu().numpy()[off:], ref), "output"
    assert not out[:off].any(), "wrote outside the step's slice"


def test_variances_read_the_given_means(hip, torch_cuda, ora):
    """TNNCuda.variances takes the means as an input: the srss lanes run
    about whatever the caller passes (here the means of another tensor)."""
    T = torch_cuda
    groups, N, bs = 4, 6, 4099
    x = ora.uniform(groups * N * bs, 66, N, -2.0, 3.0)
    other = ora.uniform(groups * N * bs, 67, N, 0.0, 1.0)
    mu, _ = ora.means_and_vars(other, groups, N, bs)
    # oracle: MeansAndVars' variance pass with mu substituted (srss per block)
    v = np.zeros(N, np.float32)
    for i in range(N):
        acc = np.float32(0)
        for g in range(groups):
            blk = x[(g * N + i) * bs:(g * N + i + 1) * bs]
            acc = np.float32(acc + np.float32(ora.srss(mu[i], blk)))
        v[i] = np.float32(acc / np.float32(groups * bs - 1))
    dv = T.zeros(N, device="cuda")
    hip.variances(x.size, N, groups, dev(T, x), 0, dev(T, mu), dv)
    hip.finish()
    assert np.array_equal(dv.cpu().numpy(), v)


def test_init_hip_selects_the_reference_lane_drop(hiplib, torch_cuda, ora):
    """initHIP (pascal/nnHip.pas; Python twin tensorium_amd.nnhip.initHIP)
    selects TNS_OPT_SRSS_QUIRK = 1, so a Boundary-B caller gets the configured
    USE_AVX2 reference's variances on tail-less blocks without asking."""
    from tensorium_amd import nnhip
    T = torch_cuda
    groups, N, bs = 8, 4, 2704   # 52^2 blocks: a multiple of 8
    x = ora.uniform(groups * N * bs, 68, N, -2.0, 3.0)
    m1, v1 = ora.means_and_vars(x, groups, N, bs, quirk=1)
    h = nnhip.initHIP(0)
    try:
        dm, dv = T.zeros(N, device="cuda"), T.zeros(N, device="cuda")
        dx = dev(T, x)
        h.means(x.size, N, groups, dx, 0, dm)
        h.variances(x.size, N, groups, dx, 0, dm, dv)
        h.finish()
        assert np.array_equal(dm.cpu().numpy(), m1) and np.array_equal(dv.cpu().numpy(), v1)
    finally:
        h.setSrssQuirk(False)


BN_BWD = [(32, 64, 1), (4, 8, 9), (8, 16, 2704), (300, 3, 65), (2, 5, 1029), (3, 4, 16),
          (8, 4, 173056), (2, 3, 43264), (8, 6, 169), (5, 2, 64), (2, 3, 20011), (1, 3, 16392)]


@pytest.mark.parametrize("quirk", [0, 1])
@pytest.mark.parametrize("groups,N,bs", BN_BWD)
def test_bn_backward_ops(hip, torch_cuda, ora, groups, N, bs, quirk):
    """batchNormBack's reductions (addDots, sMeanAndVarianceDelta with the
    sVarinceDelta_avx lane order, sNormalizeDelta) bit-exact, with and
    without the reference's tail-less lane drop (TNS_OPT_SRSS_QUIRK)."""
    n = groups * N * bs
    x = ora.uniform(n, 31, N, -2.0, 2.0)
    m, v = ora.means_and_vars(x, groups, N, bs, quirk=quirk)
    xn = ora.normalize(x.copy(), groups, N, bs, m, v)
    delta = ora.uniform(n, 32, N)
    dsc = ora.uniform(N, 33, N)
    ref_dsc = ora.add_dots(dsc.copy(), xn, delta, groups, N, bs)
    md, vd = ora.mean_var_delta(delta, x, m, v, groups, N, bs, quirk=quirk)
    ref_delta = ora.normalize_delta(x, m, v, md, vd, delta.copy(), groups, N, bs)
    T = torch_cuda
    d_dsc = dev(T, dsc)
    dmd, dvd = T.zeros(N, device="cuda"), T.zeros(N, device="cuda")
    d_delta = dev(T, delta)
    hip.setSrssQuirk(bool(quirk))
    try:
        hip.addDots(n, N, groups, dev(T, xn), dev(T, delta), 0, d_dsc)
        hip.meansAndVarsDelta(n, N, groups, d_delta, dev(T, x), 0, dev(T, m), dev(T, v), dmd, dvd)
        hip.normalizeDelta(n, N, groups, d_delta, dev(T, x), 0, dev(T, m), dev(T, v), dmd, dvd)
        hip.finish()
    finally:
        hip.setSrssQuirk(False)
    assert np.array_equal(d_dsc.cpu().numpy(), ref_dsc), "addDots"
    assert np.array_equal(dmd.cpu().numpy(), md), "mean_delta"
    assert np.array_equal(dvd.cpu().numpy(), vd), "variance_delta"
    assert np.array_equal(d_delta.cpu().numpy(), ref_delta), "normalizeDelta"
    if bs % 8 == 0 and bs >= 8:  # the quirk must matter on tail-less blocks
        md2, vd2 = ora.mean_var_delta(delta, x, m, v, groups, N, bs, quirk=1 - quirk)
        assert not np.array_equal(vd, vd2)


@pytest.mark.parametrize("groups,N,bs", [(8, 4, 173056), (8, 16, 2704), (3, 5, 169), (2, 7, 65)])
def test_conv_block_bias_sums(hip, torch_cuda, ora, groups, N, bs):
    """addSums over conv blocks (backwardBias, bs >= 64: lane-chain path)."""
    src = ora.uniform(groups * N * bs, 53, 0)
    dst = ora.uniform(N, 54, 0)
    ref = ora.add_sums(dst.copy(), src, groups, N, bs)
    d = dev(torch_cuda, dst)
    hip.backwardBias(N, d, src.size, dev(torch_cuda, src), 0, 1, groups)
    hip.finish()
    assert np.array_equal(d.cpu().numpy(), ref)


def test_softmax_xent_sum(hip, torch_cuda, ora):
    B, C = 32, 10
    x = ora.uniform(B * C, 41, 0, -5.0, 5.0)
    p = ora.softmax_rows(x, C)
    T = torch_cuda
    dx, dp = dev(T, x), T.zeros(B * C, device="cuda")
    hip.softmaxBatch(C, dx, 0, B, C, 1, C, 1, 1.0, dp, 0)
    hip.finish()
    got = dp.cpu().numpy()
    assert np.array_equal(got, p), "softmax"
    t = np.zeros(B * C, np.float32)
    t[3::C] = 1.0
    d, e = ora.softmax_xent(p, t)
    dd, de = T.zeros(B * C, device="cuda"), T.zeros(B * C, device="cuda")
    hip.crossEntropySoftmax(B * C, dev(T, p), dev(T, t), dd, de)
    out = T.zeros(1, device="cuda")
    hip.sum(B * C, de, 0, out)
    hip.finish()
    assert np.array_equal(dd.cpu().numpy(), d)
    assert np.array_equal(de.cpu().numpy(), e), "xent"
    assert float(out.item()) == ora.vssum(e), "sum"


@pytest.mark.parametrize("O", [64, 1])
def test_backward_bias_fc_sequential(hip, torch_cuda, ora, O):
    B = 32
    src = ora.uniform(B * O, 51, 0)
    dst = ora.uniform(O, 52, 0)
    ref = ora.add_sums(dst.copy(), src, B, O, 1)
    d = dev(torch_cuda, dst)
    hip.backwardBias(O, d, src.size, dev(torch_cuda, src), 0, 1, B)
    hip.finish()
    assert np.array_equal(d.cpu().numpy(), ref)


MNIST = ([784, 64, 64, 64, 64, 32, 10], [1, 1, 1, 1, 1, 4])


def unpack(widths, bn, B, buf):
    from test_oracle_train import unpack as up
    return up(widths, bn, B, buf)


@pytest.mark.parametrize("bn", [0, 1])
@pytest.mark.parametrize("steps", [1, 5])
def test_fused_mlp_train_step(hip, torch_cuda, ora, bn, steps):
    widths, acts = MNIST
    B = 32
    buf = ora.mlp_init(widths, bn, B)
    X, T_ = ora.mnist_batch(B)
    T = torch_cuda
    dbuf, dX, dT = dev(T, buf), dev(T, X), dev(T, T_)
    dcost = T.zeros(1, device="cuda")
    costs = []
    for _ in range(steps):
        costs.append(ora.mlp_train_step(widths, acts, bn, B, X, T_, 1e-2, 0.9, 1e-4, buf))
        hip.mlpTrainStep(widths, acts, bn, B, dX, dT, 1e-2, 0.9, 1e-4, dbuf, dcost)
    hip.finish()
    got = dbuf.cpu().numpy()
    bad = []
    if float(dcost.item()) != np.float32(costs[-1]):
        bad.append(("cost", float(dcost.item()), costs[-1]))
    for l, (g, r) in enumerate(zip(unpack(widths, bn, B, got), unpack(widths, bn, B, buf))):
        for name in g:
            if not np.array_equal(g[name], r[name]):
                bad.append((l, name, int((g[name] != r[name]).sum())))
    assert not bad, bad


@pytest.mark.parametrize("widths,acts,B", [
    ([101, 37, 70, 24, 10], [9, 0, 6, 4], 20),   # odd widths: scalar staging, 3-tile fallback gemm
    ([64, 48, 33, 10], [1, 13, 4], 40),          # two batch tiles, hardtan
    ([784, 64, 10], [1, 4], 2),                  # smallest batch
    ([1200, 40, 10], [1, 4], 8),                 # layer 0 past 8 k-chunks: two chunks in flight
])
@pytest.mark.parametrize("bn", [0, 1])
def test_fused_mlp_irregular_shapes(hip, torch_cuda, ora, widths, acts, B, bn):
    """The fused step at shapes off the MNIST net: every buffer element and
    the cost bit-identical to the oracle after 3 steps."""
    buf = ora.mlp_init(widths, bn, B, seed=11)
    X, T_ = ora.mnist_batch(B, seed=11, classes=widths[-1], inputs=widths[0])
    T = torch_cuda
    dbuf, dX, dT = dev(T, buf), dev(T, X), dev(T, T_)
    dcost = T.zeros(1, device="cuda")
    for _ in range(3):
        cost = ora.mlp_train_step(widths, acts, bn, B, X, T_, 1e-2, 0.9, 1e-4, buf)
        hip.mlpTrainStep(widths, acts, bn, B, dX, dT, 1e-2, 0.9, 1e-4, dbuf, dcost)
    hip.finish()
    got = dbuf.cpu().numpy()
    assert float(dcost.item()) == np.float32(cost)
    diff = np.flatnonzero(got != buf)
    assert diff.size == 0, (diff.size, diff[:10])


def test_fused_mlp_no_bn_is_bit_exact_one_step(hip, torch_cuda, ora):
    """Without BN the only transcendental is softmax's exp (in double on both
    sides), so one step should reproduce the oracle exactly."""
    widths, acts = MNIST
    B = 32
    buf = ora.mlp_init(widths, 0, B)
    X, T_ = ora.mnist_batch(B)
    T = torch_cuda
    dbuf = dev(T, buf)
    dcost = T.zeros(1, device="cuda")
    ora.mlp_train_step(widths, acts, 0, B, X, T_, 1e-2, 0.9, 1e-4, buf)
    hip.mlpTrainStep(widths, acts, 0, B, dev(T, X), dev(T, T_), 1e-2, 0.9, 1e-4, dbuf, dcost)
    hip.finish()
    got = dbuf.cpu().numpy()
    frac = float(np.mean(got == buf))
    assert frac == 1.0, f"{(1 - frac) * 100:.4f}% of buffer elements differ"


@pytest.mark.parametrize("nw,n,bn,offset", [(784 * 64, 64, True, 0), (4096 * 4097, 4097, False, 0),
                                            (1001, 7, True, 1), (0, 5, False, 0)])
def test_sgd_update_fused(hip, torch_cuda, ora, nw, n, bn, offset):
    """TConnectedLayer.update (nconnectedlayer.pas:324-359) fused into one
    pass: bit-exact against the restated axpy/scale sequence (float4 and
    scalar paths, with and without batch-norm scales)."""
    rng = np.random.default_rng(nw + n)
    mk = lambda k: rng.uniform(-1, 1, k + offset).astype(np.float32)  # noqa: E731
    W, dW, b, db = mk(nw), mk(nw), mk(n), mk(n)
    sc, dsc = (mk(n), mk(n)) if bn else (None, None)
    lr, batch, decay, mom = 1e-3, 32, 1e-4, 0.9
    lrb = np.float32(np.float32(lr) / np.float32(batch))
    ndb = np.float32(-np.float32(decay) * np.float32(batch))
    t = lambda a: None if a is None else torch_cuda.from_numpy(a.copy()).cuda()[offset:]  # noqa
    g = [t(a) for a in (W, dW, b, db, sc, dsc)]
    ref = [None if a is None else a[offset:].copy() for a in (W, dW, b, db, sc, dsc)]
    ora.sgd_update(*ref, float(lrb), float(ndb), mom)
    hip.sgdUpdate(g[0], g[1], g[2], g[3], lr, batch, decay, mom, g[4], g[5])
    hip.finish()
    for x, r in zip(g, ref):
        if r is not None:
            assert np.array_equal(x.cpu().numpy(), r)


def test_bn_null_pointers_are_arg_errors(hip, torch_cuda):
    """A null pointer from the binding is TNS_ERR_ARG (1), not a GPU fault."""
    L, T = hip.lib, torch_cuda
    x = T.zeros(64, device="cuda")
    p = x.data_ptr()
    assert L.tns_hip_means_and_vars_delta(hip.ctx, 64, 4, 2, None, p, 0, p, p, p, p) == 1
    assert L.tns_hip_normalize_delta(hip.ctx, 64, 4, 2, p, None, 0, p, p, p, p) == 1
    assert L.tns_hip_add_dots(hip.ctx, 64, 4, 2, p, None, 0, p) == 1
    assert L.tns_hip_means_and_vars(hip.ctx, 64, 4, 2, None, 0, p, p) == 1
    assert L.tns_hip_means(hip.ctx, 64, 4, 2, p, 0, None) == 1
    assert L.tns_hip_variances(hip.ctx, 64, 4, 2, p, 0, None, p) == 1
    assert L.tns_hip_variances(hip.ctx, 63, 4, 2, p, 0, p, p) == 1   # sizes do not align
    hip.finish()
