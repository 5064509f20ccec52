"""Pin the C oracle (oracle/tns_oracle.c) against the hand-derived
known-answer vectors of tests/golden/golden.npz (exact-rational transcription
of the Pascal operation order, see tests/golden/make_golden.py).

The reference itself holds no golden vectors or tests, so
this pinning is against an independent restatement, not a reference run:
parity is reported as "unpinned by reference artefacts" in DESIGN.md.
"""
import numpy as np
import pytest


def eq(a, b):
    return np.array_equal(np.asarray(a, np.float32), np.asarray(b, np.float32), equal_nan=True)


@pytest.mark.parametrize("n", [13, 8, 5, 37])
def test_sdot_lane_order(ora, golden, n):
    a, b = golden[f"sdot_{n}_a"], golden[f"sdot_{n}_b"]
    got = np.float32(ora.sdot(a, b))
    assert got == golden[f"sdot_{n}_out"][0]


def test_sdot_order_is_not_sequential(ora, golden):
    # the 8-lane fold must differ from a naive running sum for at least one case
    diffs = 0
    for n in (13, 37):
        a, b = golden[f"sdot_{n}_a"], golden[f"sdot_{n}_b"]
        s = np.float32(0)
        for x, y in zip(a, b):
            s = np.float32(s + np.float32(x * y))
        diffs += int(s != golden[f"sdot_{n}_out"][0])
    assert diffs >= 1


GEMM = ["nn_a1b0", "nn_a05b2", "nn_a1b1", "nt_a1b0", "nt_a05b2", "tn_a1b0", "tn_a2b05",
        "tt_a1b0", "tt_a05b1"]


@pytest.mark.parametrize("name", GEMM)
@pytest.mark.parametrize("threads", [1, 3])
def test_gemm_golden(ora, golden, name, threads):
    ta, tb, M, N, K, lda, ldb = (int(v) for v in golden[f"gemm_{name}_dims"])
    al, be = (float(v) for v in golden[f"gemm_{name}_ab"])
    A, B = golden[f"gemm_{name}_A"].copy(), golden[f"gemm_{name}_B"].copy()
    C = golden[f"gemm_{name}_C"].copy()
    ora.set_threads(threads)
    try:
        ora.sgemm(bool(ta), bool(tb), M, N, K, al, A, lda, B, ldb, be, C, N)
    finally:
        ora.set_threads(0)
    assert eq(C, golden[f"gemm_{name}_out"]), name


def test_beta0_is_zero_times_c(ora, golden):
    A, B, C = golden["beta0nan_A"].copy(), golden["beta0nan_B"].copy(), golden["beta0nan_C"].copy()
    ora.sgemm(False, False, 2, 2, 3, 1.0, A, 3, B, 2, 0.0, C, 2)
    assert eq(C, golden["beta0nan_out"])
    assert np.isnan(C[0]) and np.isnan(C[2]) and np.isfinite(C[1]) and np.isfinite(C[3])


@pytest.mark.parametrize("gi", range(5))
def test_im2col_golden(ora, golden, gi):
    C, H, W, k, p, s, d = (int(v) for v in golden[f"i2c_{gi}_geo"])
    col = ora.im2col(C, H, W, k, k, p, p, s, s, d, d, golden[f"i2c_{gi}_im"].copy())
    assert col.tobytes() == golden[f"i2c_{gi}_col"].tobytes()  # bit-exact


@pytest.mark.parametrize("gi", range(5))
def test_col2im_golden(ora, golden, gi):
    C, H, W, k, p, s, d = (int(v) for v in golden[f"i2c_{gi}_geo"])
    im = golden[f"c2i_{gi}_base"].copy()
    ora.col2im(C, H, W, k, k, p, p, s, s, d, d, golden[f"c2i_{gi}_colin"].copy(), im)
    assert eq(im, golden[f"c2i_{gi}_out"])


def test_bias_and_activations(ora, golden):
    x = golden["bias_x"].copy()
    ora.add_bias(x, golden["bias_b"].copy(), 3, 5, 2)
    assert eq(x, golden["bias_out"])
    y = x.copy()
    ora.activate(y, 9)
    assert eq(y, golden["leaky_out"])
    y = x.copy()
    ora.activate(y, 1)
    assert eq(y, golden["relu_out"])


BN_N = [5, 8, 13, 16, 37, 64, 67]


@pytest.mark.parametrize("n", BN_N)
@pytest.mark.parametrize("quirk", [0, 1])
def test_bn_block_reductions_golden(ora, golden, n, quirk):
    """vssum_avx2 / srss / sVarinceDelta_avx over one block, in the
    reference's lane order, with and without the tail-less lane drop."""
    a, d, mu = golden[f"bn_{n}_a"], golden[f"bn_{n}_d"], float(golden[f"bn_{n}_mu"][0])
    assert np.float32(ora.vssum(a)) == golden[f"bn_{n}_vssum"][0]
    assert np.float32(ora.srss(mu, a, quirk)) == golden[f"bn_{n}_srss_q{quirk}"][0]
    assert np.float32(ora.var_delta_avx(mu, d, a, quirk)) == golden[f"bn_{n}_vdelta_q{quirk}"][0]


def test_var_delta_lane_order_matters(ora, golden):
    """The 8-lane order is not a sequential chain on at least one block, and
    the quirk changes tail-less blocks only."""
    diffs = 0
    for n in BN_N:
        a, d, mu = golden[f"bn_{n}_a"], golden[f"bn_{n}_d"], np.float32(golden[f"bn_{n}_mu"][0])
        s = np.float32(0)
        for x, y in zip(a, d):
            s = np.float32(s + np.float32(np.float32(x - mu) * y))
        diffs += int(s != golden[f"bn_{n}_vdelta_q0"][0])
        q0, q1 = golden[f"bn_{n}_vdelta_q0"][0], golden[f"bn_{n}_vdelta_q1"][0]
        if n % 8:
            assert q0 == q1
    assert diffs >= 1
    assert golden["bn_64_vdelta_q0"][0] != golden["bn_64_vdelta_q1"][0]


@pytest.mark.parametrize("gi", range(3))
@pytest.mark.parametrize("quirk", [0, 1])
def test_bn_channel_statistics_golden(ora, golden, gi, quirk):
    """MeansAndVars and sMeanAndVarianceDelta over [groups][N][bs] tensors:
    block sums added in group order; mean_delta / variance_delta are the
    golden sums scaled as ntensors.pas:8869-8870 (Power in double)."""
    groups, N, bs = (int(v) for v in golden[f"bnc_{gi}_dims"])
    x, d = golden[f"bnc_{gi}_x"], golden[f"bnc_{gi}_d"]
    m, v = ora.means_and_vars(x, groups, N, bs, quirk=quirk)
    assert eq(m, golden[f"bnc_{gi}_mean_q{quirk}"]) and eq(v, golden[f"bnc_{gi}_var_q{quirk}"])
    md, vd = ora.mean_var_delta(d, x, m, v, groups, N, bs, quirk=quirk)
    ve = np.maximum(v, np.float32(1e-6)).astype(np.float32)
    inv = (np.float32(-1.0) / np.sqrt(ve)).astype(np.float32)
    assert eq(md, (golden[f"bnc_{gi}_msum_q{quirk}"] * inv).astype(np.float32))
    vref = (golden[f"bnc_{gi}_vsum_q{quirk}"].astype(np.float64) * -0.5
            * np.power(ve.astype(np.float64), -1.5)).astype(np.float32)
    assert eq(vd, vref)


# ---- round 3: the rest of SURVEY §8(c)'s fixture list ----------------------

@pytest.mark.parametrize("gi", range(4))
def test_bn_elementwise_golden(ora, golden, gi):
    """blockNormalize in both epsilon forms (_snormvv at blockSize 1,
    _snormblkvv otherwise), forwardScale, sMeanAndVarianceDelta with its
    final scaling, sNormalizeDelta_avx, addDots and addSums."""
    groups, N, bs = (int(v) for v in golden[f"bnn_{gi}_dims"])
    x, d, s = golden[f"bnn_{gi}_x"], golden[f"bnn_{gi}_d"], golden[f"bnn_{gi}_s"]
    m, v = golden[f"bnn_{gi}_mean"].copy(), golden[f"bnn_{gi}_var"].copy()
    assert eq(ora.normalize(x.copy(), groups, N, bs, m, v), golden[f"bnn_{gi}_norm"])
    assert eq(ora.forward_scale(x.copy(), groups, N, bs, s.copy()), golden[f"bnn_{gi}_scaled"])
    md, vd = ora.mean_var_delta(d.copy(), x.copy(), m, v, groups, N, bs)
    assert eq(md, golden[f"bnn_{gi}_md"]) and eq(vd, golden[f"bnn_{gi}_vd"])
    nd = ora.normalize_delta(x.copy(), m, v, md, vd, d.copy(), groups, N, bs)
    assert eq(nd, golden[f"bnn_{gi}_ndelta"])
    acc = golden[f"bnn_{gi}_acc"]
    assert eq(ora.add_dots(acc.copy(), x.copy(), d.copy(), groups, N, bs),
              golden[f"bnn_{gi}_dots"])
    assert eq(ora.add_sums(acc.copy(), d.copy(), groups, N, bs), golden[f"bnn_{gi}_sums"])


def test_bn_eps_forms_differ(golden):
    """The two epsilon placements give different results on the channel whose
    variance is under eps (bnn_0, blockSize 1: sqrt(max(v, eps)))."""
    x, m, v = golden["bnn_0_x"], golden["bnn_0_mean"], golden["bnn_0_var"]
    assert v[1] < np.float32(1e-6)
    other = (x[1] - m[1]) / np.maximum(np.sqrt(v[1]), np.float32(1e-6))
    assert np.float32(other) != golden["bnn_0_norm"][1]


def test_transcendental_activations_golden(ora, golden):
    x = golden["act_x"]
    assert eq(ora.activate(x.copy(), 0), golden["act_logistic"])
    t = ora.activate(x.copy(), 6)
    assert eq(t, golden["act_tanh"])
    assert np.isnan(golden["act_tanh"]).any()       # exp overflow -> NaN, as the reference
    d = golden["grad_d"]
    y = golden["act_logistic"]
    assert eq(ora.gradient(y.copy(), 0, d.copy()), golden["grad_logistic"])
    assert eq(ora.gradient(golden["grad_tanh_y"].copy(), 6, d.copy()), golden["grad_tanh"])


@pytest.mark.parametrize("gi", range(2))
def test_softmax_xent_golden(ora, golden, gi):
    rows, n = (int(v) for v in golden[f"sm_{gi}_dims"])
    temp = float(golden[f"sm_{gi}_temp"][0])
    out = ora.softmax_rows(golden[f"sm_{gi}_x"].copy(), n, temp)
    assert eq(out, golden[f"sm_{gi}_out"])
    dl, err = ora.softmax_xent(out, golden[f"sm_{gi}_truth"].copy())
    assert eq(dl, golden[f"sm_{gi}_delta"]) and eq(err, golden[f"sm_{gi}_err"])
    assert np.float32(ora.vssum(err)) == golden[f"sm_{gi}_cost"][0]


@pytest.mark.parametrize("tag", ["bn", "nobn"])
def test_sgd_update_golden(ora, golden, tag):
    lr, mom, decay = (np.float32(v) for v in golden["sgd_hyper"])
    batch = int(golden["sgd_batch"][0])
    W, dW = golden["sgd_W"].copy(), golden["sgd_dW"].copy()
    b, db = golden["sgd_b"].copy(), golden["sgd_db"].copy()
    s = golden["sgd_s"].copy() if tag == "bn" else None
    ds = golden["sgd_ds"].copy() if tag == "bn" else None
    lrb = np.float32(lr / np.float32(batch))
    ndb = np.float32(-decay * np.float32(batch))
    ora.sgd_update(W, dW, b, db, s, ds, float(lrb), float(ndb), float(mom))
    assert eq(W, golden[f"sgd_{tag}_W_out"]) and eq(dW, golden[f"sgd_{tag}_dW_out"])
    assert eq(b, golden[f"sgd_{tag}_b_out"]) and eq(db, golden[f"sgd_{tag}_db_out"])
    if tag == "bn":
        assert eq(s, golden["sgd_bn_s_out"]) and eq(ds, golden["sgd_bn_ds_out"])


def test_mlp_bn_train_step_golden(ora, golden):
    """One whole connected-network train step with batch norm and softmax
    (config 5's structure at batch 32, reduced width): every array of the
    packed buffer after the step, and the cost, bit for bit."""
    widths = [int(v) for v in golden["mlp_widths"]]
    acts = [int(v) for v in golden["mlp_acts"]]
    B = int(golden["mlp_B"][0])
    lr, mom, decay = (float(v) for v in golden["mlp_hyper"])
    buf = golden["mlp_buf_in"].copy()
    assert buf.size == ora.mlp_buffer_floats(widths, True, B)
    cost = ora.mlp_train_step(widths, acts, True, B, golden["mlp_X"].copy(),
                              golden["mlp_T"].copy(), lr, mom, decay, buf)
    exp = golden["mlp_buf_out"]
    bad = np.flatnonzero(~((buf == exp) | (np.isnan(buf) & np.isnan(exp))))
    assert bad.size == 0, f"{bad.size} buffer floats differ, first at {bad[:8]}"
    assert np.float32(cost) == golden["mlp_cost"][0]
