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
