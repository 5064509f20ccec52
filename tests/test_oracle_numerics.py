"""Oracle sanity at larger sizes: agreement with float64 numpy within the
componentwise dot-product bound used for all GEMM parity:
    |C - C64| <= tol * (|alpha| |A||B| + |beta| |C0|)_ij
plus exact small-integer known answers (any summation order is exact)."""
import numpy as np
import pytest


def ref64(ta, tb, A, B, alpha, beta, C0):
    a = A.T if ta else A
    b = B.T if tb else B
    a64, b64 = a.astype(np.float64), b.astype(np.float64)
    c = alpha * (a64 @ b64) + beta * C0.astype(np.float64)
    bound = abs(alpha) * (np.abs(a64) @ np.abs(b64)) + abs(beta) * np.abs(C0.astype(np.float64))
    return c, bound


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(37, 53, 61), (1, 97, 33), (64, 1, 129), (128, 96, 300)])
def test_gemm_vs_float64(ora, ta, tb, M, N, K):
    rng = np.random.default_rng(M * 1000 + N * 10 + K)
    A = rng.uniform(-1, 1, (K, M) if ta else (M, K)).astype(np.float32)
    B = rng.uniform(-1, 1, (N, K) if tb else (K, N)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (M, N)).astype(np.float32)
    for alpha, beta in [(1.0, 0.0), (0.5, 2.0), (1.0, 1.0)]:
        C = C0.copy()
        ora.sgemm(bool(ta), bool(tb), M, N, K, alpha, A, A.shape[1], B, B.shape[1], beta, C, N)
        c64, bound = ref64(ta, tb, A, B, alpha, beta, C0)
        assert np.all(np.abs(C - c64) <= 1e-5 * bound + 1e-30)


def test_gemm_exact_integers(ora):
    rng = np.random.default_rng(7)
    M, N, K = 19, 23, 29
    A = rng.integers(-8, 8, (M, K)).astype(np.float32)
    B = rng.integers(-8, 8, (K, N)).astype(np.float32)
    exact = (A.astype(np.int64) @ B.astype(np.int64)).astype(np.float32)
    for ta, tb in [(0, 0), (0, 1), (1, 0), (1, 1)]:
        a = np.ascontiguousarray(A.T) if ta else A
        b = np.ascontiguousarray(B.T) if tb else B
        C = np.zeros((M, N), np.float32)
        ora.sgemm(bool(ta), bool(tb), M, N, K, 1.0, a, a.shape[1], b, b.shape[1], 0.0, C, N)
        assert np.array_equal(C, exact)


def test_gemm_rows_equals_full(ora):
    rng = np.random.default_rng(3)
    M, N, K = 64, 80, 96
    A = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    B = rng.uniform(-1, 1, (K, N)).astype(np.float32)
    full = np.zeros((M, N), np.float32)
    ora.sgemm(False, False, M, N, K, 1.0, A, K, B, N, 0.0, full, N)
    part = np.zeros((M, N), np.float32)
    ora.sgemm_rows(False, False, 8, 24, M, N, K, 1.0, A, K, B, N, 0.0, part, N)
    assert np.array_equal(part[8:24], full[8:24])


def test_threads_do_not_change_results(ora):
    rng = np.random.default_rng(11)
    M, N, K = 33, 65, 130
    A = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    B = rng.uniform(-1, 1, (K, N)).astype(np.float32)
    outs = []
    for t in (1, 2, 5, 8):
        ora.set_threads(t)
        C = np.zeros((M, N), np.float32)
        ora.sgemm(False, False, M, N, K, 1.0, A, K, B, N, 0.0, C, N)
        outs.append(C)
    ora.set_threads(0)
    for o in outs[1:]:
        assert o.tobytes() == outs[0].tobytes()


def test_im2col_1x1_identity(ora):
    x = np.arange(2 * 3 * 4, dtype=np.float32)
    col = ora.im2col(2, 3, 4, 1, 1, 0, 0, 1, 1, 1, 1, x)
    assert col.ravel().tobytes() == x.tobytes()


def test_col2im_is_adjoint_of_im2col_without_dilation(ora):
    # <im2col(x), y> == <x, col2im(y)> when dilation == 1 (the reference's
    # col2im formula only departs from the adjoint for dilation > 1)
    rng = np.random.default_rng(5)
    C, H, W, k, p, s = 3, 9, 7, 3, 1, 2
    x = rng.integers(-4, 4, C * H * W).astype(np.float32)
    col = ora.im2col(C, H, W, k, k, p, p, s, s, 1, 1, x)
    y = rng.integers(-4, 4, col.size).astype(np.float32)
    back = np.zeros(C * H * W, np.float32)
    ora.col2im(C, H, W, k, k, p, p, s, s, 1, 1, y.copy(), back)
    assert float(np.dot(col.ravel().astype(np.float64), y)) == float(np.dot(x.astype(np.float64), back))


def test_conv_forward_matches_direct(ora):
    rng = np.random.default_rng(9)
    batch, C, H, W, F, k, s, p = 2, 3, 11, 11, 5, 3, 2, 1
    x = rng.uniform(0, 1, (batch, C, H, W)).astype(np.float32)
    w = rng.uniform(-0.3, 0.3, (F, C * k * k)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, F).astype(np.float32)
    out = ora.conv_forward(x, w, b, F, k, s, p, 4)
    # direct float64 convolution
    oh = (H + 2 * p - k) // s + 1
    xp = np.pad(x.astype(np.float64), ((0, 0), (0, 0), (p, p), (p, p)))
    ref = np.zeros((batch, F, oh, oh))
    wk = w.reshape(F, C, k, k).astype(np.float64)
    for i in range(oh):
        for j in range(oh):
            patch = xp[:, :, i * s:i * s + k, j * s:j * s + k]
            ref[:, :, i, j] = np.einsum("bckl,fckl->bf", patch, wk)
    ref += b[None, :, None, None]
    assert np.allclose(out, ref, atol=1e-5, rtol=1e-5)


def test_uniform_is_deterministic_and_in_range(ora):
    a = ora.uniform(1000, 2, 7)
    b = ora.uniform(1000, 2, 7)
    c = ora.uniform(1000, 2, 8)
    assert a.tobytes() == b.tobytes() and a.tobytes() != c.tobytes()
    assert a.min() >= -1.0 and a.max() < 1.0
