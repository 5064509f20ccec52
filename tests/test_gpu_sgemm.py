"""SGEMM parity on the GPU (boundary B device API and boundary A host API)
against the oracle (restated cblas_sgemm, ntensors.pas:2231-2304).

Bar:
  * NN and TN: bit-identical to the reference's ascending-k FMA chain
    (gfx950 f32 MFMA is an exact k-ordered fmaf chain).
  * NT: bit-identical to the reference's sdot_avx2 order (8 residue chains
    k mod 8, pairwise lane sum, alpha product, C add; sgemm_sdot.hip);
    with TNS_OPT_NT_SDOT = 0, within the componentwise bound below.
  * TT: bit-identical to the reference's scalar s_tt (alpha*A, *B, + sum,
    each rounded; sgemm_tt.hip on the VALU); with TNS_OPT_TT_EXACT = 0 (the
    MFMA kernel) componentwise |C - C_ref| <= 1e-4 * (|alpha||A||B| +
    |beta||C0|)_ij.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4


def bound(ta, tb, A, B, alpha, beta, C0):
    a = A.T if ta else A
    b = B.T if tb else B
    return abs(alpha) * (np.abs(a.astype(np.float64)) @ np.abs(b.astype(np.float64))) + \
        abs(beta) * np.abs(C0.astype(np.float64))


def run_dev(hip, torch, ta, tb, A, B, C0, alpha, beta):
    M, N = C0.shape
    K = A.shape[0] if ta else A.shape[1]
    dA, dB, dC = (torch.from_numpy(x).cuda() for x in (A, B, C0.copy()))
    hip.gemm(ta, tb, M, N, K, alpha, dA, 0, A.shape[1], dB, 0, B.shape[1], beta, dC, 0, N)
    hip.finish()
    return dC.cpu().numpy()


def run_ref(ora, ta, tb, A, B, C0, alpha, beta):
    M, N = C0.shape
    K = A.shape[0] if ta else A.shape[1]
    C = C0.copy()
    ora.sgemm(bool(ta), bool(tb), M, N, K, alpha, A, A.shape[1], B, B.shape[1], beta, C, N)
    return C


def operands(rng, ta, tb, M, N, K):
    A = rng.uniform(-1, 1, (K, M) if ta else (M, K)).astype(np.float32)
    B = rng.uniform(-1, 1, (N, K) if tb else (K, N)).astype(np.float32)
    C0 = rng.uniform(-1, 1, (M, N)).astype(np.float32)
    return A, B, C0


SHAPES = [(1, 1, 1), (5, 7, 13), (37, 53, 61), (128, 128, 32), (129, 130, 33), (256, 256, 256),
          (32, 1000, 27), (255, 2704 // 4, 256), (1, 513, 300), (300, 1, 64), (64, 64, 1),
          (200, 72, 0)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("ta,tb", [(0, 0), (1, 0)])
def test_nn_tn_bit_exact(hip, torch_cuda, ora, M, N, K, ta, tb):
    rng = np.random.default_rng(M * 7919 + N * 31 + K)
    A, B, C0 = operands(rng, ta, tb, M, N, K)
    for alpha, beta in [(1.0, 0.0), (0.5, 2.0), (1.0, 1.0), (-1.5, 0.25)]:
        got = run_dev(hip, torch_cuda, ta, tb, A, B, C0, alpha, beta)
        ref = run_ref(ora, ta, tb, A, B, C0, alpha, beta)
        assert np.array_equal(got, ref), (M, N, K, alpha, beta,
                                          float(np.abs(got - ref).max()))


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("ta,tb", [(0, 1), (1, 1), (0, 0), (1, 0)])
def test_all_transposes_within_bound(hip, torch_cuda, ora, M, N, K, ta, tb):
    rng = np.random.default_rng(M * 131 + N * 17 + K + 5)
    A, B, C0 = operands(rng, ta, tb, M, N, K)
    for alpha, beta in [(1.0, 0.0), (0.5, 2.0)]:
        got = run_dev(hip, torch_cuda, ta, tb, A, B, C0, alpha, beta)
        ref = run_ref(ora, ta, tb, A, B, C0, alpha, beta)
        bnd = bound(ta, tb, A, B, alpha, beta, C0)
        err = np.abs(got.astype(np.float64) - ref)
        assert np.all(err <= TOL * bnd + 1e-30), float((err / (bnd + 1e-30)).max())


NT_SHAPES = SHAPES + [(32, 4096, 4096), (32, 64, 784), (10, 32, 32), (3, 5, 8), (3, 5, 9),
                     (33, 65, 15), (64, 1152, 2704), (70, 90, 2304), (32, 27, 173056),
                     (64, 288, 20001), (1000, 2100, 169)]


@pytest.mark.parametrize("M,N,K", NT_SHAPES)
def test_nt_sdot_bit_exact(hip, torch_cuda, ora, M, N, K):
    """gemm(NoTrans, Trans) = s_nt over sdot_avx2 (ntensors.pas:1957-2005,
    1233-1306): every K mod 8 tail, float4 and scalar staging, skinny FC
    shapes (batch 32) and conv dW shapes."""
    rng = np.random.default_rng(M * 7 + N * 3 + K + 11)
    A, B, C0 = operands(rng, 0, 1, M, N, K)
    for alpha, beta in [(1.0, 0.0), (0.5, 2.0), (1.0, 1.0), (-1.5, 0.25)]:
        got = run_dev(hip, torch_cuda, 0, 1, A, B, C0, alpha, beta)
        ref = run_ref(ora, 0, 1, A, B, C0, alpha, beta)
        assert np.array_equal(got, ref), (M, N, K, alpha, beta,
                                          float(np.abs(got - ref).max()))
        if M * N * K > 1e8:
            break


def test_nt_sdot_batched_offsets_and_plain_order(hip, torch_cuda, ora):
    """Strided-batched NT with element offsets and padded leading dims; then
    the plain-order option (one ascending chain per element) within bound."""
    rng = np.random.default_rng(12)
    batch, M, N, K, lda, ldb, off = 3, 45, 70, 37, 41, 39, 5
    A = rng.uniform(-1, 1, off + batch * M * lda).astype(np.float32)
    B = rng.uniform(-1, 1, off + batch * N * ldb).astype(np.float32)
    C = rng.uniform(-1, 1, off + batch * M * N).astype(np.float32)
    dA, dB, dC = (torch_cuda.from_numpy(x.copy()).cuda() for x in (A, B, C))
    hip.gemmStridedBatched(False, True, M, N, K, 0.5, dA, off, lda, M * lda, dB, off, ldb,
                           N * ldb, 1.0, dC, off, N, M * N, batch)
    hip.finish()
    ref = C.copy()
    ora.sgemm_batch_strided(False, True, M, N, K, 0.5, A[off:], lda, M * lda, B[off:], ldb,
                            N * ldb, 1.0, ref[off:], N, M * N, batch)
    assert np.array_equal(dC.cpu().numpy(), ref)
    Mq, Nq, Kq = 129, 130, 67
    A2, B2, C2 = operands(rng, 0, 1, Mq, Nq, Kq)
    hip.setNtSdot(False)
    try:
        got = run_dev(hip, torch_cuda, 0, 1, A2, B2, C2, 1.0, 0.0)
    finally:
        hip.setNtSdot(True)
    ref = run_ref(ora, 0, 1, A2, B2, C2, 1.0, 0.0)
    bnd = bound(0, 1, A2, B2, 1.0, 0.0, C2)
    assert np.all(np.abs(got.astype(np.float64) - ref) <= TOL * bnd + 1e-30)


def test_nt_sdot_scalar_offsets_many_tiles(hip, torch_cuda, ora):
    """Scalar-staged 32 x 64 form with 32-bit row offsets (>= 1024 tiles, odd
    K): ragged M / N rows clamped to the last row, padded leading dims,
    element offsets and a strided batch."""
    rng = np.random.default_rng(21)
    batch, M, N, K, lda, ldb, off = 2, 500, 2001, 37, 41, 39, 5
    A = rng.uniform(-1, 1, off + batch * M * lda).astype(np.float32)
    B = rng.uniform(-1, 1, off + batch * N * ldb).astype(np.float32)
    C = rng.uniform(-1, 1, off + batch * M * N).astype(np.float32)
    dA, dB, dC = (torch_cuda.from_numpy(x.copy()).cuda() for x in (A, B, C))
    hip.gemmStridedBatched(False, True, M, N, K, 0.5, dA, off, lda, M * lda, dB, off, ldb,
                           N * ldb, 1.0, dC, off, N, M * N, batch)
    hip.finish()
    ref = C.copy()
    ora.sgemm_batch_strided(False, True, M, N, K, 0.5, A[off:], lda, M * lda, B[off:], ldb,
                            N * ldb, 1.0, ref[off:], N, M * N, batch)
    assert np.array_equal(dC.cpu().numpy(), ref)


CHAIN_SHAPES = [(1, 1, 1), (3, 5, 9), (33, 65, 15), (37, 53, 61), (32, 27, 2704), (17, 40, 1029),
                (64, 288, 4100), (70, 90, 2304), (5, 7, 0)]


@pytest.mark.parametrize("M,N,K", CHAIN_SHAPES)
def test_nt_sdot_every_form_bit_exact(hip, torch_cuda, ora, M, N, K):
    """Every kernel of the sdot-order NT product (TNS_OPT_SDOT_FORM: the MFMA
    kernel, each VALU chain variant, sgemm_sdot_chains.hip, and each
    residue-register form, sgemm_sdot_rc.hip) gives the
    reference's s_nt/sdot_avx2 result bit for bit: K mod 8 tails, K not a
    multiple of 4 (scalar staging), ragged tiles, every beta mode."""
    rng = np.random.default_rng(M * 5 + N * 7 + K + 1)
    A, B, C0 = operands(rng, 0, 1, M, N, K)
    refs = {ab: run_ref(ora, 0, 1, A, B, C0, *ab) for ab in [(1.0, 0.0), (0.5, 2.0), (1.0, 1.0)]}
    try:
        forms = list(range(hip.sdotChainsVariants() + 1))
        forms += [64 + v for v in range(hip.sdotRcVariants())]
        for form in forms:
            hip.setSdotForm(form)
            for (alpha, beta), ref in refs.items():
                got = run_dev(hip, torch_cuda, 0, 1, A, B, C0, alpha, beta)
                assert np.array_equal(got, ref), (form, M, N, K, alpha, beta,
                                                  float(np.abs(got - ref).max()))
    finally:
        hip.setSdotForm(-1)


def test_nt_sdot_chains_batched_offsets(hip, torch_cuda, ora):
    """Strided-batched NT with offsets / padded leading dims on every chain
    variant (the conv dW call shape: batch of images, BETA via the driver)."""
    rng = np.random.default_rng(21)
    batch, M, N, K, lda, ldb, off = 3, 45, 70, 1037, 1041, 1039, 5
    A = rng.uniform(-1, 1, off + batch * M * lda).astype(np.float32)
    B = rng.uniform(-1, 1, off + batch * N * ldb).astype(np.float32)
    C = rng.uniform(-1, 1, off + batch * M * N).astype(np.float32)
    ref = C.copy()
    ora.sgemm_batch_strided(False, True, M, N, K, 0.5, A[off:], lda, M * lda, B[off:], ldb,
                            N * ldb, 1.0, ref[off:], N, M * N, batch)
    dA, dB = (torch_cuda.from_numpy(x.copy()).cuda() for x in (A, B))
    try:
        forms = list(range(1, hip.sdotChainsVariants() + 1))
        forms += [64 + v for v in range(hip.sdotRcVariants())]
        for form in forms:
            hip.setSdotForm(form)
            dC = torch_cuda.from_numpy(C.copy()).cuda()
            hip.gemmStridedBatched(False, True, M, N, K, 0.5, dA, off, lda, M * lda, dB, off, ldb,
                                   N * ldb, 1.0, dC, off, N, M * N, batch)
            hip.finish()
            assert np.array_equal(dC.cpu().numpy(), ref), form
    finally:
        hip.setSdotForm(-1)


@pytest.mark.parametrize("M,N,K", SHAPES + [(2945, 2945, 37)])
def test_tt_bit_exact(hip, torch_cuda, ora, M, N, K):
    """gemm(Trans, Trans) = s_tt (ntensors.pas:2159-2182): both tile sizes
    (2945^2 takes the 128x128 tiles), every K mod 16 tail, K = 0."""
    rng = np.random.default_rng(M * 5 + N * 13 + K + 3)
    A, B, C0 = operands(rng, 1, 1, M, N, K)
    for alpha, beta in [(1.0, 0.0), (0.5, 2.0), (1.0, 1.0), (-1.5, 0.25)]:
        got = run_dev(hip, torch_cuda, 1, 1, A, B, C0, alpha, beta)
        ref = run_ref(ora, 1, 1, A, B, C0, alpha, beta)
        assert np.array_equal(got, ref), (M, N, K, alpha, beta,
                                          float(np.abs(got - ref).max()))
        if M * N * K > 1e8:
            break


def test_tt_batched_offsets_and_mfma_option(hip, torch_cuda, ora):
    """Strided-batched TT with element offsets and padded leading dims; then
    the MFMA kernel (TNS_OPT_TT_EXACT = 0) within bound."""
    rng = np.random.default_rng(21)
    batch, M, N, K, lda, ldb, off = 3, 45, 70, 37, 49, 39, 5
    A = rng.uniform(-1, 1, off + batch * K * lda).astype(np.float32)
    B = rng.uniform(-1, 1, off + batch * N * ldb).astype(np.float32)
    C = rng.uniform(-1, 1, off + batch * M * N).astype(np.float32)
    dA, dB, dC = (torch_cuda.from_numpy(x.copy()).cuda() for x in (A, B, C))
    hip.gemmStridedBatched(True, True, M, N, K, 0.5, dA, off, lda, K * lda, dB, off, ldb,
                           N * ldb, 2.0, dC, off, N, M * N, batch)
    hip.finish()
    ref = C.copy()
    ora.sgemm_batch_strided(True, True, M, N, K, 0.5, A[off:], lda, K * lda, B[off:], ldb,
                            N * ldb, 2.0, ref[off:], N, M * N, batch)
    assert np.array_equal(dC.cpu().numpy(), ref)
    A2, B2, C2 = operands(rng, 1, 1, 129, 130, 67)
    hip.setTtExact(False)
    try:
        got = run_dev(hip, torch_cuda, 1, 1, A2, B2, C2, 1.0, 0.0)
    finally:
        hip.setTtExact(True)
    ref = run_ref(ora, 1, 1, A2, B2, C2, 1.0, 0.0)
    assert not np.array_equal(got, ref)  # the MFMA kernel fuses: a different rounding
    bnd = bound(1, 1, A2, B2, 1.0, 0.0, C2)
    assert np.all(np.abs(got.astype(np.float64) - ref) <= TOL * bnd + 1e-30)


def test_unaligned_leading_dims_and_offsets(hip, torch_cuda, ora):
    # lda/ldb/ldc larger than the logical width, element offsets into buffers
    rng = np.random.default_rng(1)
    M, N, K, lda, ldb, ldc, off = 45, 70, 33, 37, 75, 73, 3
    A = rng.uniform(-1, 1, off + M * lda).astype(np.float32)
    B = rng.uniform(-1, 1, off + K * ldb).astype(np.float32)
    C = rng.uniform(-1, 1, off + M * ldc).astype(np.float32)
    dA, dB, dC = (torch_cuda.from_numpy(x.copy()).cuda() for x in (A, B, C))
    hip.gemm(False, False, M, N, K, 1.0, dA, off, lda, dB, off, ldb, 0.5, dC, off, ldc)
    hip.finish()
    ref = C.copy()
    ora.sgemm(False, False, M, N, K, 1.0, A[off:], lda, B[off:], ldb, 0.5, ref[off:], ldc)
    assert np.array_equal(dC.cpu().numpy(), ref)


def test_strided_batched_shared_a(hip, torch_cuda, ora):
    # conv-style: strideA = 0 (weights shared), nConvolutionLayer.pas:1078
    rng = np.random.default_rng(2)
    batch, M, N, K = 5, 64, 300, 75
    A = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    B = rng.uniform(-1, 1, (batch, K, N)).astype(np.float32)
    C = np.zeros((batch, M, N), np.float32)
    dA, dB, dC = (torch_cuda.from_numpy(x.copy()).cuda() for x in (A, B, C))
    hip.gemmStridedBatched(False, False, M, N, K, 1.0, dA, 0, K, 0, dB, 0, N, K * N, 0.0, dC, 0,
                           N, M * N, batch)
    hip.finish()
    ref = C.copy()
    ora.sgemm_batch_strided(False, False, M, N, K, 1.0, A, K, 0, B, N, K * N, 0.0, ref, N, M * N,
                            batch)
    assert np.array_equal(dC.cpu().numpy(), ref)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False)])
@pytest.mark.parametrize("layout", ["strided", "irregular", "host"])
def test_gemm_batched_pointer_arrays(hip, torch_cuda, ora, ta, tb, layout):
    """TNNCuda.gemmBatched (nncuda.pas:727-760): arrays of matrix pointers
    written to the device with writeBuffer, as nConvolutionLayer.pas:1083-1085
    builds them (shared weights: every A entry the same), equally spaced
    (one strided launch), irregular (GEMM by GEMM), or host-resident."""
    T = torch_cuda
    batch, M, N, K = 5, 48, 70, 37
    rng = np.random.default_rng(7)
    A = rng.uniform(-1, 1, (M * K,)).astype(np.float32)
    Bs = [rng.uniform(-1, 1, (K * N,)).astype(np.float32) for _ in range(batch)]
    C0 = [rng.uniform(-1, 1, (M * N,)).astype(np.float32) for _ in range(batch)]
    off = 3
    dA = T.from_numpy(np.concatenate([np.zeros(off, np.float32), A])).cuda()
    if layout == "irregular":   # separate allocations, unequal gaps
        dB = [T.from_numpy(np.concatenate([np.zeros(off, np.float32), b])).cuda() for b in Bs]
        dC = [T.from_numpy(np.concatenate([np.zeros(off, np.float32), c])).cuda() for c in C0]
        pb = [t.data_ptr() for t in dB]
        pc = [t.data_ptr() for t in dC]
    else:
        bigB = T.from_numpy(np.concatenate([np.zeros(off, np.float32), *Bs])).cuda()
        bigC = T.from_numpy(np.concatenate([np.zeros(off, np.float32), *C0])).cuda()
        pb = [bigB.data_ptr() + 4 * i * K * N for i in range(batch)]
        pc = [bigC.data_ptr() + 4 * i * M * N for i in range(batch)]
    pa = [dA.data_ptr()] * batch
    lda, ldb = (M if ta else K), (K if tb else N)
    if layout == "host":
        arrs = [np.array(p, np.int64) for p in (pa, pb, pc)]
        args = [a.ctypes.data for a in arrs]
    else:
        args = [T.zeros(batch, dtype=T.int64, device="cuda") for _ in range(3)]
        for d, p in zip(args, (pa, pb, pc)):   # writeBuffer of the pointer arrays
            host = np.array(p, np.int64)
            hip.lib.tns_hip_write_buffer(hip.ctx, d.data_ptr(), host.nbytes, host.ctypes.data)
    hip.gemmBatched(ta, tb, M, N, K, 1.0, args[0], off, lda, args[1], off, ldb, 0.5, args[2], off,
                    N, batch)
    hip.finish()
    if layout == "irregular":
        got = [t.cpu().numpy()[off:] for t in dC]
    else:
        g = bigC.cpu().numpy()[off:]
        got = [g[i * M * N:(i + 1) * M * N] for i in range(batch)]
    for i in range(batch):
        ref = C0[i].copy()
        ora.sgemm(ta, tb, M, N, K, 1.0, A, lda, Bs[i], ldb, 0.5, ref, N)
        assert np.array_equal(got[i], ref), i


@pytest.mark.parametrize("alias", ["overlap", "c_is_b"])
def test_gemm_batched_dependent_entries_in_order(hip, torch_cuda, ora, alias):
    """gemmBatched whose equally spaced entries are NOT independent: C entries
    one row apart (each GEMM reads rows the previous one wrote, BETA = 1), or
    C entry i the B entry i+1 — run GEMM by GEMM in array order (the header's
    contract), not as one concurrent strided launch: bit-exact against the
    oracle applied entry by entry to one buffer."""
    T = torch_cuda
    batch, M, N, K = 4, 24, 32, 32
    rng = np.random.default_rng(11)
    A = rng.uniform(-1, 1, (M * K,)).astype(np.float32)
    if alias == "overlap":
        buf = rng.uniform(-1, 1, (M * N + (batch - 1) * N,)).astype(np.float32)
        Bs = rng.uniform(-1, 1, (batch * K * N,)).astype(np.float32)
        dA, dB, dBuf = (T.from_numpy(x.copy()).cuda() for x in (A, Bs, buf))
        pa = [dA.data_ptr()] * batch
        pb = [dB.data_ptr() + 4 * i * K * N for i in range(batch)]
        pc = [dBuf.data_ptr() + 4 * i * N for i in range(batch)]
        ref = buf.copy()
        for i in range(batch):
            c = ref[i * N:i * N + M * N].copy()
            ora.sgemm(False, False, M, N, K, 1.0, A, K, Bs[i * K * N:(i + 1) * K * N], N, 1.0, c, N)
            ref[i * N:i * N + M * N] = c
    else:  # K == M: C_i (M x N) is B_{i+1} (K x N)
        buf = rng.uniform(-1, 1, ((batch + 1) * K * N,)).astype(np.float32)
        dA, dBuf = (T.from_numpy(x.copy()).cuda() for x in (A, buf))
        pa = [dA.data_ptr()] * batch
        pb = [dBuf.data_ptr() + 4 * i * K * N for i in range(batch)]
        pc = [dBuf.data_ptr() + 4 * (i + 1) * K * N for i in range(batch)]
        ref = buf.copy()
        for i in range(batch):
            c = ref[(i + 1) * K * N:(i + 2) * K * N].copy()
            ora.sgemm(False, False, M, N, K, 1.0, A, K, ref[i * K * N:(i + 1) * K * N].copy(), N,
                      1.0, c, N)
            ref[(i + 1) * K * N:(i + 2) * K * N] = c
    arrs = [np.array(p, np.int64) for p in (pa, pb, pc)]
    hip.gemmBatched(False, False, M, N, K, 1.0, arrs[0].ctypes.data, 0, K, arrs[1].ctypes.data, 0,
                    N, 1.0, arrs[2].ctypes.data, 0, N, batch)
    hip.finish()
    assert np.array_equal(dBuf.cpu().numpy(), ref)


def test_beta0_strict_propagates_nan(hip, torch_cuda, hiplib):
    A = np.ones((4, 4), np.float32)
    C = np.zeros((4, 4), np.float32)
    C[1, 2] = np.nan
    C[3, 0] = np.inf
    dA, dB, dC = (torch_cuda.from_numpy(x.copy()).cuda() for x in (A, A, C))
    hip.gemm(False, False, 4, 4, 4, 1.0, dA, 0, 4, dB, 0, 4, 0.0, dC, 0, 4)
    hip.finish()
    out = dC.cpu().numpy()
    assert np.isnan(out[1, 2]) and np.isnan(out[3, 0]) and out[0, 0] == 4.0
    # BLAS convention when strict mode is off: C not read
    hiplib.tns_set_option(0, 0)
    try:
        dC = torch_cuda.from_numpy(C.copy()).cuda()
        hip.gemm(False, False, 4, 4, 4, 1.0, dA, 0, 4, dB, 0, 4, 0.0, dC, 0, 4)
        hip.finish()
        assert np.all(dC.cpu().numpy() == 4.0)
    finally:
        hiplib.tns_set_option(0, 1)


def test_host_api_matmul_accumulates(hiplib, torch_cuda, ora):
    # boundary A: TSingleTensor.matMul via the op-table drop-in (beta = One)
    from tensorium_amd.ntensors import matMul
    rng = np.random.default_rng(3)
    a = rng.uniform(-1, 1, (256, 256)).astype(np.float32)
    b = rng.uniform(-1, 1, (256, 256)).astype(np.float32)
    c = rng.uniform(-1, 1, (256, 256)).astype(np.float32)
    ref = c.copy()
    ora.sgemm(False, False, 256, 256, 256, 1.0, a, 256, b, 256, 1.0, ref, 256)
    got = matMul(a, b, c.copy())
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_host_api_all_transposes(hiplib, torch_cuda, ora, ta, tb):
    from tensorium_amd.ntensors import bind_hip_op_table
    ops = bind_hip_op_table()
    rng = np.random.default_rng(4 + ta * 2 + tb)
    M, N, K = 70, 90, 110
    A, B, C0 = operands(rng, ta, tb, M, N, K)
    C = C0.copy()
    ops.gemm(101, 112 if ta else 111, 112 if tb else 111, M, N, K, 0.5, A.ctypes.data,
             A.shape[1], B.ctypes.data, B.shape[1], 2.0, C.ctypes.data, N)
    assert hiplib.tns_last_error() == b""
    ref = run_ref(ora, ta, tb, A, B, C0, 0.5, 2.0)
    assert np.array_equal(C, ref)


def test_4096_cubed_sampled_rows_bit_exact(hip, torch_cuda, ora):
    """Full BASELINE size: GPU 4096^3 against the oracle on 24 sampled rows
    (the oracle restricted to those rows computes the identical chains)."""
    n = 4096
    A = ora.uniform(n * n, 2, 0).reshape(n, n)
    B = ora.uniform(n * n, 2, 1).reshape(n, n)
    dA, dB = torch_cuda.from_numpy(A).cuda(), torch_cuda.from_numpy(B).cuda()
    dC = torch_cuda.zeros((n, n), device="cuda")
    hip.gemm(False, False, n, n, n, 1.0, dA, 0, n, dB, 0, n, 0.0, dC, 0, n)
    hip.finish()
    got = dC.cpu().numpy()
    rows = [0, 1, 127, 128, 129, 1000, 2047, 2048, 3071, 4095] + list(range(600, 614))
    ref = np.zeros((n, n), np.float32)
    for r in rows:
        ora.sgemm_rows(False, False, r, r + 1, n, n, n, 1.0, A, n, B, n, 0.0, ref, n)
        assert np.array_equal(got[r], ref[r]), r
    # size-independent property: checksum linearity  1^T (A B) = (1^T A) B
    lhs = got.astype(np.float64).sum(axis=0)
    rhs = A.astype(np.float64).sum(axis=0) @ B.astype(np.float64)
    scale = np.abs(A).astype(np.float64).sum(axis=0) @ np.abs(B).astype(np.float64)
    assert np.all(np.abs(lhs - rhs) <= 1e-4 * scale)


def test_every_tile_variant_bit_exact(hip, torch_cuda, ora):
    """Each tile shape of the tuning table, forced, on ragged shapes: NN/TN
    bit-exact; variants limited to float4/NN report UNSUPPORTED otherwise."""
    from tensorium_amd._abi import TnsError
    names = hip.gemmVariants()
    for v, name in enumerate(names):
        for (M, N, K) in [(37, 53, 61), (129, 130, 33), (256, 260, 96), (64, 512, 40)]:
            for ta in (0, 1):
                rng = np.random.default_rng(v * 1000 + M + ta)
                A, B, C0 = operands(rng, ta, 0, M, N, K)
                dA, dB, dC = (torch_cuda.from_numpy(x).cuda() for x in (A, B, C0.copy()))
                try:
                    hip.gemmVariant(v, bool(ta), False, M, N, K, 0.5, dA, 0, A.shape[1], 0,
                                    dB, 0, B.shape[1], 0, 2.0, dC, 0, N, 0, 1)
                except TnsError:
                    continue
                hip.finish()
                ref = run_ref(ora, ta, 0, A, B, C0, 0.5, 2.0)
                assert np.array_equal(dC.cpu().numpy(), ref), (name, M, N, K, ta)


@pytest.mark.parametrize("M,N,K", [(256, 256, 32), (512, 768, 96), (256, 512, 2080)])
def test_nn_big_kernel_bit_exact(hip, torch_cuda, ora, M, N, K):
    """The dedicated large-NN kernels (sgemm_nn_big.hip: LDS-DMA B, permuted /
    swizzled transposed A), forced at small multiples of its 256x256x32 tile:
    every beta mode and alpha != 1 (the A_PART pre-multiply), bit-exact."""
    forms = [v for v, n in enumerate(hip.gemmVariants()) if n.endswith("nn_big")]
    assert len(forms) >= 7   # (+1 in the diagnostics build)
    rng = np.random.default_rng(M + N + K)
    A, B, C0 = operands(rng, 0, 0, M, N, K)
    C0[0, 0] = np.nan  # strict beta = 0 keeps 0*NaN (ntensors.pas:2259)
    for alpha, beta in [(1.0, 0.0), (0.5, 2.0), (1.0, 1.0), (-1.5, 0.25)]:
        ref = run_ref(ora, 0, 0, A, B, C0, alpha, beta)
        for v in forms:
            dA, dB, dC = (torch_cuda.from_numpy(x).cuda() for x in (A, B, C0.copy()))
            hip.gemmVariant(v, False, False, M, N, K, alpha, dA, 0, K, 0, dB, 0, N, 0, beta, dC,
                            0, N, 0, 1)
            hip.finish()
            got = dC.cpu().numpy()
            assert np.array_equal(got, ref, equal_nan=True), (v, alpha, beta)


def test_nn_big_kernel_batched(hip, torch_cuda, ora):
    """Strided-batched through the large-NN kernels (blockIdx.y = batch)."""
    forms = [v for v, n in enumerate(hip.gemmVariants()) if n.endswith("nn_big")]
    rng = np.random.default_rng(5)
    batch, M, N, K = 3, 256, 256, 64
    A = rng.uniform(-1, 1, (batch, M, K)).astype(np.float32)
    B = rng.uniform(-1, 1, (batch, K, N)).astype(np.float32)
    C = rng.uniform(-1, 1, (batch, M, N)).astype(np.float32)
    ref = C.copy()
    ora.sgemm_batch_strided(False, False, M, N, K, 1.0, A.reshape(-1), K, M * K, B.reshape(-1), N,
                            K * N, 1.0, ref.reshape(-1), N, M * N, batch)
    for v in forms:
        dA, dB, dC = (torch_cuda.from_numpy(x.copy()).cuda() for x in (A, B, C))
        hip.gemmVariant(v, False, False, M, N, K, 1.0, dA, 0, K, M * K, dB, 0, N, K * N, 1.0, dC,
                        0, N, M * N, batch)
        hip.finish()
        assert np.array_equal(dC.cpu().numpy(), ref), v
