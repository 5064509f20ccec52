"""Boundary A's host-pointer GEMM pipeline (chunked uploads / GEMMs /
downloads on two streams) and the single-process multi-device entry point
tns_hip_sgemm_strided_batched_multi.

The one-GPU box can only give several CONTEXTS on the same device, so the
multi-device path is exercised with devices [0], [0, 0] and [0, 0, 0]: the
shards, the per-slot threads and pipelines and the shared-operand broadcast
(a device-to-device copy when both slots sit on one device, a peer copy
otherwise) all run; results must be bit-identical to the single-call path
and to the oracle.  Host gaps (ldc > N, strideC > M*ldc) must survive."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _p(a):
    return a.ctypes.data


def _ref(ora, ta, tb, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C0, ldc, sC, batch):
    ref = C0.copy()
    ora.sgemm_batch_strided(bool(ta), bool(tb), M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, ref,
                            ldc, sC, batch)
    return ref


def _case(rng, ta, tb, M, N, K, batch, shared_a=False, ldc_pad=0, gap=0):
    lda = M if ta else K
    ldb = K if tb else N
    ldc = N + ldc_pad
    a_one, b_one = (K if ta else M) * lda, (N if tb else K) * ldb
    sA = 0 if shared_a else a_one
    sB, sC = b_one, M * ldc + gap
    A = rng.uniform(-1, 1, max(a_one if shared_a else batch * a_one, 1)).astype(np.float32)
    B = rng.uniform(-1, 1, batch * b_one).astype(np.float32)
    C0 = rng.uniform(-1, 1, batch * sC).astype(np.float32)
    return lda, ldb, ldc, sA, sB, sC, A, B, C0


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("ta,tb,shared,beta,ldc_pad,gap", [
    (0, 0, False, 0.0, 0, 0), (1, 0, True, 1.0, 3, 5), (0, 1, False, 0.5, 0, 7),
    (1, 1, True, 0.0, 2, 0)])
def test_multi_device_strided_batched(hiplib, torch_cuda, ora, devices, ta, tb, shared, beta,
                                      ldc_pad, gap):
    rng = np.random.default_rng(len(devices) * 100 + ta * 10 + tb)
    M, N, K, batch = 67, 45, 53, 7
    lda, ldb, ldc, sA, sB, sC, A, B, C0 = _case(rng, ta, tb, M, N, K, batch, shared, ldc_pad, gap)
    ref = _ref(ora, ta, tb, M, N, K, 0.75, A, lda, sA, B, ldb, sB, beta, C0, ldc, sC, batch)
    got = C0.copy()
    dev = (C.c_int32 * len(devices))(*devices)
    rc = hiplib.tns_hip_sgemm_strided_batched_multi(dev, len(devices), ta, tb, M, N, K, 0.75,
                                                    _p(A), lda, sA, _p(B), ldb, sB, beta,
                                                    _p(got), ldc, sC, batch)
    assert rc == 0, hiplib.tns_last_error()
    # the reference's exact per-element chains; gaps untouched
    assert np.array_equal(got, ref)
    single = C0.copy()
    hiplib.tns_cblas_sgemm_batch_strided(101, 112 if ta else 111, 112 if tb else 111, M, N, K,
                                         0.75, _p(A), lda, sA, _p(B), ldb, sB, beta, _p(single),
                                         ldc, sC, batch)
    assert hiplib.tns_last_error() == b""
    assert np.array_equal(single, got)


@pytest.mark.parametrize("devices", [[0, 1], [1, 0, 1]])
def test_multi_device_distinct_gpus(hiplib, torch_cuda, ora, devices):
    """The real cross-device branch: shards on distinct GPUs, the shared
    operand peer-copied over xGMI (hipMemcpyPeerAsync) and per-thread
    hipSetDevice onto the second GPU.  Needs two GPUs (skipped on the 1-GPU
    box; runs wherever the multi-GPU evidence is gathered)."""
    if hiplib.tns_device_count() < 2:
        pytest.skip("needs >= 2 GPUs (the cross-device peer-copy branch)")
    for shared in (True, False):
        rng = np.random.default_rng(31 + len(devices) + shared)
        M, N, K, batch = 96, 80, 72, 9
        lda, ldb, ldc, sA, sB, sC, A, B, C0 = _case(rng, 0, 0, M, N, K, batch, shared, 1, 3)
        ref = _ref(ora, 0, 0, M, N, K, 1.0, A, lda, sA, B, ldb, sB, 0.0, C0, ldc, sC, batch)
        got = C0.copy()
        dev = (C.c_int32 * len(devices))(*devices)
        rc = hiplib.tns_hip_sgemm_strided_batched_multi(dev, len(devices), 0, 0, M, N, K, 1.0,
                                                        _p(A), lda, sA, _p(B), ldb, sB, 0.0,
                                                        _p(got), ldc, sC, batch)
        assert rc == 0, hiplib.tns_last_error()
        assert np.array_equal(got, ref), (devices, shared)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_device_single_gemm_no_broadcast(hiplib, torch_cuda, ora, devices):
    """A batch-1 call over several slots (the op-table's plain gemm with
    tns_set_op_devices): only slot 0 has work, nothing is broadcast, and the
    result is the single-device one."""
    rng = np.random.default_rng(77)
    M, N, K = 130, 70, 90
    lda, ldb, ldc, sA, sB, sC, A, B, C0 = _case(rng, 0, 0, M, N, K, 1, True)
    ref = _ref(ora, 0, 0, M, N, K, 1.0, A, lda, 0, B, ldb, 0, 0.5, C0, ldc, sC, 1)
    got = C0.copy()
    dev = (C.c_int32 * len(devices))(*devices)
    rc = hiplib.tns_hip_sgemm_strided_batched_multi(dev, len(devices), 0, 0, M, N, K, 1.0, _p(A),
                                                    lda, 0, _p(B), ldb, 0, 0.5, _p(got), ldc, sC, 1)
    assert rc == 0, hiplib.tns_last_error()
    assert np.array_equal(got, ref)


def test_op_table_spread_over_devices(hiplib, torch_cuda, ora):
    """tns_set_op_devices makes the unmodified op-table pointer
    (gemmStridedBatched) run sharded; n = 1 restores the default context."""
    rng = np.random.default_rng(11)
    M, N, K, batch = 40, 33, 29, 5
    lda, ldb, ldc, sA, sB, sC, A, B, C0 = _case(rng, 0, 0, M, N, K, batch)
    ref = _ref(ora, 0, 0, M, N, K, 1.0, A, lda, sA, B, ldb, sB, 0.0, C0, ldc, sC, batch)
    dev = (C.c_int32 * 2)(0, 0)
    assert hiplib.tns_set_op_devices(dev, 2) == 0
    try:
        got = C0.copy()
        hiplib.tns_cblas_sgemm_batch_strided(101, 111, 111, M, N, K, 1.0, _p(A), lda, sA, _p(B),
                                             ldb, sB, 0.0, _p(got), ldc, sC, batch)
        assert hiplib.tns_last_error() == b""
        assert np.array_equal(got, ref)
    finally:
        assert hiplib.tns_set_op_devices(dev, 1) == 0
    bad = (C.c_int32 * 1)(99)
    assert hiplib.tns_set_op_devices(bad, 1) == 1
    hiplib.tns_clear_error()


@pytest.mark.parametrize("ta,tb,beta,M", [(0, 0, 0.0, 2048), (1, 0, 1.0, 2100), (0, 1, 2.0, 1536),
                                          (1, 1, 0.0, 1030)])
def test_host_pipeline_row_chunks(hiplib, hip, torch_cuda, ta, tb, beta, M):
    """One GEMM split into row chunks of C (A's rows, or A's columns when
    transposed, uploaded per chunk; B once): bit-identical to the same GEMM
    run on device-resident operands."""
    torch = torch_cuda
    rng = np.random.default_rng(M + ta)
    N, K = 384, 320
    lda, ldb, ldc = (M if ta else K), (K if tb else N), N + 4
    A = rng.uniform(-1, 1, (K if ta else M) * lda).astype(np.float32)
    B = rng.uniform(-1, 1, (N if tb else K) * ldb).astype(np.float32)
    C0 = rng.uniform(-1, 1, M * ldc).astype(np.float32)
    got = C0.copy()
    hiplib.tns_cblas_sgemm(101, 112 if ta else 111, 112 if tb else 111, M, N, K, 1.25, _p(A), lda,
                           _p(B), ldb, beta, _p(got), ldc)
    assert hiplib.tns_last_error() == b""
    dA, dB, dC = (torch.from_numpy(x.copy()).cuda() for x in (A, B, C0))
    hip.gemm(ta, tb, M, N, K, 1.25, dA, 0, lda, dB, 0, ldb, beta, dC, 0, ldc)
    hip.finish()
    assert np.array_equal(got, dC.cpu().numpy())
