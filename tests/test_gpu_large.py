"""Maximum sizes: operands past 2^31 elements (64-bit indexing in the GEMM,
the sdot NT kernel and im2col) and a conv image past the implicit GEMM's
32-bit buffer range (the library schedule falls back to im2col + GEMM, the
forced implicit schedule reports an error).  Checked bit-exact against the
oracle on sampled rows / pixels (the full products would take the oracle
minutes).  Device memory per test: <= 25 GB of the MI355X's 288 GB."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free(torch):
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("tb", [False, True])
def test_gemm_output_past_2p31_elements(hip, torch_cuda, ora, tb):
    torch = torch_cuda
    M, N, K = 65600, 32775, 5  # C: 2.15e9 elements (8.6 GB)
    assert M * N > 2 ** 31
    g = torch.Generator(device="cuda").manual_seed(7)
    A = torch.rand(M, K, device="cuda", generator=g) * 2 - 1
    B = torch.rand((N, K) if tb else (K, N), device="cuda", generator=g) * 2 - 1
    C = torch.empty(M, N, device="cuda")
    hip.gemm(False, tb, M, N, K, 1.0, A, 0, K, B, 0, K if tb else N, 0.0, C, 0, N)
    hip.finish()
    a, b = A.cpu().numpy(), B.cpu().numpy()
    for r in (0, 1, 32767, 65535, 65536, M - 1):
        ref = np.zeros((1, N), np.float32)
        ora.sgemm(False, tb, 1, N, K, 1.0, a[r:r + 1].copy(), K, b, K if tb else N, 0.0, ref, N)
        assert np.array_equal(C[r].cpu().numpy(), ref[0]), r
    del A, B, C
    _free(torch)


def test_im2col_past_2p31_elements(hip, torch_cuda, ora):
    torch = torch_cuda
    C, H, k = 72, 2048, 3  # col: 72*9 x 2048^2 = 2.7e9 elements (10.9 GB)
    x = torch.rand(C, H, H, device="cuda")
    col = torch.empty(C * k * k, H * H, device="cuda")
    assert col.numel() > 2 ** 31
    hip.im2col(C, H, H, k, k, 1, 1, 1, 1, 1, 1, x, 0, col, 0)
    hip.finish()
    for c in (0, 35, C - 1):
        plane = x[c].cpu().numpy()
        ref = ora.im2col(1, H, H, k, k, 1, 1, 1, 1, 1, 1, plane.reshape(1, 1, H, H).copy())[0]
        for kk in (0, 4, 8):
            assert np.array_equal(col[c * 9 + kk].cpu().numpy(), ref[kk]), (c, kk)
    del x, col
    _free(torch)


def test_conv_image_past_implicit_range_falls_back(hip, torch_cuda, ora):
    """One 130 x 2048 x 2048 image (2.2 GB > 2^31 B): the library schedule
    runs im2col + GEMM (19.6 GB workspace); the forced implicit schedule is
    refused with an error, never computed with wrapped offsets."""
    from tensorium_amd._abi import TnsError
    torch = torch_cuda
    Cin, H, F, k = 130, 2048, 3, 3
    K = Cin * k * k
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.rand(1, Cin, H, H, device="cuda", generator=g)
    w = (torch.rand(F, K, device="cuda", generator=g) * 2 - 1) * 0.05
    b = torch.rand(F, device="cuda", generator=g) * 0.2 - 0.1
    out = torch.full((1, F, H, H), float("nan"), device="cuda")
    with pytest.raises(TnsError):
        hip.convForward(1, Cin, H, H, x, w, b, F, k, 1, 1, 1, 9, None, out, fused=3)
    hip.convForward(1, Cin, H, H, x, w, b, F, k, 1, 1, 1, 9, None, out, fused=1)
    hip.finish()
    got = out[0].reshape(F, -1)
    wn, bn = w.cpu().numpy(), b.cpu().numpy()
    pix = [0, 1, H - 1, H, H * H // 2 + 17, H * H - 1]
    xs = x[0].cpu().numpy()
    xp = np.pad(xs, ((0, 0), (1, 1), (1, 1)))
    for p in pix:
        r, cc = divmod(p, H)
        colp = np.ascontiguousarray(xp[:, r:r + 3, cc:cc + 3].reshape(K, 1))
        ref = np.zeros((F, 1), np.float32)
        ora.sgemm(False, False, F, 1, K, 1.0, wn, K, colp, 1, 0.0, ref, 1)
        v = (ref[:, 0] + bn).astype(np.float32)  # forwardBias: one rounding
        v = np.where(v < 0, v * np.float32(0.1), v).astype(np.float32)  # leaky (AVX2 0.1f)
        assert np.array_equal(got[:, p].cpu().numpy(), v), p
    del x, w, b, out, got
    _free(torch)
