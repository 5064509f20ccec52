"""im2col / col2im on the GPU vs the oracle (sim2Col ntensors.pas:11415-11532,
scol2im 11650-11879).  Bar: bit-exact (memcmp) for im2col; col2im is a
gather that adds in the reference's single-threaded order => bit-exact too."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GEOS = [  # C, H, W, k, pad, stride, dil
    (3, 7, 5, 3, 1, 1, 1), (5, 9, 11, 3, 1, 2, 1), (3, 8, 8, 1, 0, 1, 1), (2, 10, 7, 3, 0, 2, 2),
    (5, 13, 13, 3, 1, 1, 2), (3, 6, 9, 1, 0, 2, 1), (4, 16, 16, 3, 1, 2, 1), (1, 5, 5, 5, 2, 1, 1),
    (3, 416 // 8, 416 // 8, 3, 1, 1, 1), (2, 3, 3, 3, 0, 1, 1), (2, 4, 4, 3, 0, 3, 2),
]


@pytest.mark.parametrize("geo", GEOS)
@pytest.mark.parametrize("batch", [1, 3])
def test_im2col_bit_exact(hip, torch_cuda, ora, geo, batch):
    C, H, W, k, p, s, d = geo
    x = ora.uniform(batch * C * H * W, 3, sum(geo))
    ref = ora.im2col(C, H, W, k, k, p, p, s, s, d, d, x, batch=batch)
    if ref.size == 0:
        return
    dx = torch_cuda.from_numpy(x).cuda()
    dcol = torch_cuda.full(ref.shape, float("nan"), device="cuda")
    hip.im2colStridedBatched(C, H, W, k, k, p, p, s, s, d, d, dx, C * H * W, 0, dcol,
                             ref[0].size, 0, batch)
    hip.finish()
    assert dcol.cpu().numpy().tobytes() == ref.tobytes()


def test_im2col_single_with_offsets(hip, torch_cuda, ora):
    C, H, W, k, p, s, d = 3, 9, 9, 3, 1, 2, 1
    x = ora.uniform(7 + C * H * W, 3, 99)
    ref = ora.im2col(C, H, W, k, k, p, p, s, s, d, d, x[7:].copy())
    dx = torch_cuda.from_numpy(x).cuda()
    dcol = torch_cuda.zeros(5 + ref.size, device="cuda")
    hip.im2col(C, H, W, k, k, p, p, s, s, d, d, dx, 7, dcol, 5)
    hip.finish()
    assert dcol.cpu().numpy()[5:].tobytes() == ref.ravel().tobytes()


@pytest.mark.parametrize("geo", GEOS)
@pytest.mark.parametrize("batch", [1, 2])
def test_col2im_bit_exact(hip, torch_cuda, ora, geo, batch):
    C, H, W, k, p, s, d = geo
    oh = ora.out_dim(H, p, k, d, s)
    ow = ora.out_dim(W, p, k, d, s)
    if oh <= 0 or ow <= 0:
        return
    col = ora.uniform(batch * C * k * k * oh * ow, 4, sum(geo))
    base = ora.uniform(batch * C * H * W, 5, sum(geo))
    ref = ora.col2im(C, H, W, k, k, p, p, s, s, d, d, col.copy(), base.copy(), batch=batch)
    dcol = torch_cuda.from_numpy(col).cuda()
    dim = torch_cuda.from_numpy(base.copy()).cuda()
    hip.col2imStridedBatched(C, H, W, k, k, p, p, s, s, d, d, dcol, col.size // batch, 0, dim,
                             C * H * W, 0, batch)
    hip.finish()
    assert np.array_equal(dim.cpu().numpy(), ref)


def test_host_api_im2col_col2im(hiplib, torch_cuda, ora):
    from tensorium_amd.ntensors import bind_hip_op_table
    ops = bind_hip_op_table()
    C, H, W, k, p, s, d, batch = 3, 11, 10, 3, 1, 2, 1, 2
    x = ora.uniform(batch * C * H * W, 6, 0)
    ref = ora.im2col(C, H, W, k, k, p, p, s, s, d, d, x, batch=batch)
    col = np.zeros_like(ref)
    ops.im2colStridedBatchedvv(C, H, W, k, k, p, p, s, s, d, d, x.ctypes.data, C * H * W, 0,
                               col.ctypes.data, ref[0].size, 0, batch)
    assert hiplib.tns_last_error() == b""
    assert col.tobytes() == ref.tobytes()
    base = ora.uniform(C * H * W, 7, 0)
    im = base.copy()
    ops.col2imvv(C, H, W, k, k, p, p, s, s, d, d, ref[0].ctypes.data, 0, im.ctypes.data, 0, 1, 0)
    want = ora.col2im(C, H, W, k, k, p, p, s, s, d, d, ref[0].copy(), base.copy())
    assert np.array_equal(im, want)


def test_im2col_yolo_first_layer_full_size(hip, torch_cuda, ora):
    # BASELINE size: 8 x 3 x 416 x 416, k3 s1 p1 (col 27 x 173056 per image)
    batch, C, H = 8, 3, 416
    x = ora.uniform(batch * C * H * H, 3, 0, 0.0, 1.0)
    ref = ora.im2col(C, H, H, 3, 3, 1, 1, 1, 1, 1, 1, x, batch=batch)
    dx = torch_cuda.from_numpy(x).cuda()
    dcol = torch_cuda.empty(ref.shape, device="cuda")
    hip.im2colStridedBatched(C, H, H, 3, 3, 1, 1, 1, 1, 1, 1, dx, C * H * H, 0, dcol,
                             ref[0].size, 0, batch)
    hip.finish()
    assert dcol.cpu().numpy().tobytes() == ref.tobytes()
