"""Conv2D / conv-layer forward on the GPU vs the oracle (TTensor.Conv2D,
ntensors.pas:8252-8349; TConvolutionalLayer.forward, nConvolutionLayer.pas:
457-569).  Conv GEMMs are NN, so with bias add and leaky/linear/relu the whole
layer is bit-exact; YOLOv3 layers are checked per layer (teacher forcing:
each layer gets the oracle's input), batch 8 at full 416 resolution for a
layer subset, all 75 layers at batch 1."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def conv_case(hip, torch, ora, batch, C, H, F, k, s, p, act, fused, seed=0, dil=1):
    x = ora.uniform(batch * C * H * H, 3, seed, 0.0, 1.0).reshape(batch, C, H, H)
    sc = float(np.sqrt(2.0 / (k * k * C)))
    w = ora.uniform(F * C * k * k, 30 + seed, seed, -sc, sc)
    b = ora.uniform(F, 60 + seed, seed, -0.1, 0.1)
    ref = ora.conv_forward(x, w, b, F, k, s, p, act, dil) if dil != 1 else \
        ora.conv_forward(x, w, b, F, k, s, p, act)
    dx, dw, db = (torch.from_numpy(t).cuda() for t in (x, w, b))
    out = torch.full(ref.shape, float("nan"), device="cuda")
    hip.convForward(batch, C, H, H, dx, dw, db, F, k, s, p, dil, act, None, out, fused=fused)
    hip.finish()
    return out.cpu().numpy(), ref


@pytest.mark.parametrize("fused", [0, 1, 2, 3])
@pytest.mark.parametrize("batch,C,H,F,k,s,p,act", [
    (2, 3, 17, 8, 3, 1, 1, 9), (3, 5, 12, 7, 3, 2, 1, 9), (2, 16, 9, 5, 1, 1, 0, 4),
    (1, 4, 20, 33, 3, 2, 1, 1), (2, 3, 13, 6, 5, 1, 2, 0)])
def test_conv_forward_small(hip, torch_cuda, ora, fused, batch, C, H, F, k, s, p, act):
    got, ref = conv_case(hip, torch_cuda, ora, batch, C, H, F, k, s, p, act, fused)
    assert np.array_equal(got, ref)


def test_conv2d_driver_matches_oracle(hip, torch_cuda, ora):
    batch, C, H, F, k, s, p = 2, 6, 15, 9, 3, 2, 1
    x = ora.uniform(batch * C * H * H, 3, 77).reshape(batch, C, H, H)
    w = ora.uniform(F * C * k * k, 4, 77, -0.2, 0.2)
    ref = ora.conv2d(x, w, F, k, p, s)
    dx, dw = torch_cuda.from_numpy(x).cuda(), torch_cuda.from_numpy(w).cuda()
    out = torch_cuda.zeros(ref.shape, device="cuda")
    hip.conv2d(batch, C, H, H, dx, dw, F, k, k, p, p, s, s, 1, 1, None, out)
    hip.finish()
    assert np.array_equal(out.cpu().numpy(), ref)


def test_yolov3_all_layers_batch1_bit_exact(hip, torch_cuda, ora):
    from tensorium_amd.yolo import yolov3_conv_table
    for spec in yolov3_conv_table():
        got, ref = conv_case(hip, torch_cuda, ora, 1, spec.c, spec.h, spec.filters, spec.size,
                             spec.stride, spec.pad, spec.activation, True, seed=spec.index)
        assert np.array_equal(got, ref), spec


@pytest.mark.parametrize("idx", [0, 1, 2, 11, 62, 74])
def test_yolov3_layers_batch8_full_size(hip, torch_cuda, ora, idx):
    from tensorium_amd.yolo import yolov3_conv_table
    spec = yolov3_conv_table()[idx]
    got, ref = conv_case(hip, torch_cuda, ora, 8, spec.c, spec.h, spec.filters, spec.size,
                         spec.stride, spec.pad, spec.activation, True, seed=spec.index)
    assert np.array_equal(got, ref), spec


# implicit GEMM: every tile shape, ragged N (oh*ow not a multiple of BN),
# K = C*k*k not a multiple of 32, strides, padding, and filter counts
# straddling the tile rows
IMPLICIT_CASES = [
    (2, 3, 17, 8, 3, 1, 1, 9), (3, 5, 12, 70, 3, 2, 1, 9), (1, 7, 31, 129, 3, 1, 1, 9),
    (2, 13, 26, 40, 3, 2, 1, 1), (1, 2, 9, 300, 5, 1, 2, 4), (2, 33, 19, 64, 3, 1, 1, 9),
    (1, 64, 52, 128, 3, 1, 1, 9), (1, 32, 53, 256, 3, 2, 1, 9)]


CONV_VARIANTS = (1, 2, 4, 6, 12, 13, 14, 15, 18, 19, 20, 21, 22)  # with implicit-conv instances


@pytest.mark.parametrize("pad", [0, 1])
@pytest.mark.parametrize("variant", [-1, 0, 1, 2, 3, 4, 5, 6, 12, 13, 14, 15, 16, 18, 19, 20, 21,
                                     22])
def test_conv_implicit_variants_bit_exact(hip, torch_cuda, ora, variant, pad):
    """Every tile shape with an implicit-conv instantiation (others report
    UNSUPPORTED), both gather forms (padded copy / bounds-checked)."""
    from tensorium_amd._abi import TnsError
    hip.setConvVariant(variant)
    hip.setConvPad(pad)
    try:
        for i, case in enumerate(IMPLICIT_CASES):
            try:
                got, ref = conv_case(hip, torch_cuda, ora, *case, fused=3, seed=i)
            except TnsError:
                assert variant not in CONV_VARIANTS and variant >= 0, variant
                return
            assert np.array_equal(got, ref), (variant, pad, case)
    finally:
        hip.setConvVariant(-1)
        hip.setConvPad(-1)


@pytest.mark.parametrize("pad", [0, 1])
def test_conv_implicit_dilation(hip, torch_cuda, ora, pad):
    hip.setConvPad(pad)
    try:
        for i, (batch, C, H, F, k, s, p, d) in enumerate([(2, 4, 21, 12, 3, 1, 2, 2),
                                                          (1, 3, 30, 40, 3, 2, 2, 3)]):
            got, ref = conv_case(hip, torch_cuda, ora, batch, C, H, F, k, s, p, 9, 3, seed=i,
                                 dil=d)
            got2, _ = conv_case(hip, torch_cuda, ora, batch, C, H, F, k, s, p, 9, 2, seed=i,
                                dil=d)
            assert np.array_equal(got, ref)
            assert np.array_equal(got2, ref)
    finally:
        hip.setConvPad(-1)


# direct kernel (conv_direct.hip): 3-channel 3x3 layers with 16 or 32
# filters — ragged pixel counts, strides, paddings beyond the window,
# dilation, every activation form (logistic/tanh evaluated in the kernel)
DIRECT_CASES = [(2, 3, 17, 32, 3, 1, 1, 9, 1), (3, 3, 12, 16, 3, 2, 1, 0, 1),
                (1, 3, 30, 32, 3, 1, 2, 6, 2), (2, 3, 9, 16, 3, 1, 0, 1, 1),
                (1, 3, 40, 32, 3, 2, 0, 4, 1), (1, 3, 33, 32, 3, 1, 3, 13, 2)]


@pytest.mark.parametrize("fused", [1, 3])
@pytest.mark.parametrize("case", DIRECT_CASES)
def test_conv_direct_bit_exact(hip, torch_cuda, ora, fused, case):
    batch, C, H, F, k, s, p, act, dil = case
    got, ref = conv_case(hip, torch_cuda, ora, batch, C, H, F, k, s, p, act, fused, seed=5,
                         dil=dil)
    assert np.array_equal(got, ref), case


@pytest.mark.parametrize("idx", [0, 1, 2, 11, 62, 74])
def test_yolov3_layers_batch8_implicit(hip, torch_cuda, ora, idx):
    from tensorium_amd.yolo import yolov3_conv_table
    spec = yolov3_conv_table()[idx]
    got, ref = conv_case(hip, torch_cuda, ora, 8, spec.c, spec.h, spec.filters, spec.size,
                         spec.stride, spec.pad, spec.activation, 3, seed=spec.index)
    assert np.array_equal(got, ref), spec


@pytest.mark.parametrize("batch,C,H,F,k,s,p,act", [
    (2, 3, 17, 8, 3, 1, 1, 9), (3, 5, 12, 7, 3, 2, 1, 9), (2, 16, 9, 5, 1, 1, 0, 4),
    (2, 6, 13, 33, 3, 1, 1, 1), (1, 32, 26, 64, 3, 2, 1, 9), (10, 4, 9, 8, 3, 1, 1, 9)])
def test_conv_backward_matches_oracle(hip, torch_cuda, ora, batch, C, H, F, k, s, p, act):
    """delta (derived), state_delta (TN + col2im), weight_updates (NT in the
    reference's sdot order) and bias_updates (addSums order) bit-exact.  Batch
    10 takes the dW partials past one 8-image load group of add_in_order."""
    rng = np.random.default_rng(batch * 1000 + C * 10 + H)
    oh = (H + 2 * p - k) // s + 1
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.3, 0.3, F * C * k * k).astype(np.float32)
    out = rng.uniform(-1, 1, (batch, F, oh, oh)).astype(np.float32)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu0 = rng.uniform(-1, 1, F).astype(np.float32)
    wu0 = rng.uniform(-1, 1, F * C * k * k).astype(np.float32)
    sd0 = rng.uniform(-1, 1, x.shape).astype(np.float32)
    rd, rbu, rwu, rsd = d0.copy(), bu0.copy(), wu0.copy(), sd0.copy()
    ora.conv_backward(x, w, F, k, s, p, act, out, rd, rbu, rwu, rsd)
    t = lambda a: torch_cuda.from_numpy(a.copy()).cuda()  # noqa: E731
    dx, dw, dout, dd, dbu, dwu, dsd = map(t, (x, w, out, d0, bu0, wu0, sd0))
    hip.convBackward(batch, C, H, H, dx, dw, F, k, s, p, 1, act, dout, dd, dbu, dwu, None, dsd)
    hip.finish()
    assert np.array_equal(dd.cpu().numpy(), rd)
    assert np.array_equal(dsd.cpu().numpy(), rsd)
    assert np.array_equal(dwu.cpu().numpy(), rwu)
    assert np.array_equal(dbu.cpu().numpy(), rbu)


@pytest.mark.parametrize("idx", [0, 2, 11, 74])
def test_conv_backward_yolov3_batch8(hip, torch_cuda, ora, idx):
    """YOLOv3 layer shapes at batch 8: the dW partial sums of all images in
    one batched sdot launch, added to weight_updates in image order — bit-exact
    against the reference's per-image beta = 1 loop."""
    from tensorium_amd.yolo import yolov3_conv_table
    spec = yolov3_conv_table()[idx]
    batch, C, H, F, k, s, p = 8, spec.c, spec.h, spec.filters, spec.size, spec.stride, spec.pad
    rng = np.random.default_rng(idx)
    oh = (H + 2 * p - k) // s + 1
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.1, 0.1, F * C * k * k).astype(np.float32)
    out = rng.uniform(-1, 1, (batch, F, oh, oh)).astype(np.float32)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu0 = rng.uniform(-1, 1, F).astype(np.float32)
    wu0 = rng.uniform(-1, 1, F * C * k * k).astype(np.float32)
    rd, rbu, rwu = d0.copy(), bu0.copy(), wu0.copy()
    ora.conv_backward(x, w, F, k, s, p, spec.activation, out, rd, rbu, rwu, None)
    t = lambda a: torch_cuda.from_numpy(a.copy()).cuda()  # noqa: E731
    dx, dw, dout, dd, dbu, dwu = map(t, (x, w, out, d0, bu0, wu0))
    hip.convBackward(batch, C, H, H, dx, dw, F, k, s, p, 1, spec.activation, dout, dd, dbu, dwu)
    hip.finish()
    assert np.array_equal(dd.cpu().numpy(), rd)
    assert np.array_equal(dwu.cpu().numpy(), rwu)
    assert np.array_equal(dbu.cpu().numpy(), rbu)


DX_CASES = [(2, 64, 13, 64, 3, 1, 1, 9), (2, 128, 13, 64, 3, 1, 1, 1), (1, 128, 20, 128, 3, 2, 1, 9),
            (2, 64, 9, 128, 1, 1, 0, 4), (3, 64, 11, 96, 3, 1, 1, 9)]


def _dx_case(hip, torch, ora, batch, C, H, F, k, s, p, act, seed):
    rng = np.random.default_rng(seed)
    oh = (H + 2 * p - k) // s + 1
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.3, 0.3, F * C * k * k).astype(np.float32)
    out = rng.uniform(-1, 1, (batch, F, oh, oh)).astype(np.float32)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu0 = rng.uniform(-1, 1, F).astype(np.float32)
    wu0 = rng.uniform(-1, 1, F * C * k * k).astype(np.float32)
    sd0 = rng.uniform(-1, 1, x.shape).astype(np.float32)
    rd, rbu, rwu, rsd = d0.copy(), bu0.copy(), wu0.copy(), sd0.copy()
    ora.conv_backward(x, w, F, k, s, p, act, out, rd, rbu, rwu, rsd)
    t = lambda a: torch.from_numpy(a.copy()).cuda()  # noqa: E731
    dx, dw, dout, dd, dbu, dwu, dsd = map(t, (x, w, out, d0, bu0, wu0, sd0))
    hip.convBackward(batch, C, H, H, dx, dw, F, k, s, p, 1, act, dout, dd, dbu, dwu, None, dsd)
    hip.finish()
    return dsd.cpu().numpy(), rsd


def test_conv_backward_dx_tiles(hip, torch_cuda, ora):
    """Every k-major-A conv tile of the backward's col = W^T . delta
    (conv_tile4.hip, TNS_OPT_DX_TILE = v: all images in one launch, the delta
    planes as a 1x1 convolution's images) — state.delta bit-exact against
    the reference's TN GEMM + scol2im; forms whose tile does not divide the
    layer report UNSUPPORTED."""
    from tensorium_amd._abi import TnsError
    nv = hip.convDxTiles()
    assert nv >= 4
    ran = 0
    hip.setDxFused(0)
    try:
        for v in range(nv):
            hip.setDxTile(v)
            for i, case in enumerate(DX_CASES):
                try:
                    got, ref = _dx_case(hip, torch_cuda, ora, *case, seed=50 + i)
                except TnsError:
                    continue
                ran += 1
                assert np.array_equal(got, ref), (v, case)
    finally:
        hip.setDxTile(-1)
        hip.setDxFused(1)
    assert ran >= 2 * nv


DX3_CASES = [(2, 64, 13, 64, 3, 1, 1, 9), (2, 128, 11, 96, 3, 1, 1, 1), (3, 64, 9, 128, 3, 1, 0, 9),
             (1, 128, 20, 128, 3, 1, 1, 4), (2, 64, 6, 64, 3, 1, 2, 9), (2, 32, 15, 64, 3, 1, 1, 9)]


def test_conv_backward_dx_conv_forms(hip, torch_cuda, ora):
    """Every implicit transposed-convolution form of state.delta (conv_tile4
    DX, TNS_OPT_DX_CONV = v: each tap's filter chain from +0, added to the
    pixel at the tap's end in scol2im's order, out-of-window taps skipped) —
    bit-exact against the reference's TN GEMM + scol2im on stride-1 3x3
    layers with pads 0, 1 and 2 and ragged pixel counts; forms whose tiles do
    not divide C or F report UNSUPPORTED."""
    from tensorium_amd._abi import TnsError
    nv = hip.convDxConvs()
    assert nv >= 3
    ran = 0
    try:
        for v in range(nv):
            hip.setDxConv(v)
            for i, case in enumerate(DX3_CASES):
                try:
                    got, ref = _dx_case(hip, torch_cuda, ora, *case, seed=80 + i)
                except TnsError:
                    continue
                ran += 1
                assert np.array_equal(got, ref), (v, case)
    finally:
        hip.setDxConv(-1)
    assert ran >= 2 * nv


DX3S2_CASES = [(2, 64, 14, 64, 3, 2, 1, 9), (2, 32, 16, 64, 3, 2, 1, 1), (1, 64, 13, 128, 3, 2, 1, 9),
               (2, 64, 12, 64, 3, 2, 0, 9), (2, 128, 10, 128, 3, 2, 2, 4), (3, 32, 11, 128, 3, 2, 1, 9)]


def test_conv_backward_dx_conv_stride2_forms(hip, torch_cuda, ora):
    """state.delta of stride-2 3x3 layers as four implicit transposed
    convolutions, one per output pixel parity class (each over the taps
    col2im adds to that class, in (kr, kc) order; every DX form forced) —
    bit-exact against the reference's TN GEMM + scol2im: pads 0, 1, 2, odd
    and even planes (classes of unequal size), batch 1 .. 3."""
    from tensorium_amd._abi import TnsError
    nv = hip.convDxConvs()
    ran = 0
    try:
        for v in range(nv):
            hip.setDxConv(v)
            for i, case in enumerate(DX3S2_CASES):
                try:
                    got, ref = _dx_case(hip, torch_cuda, ora, *case, seed=120 + i)
                except TnsError:
                    continue
                ran += 1
                assert np.array_equal(got, ref), (v, case)
    finally:
        hip.setDxConv(-1)
    assert ran >= 2 * nv


@pytest.mark.parametrize("idx", [2, 28, 45])
def test_conv_backward_overlap_matches_sequential(hip, torch_cuda, ora, idx):
    """dW and state.delta on two streams (TNS_OPT_BWD_OVERLAP = 1, the
    default: state.delta's chain on the context's side stream with its own
    col buffer) against the sequential schedule and the oracle: delta,
    weight_updates, bias_updates and state.delta all identical (1x1 layer,
    3x3 layers whose dW reads an im2col matrix)."""
    from tensorium_amd.yolo import yolov3_conv_table
    spec = yolov3_conv_table()[idx]
    batch, C, H, F, k, s, p = 8, spec.c, spec.h, spec.filters, spec.size, spec.stride, spec.pad
    rng = np.random.default_rng(300 + idx)
    oh = (H + 2 * p - k) // s + 1
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.1, 0.1, F * C * k * k).astype(np.float32)
    out = rng.uniform(-1, 1, (batch, F, oh, oh)).astype(np.float32)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu0 = rng.uniform(-1, 1, F).astype(np.float32)
    wu0 = rng.uniform(-1, 1, F * C * k * k).astype(np.float32)
    sd0 = rng.uniform(-1, 1, x.shape).astype(np.float32)
    rd, rbu, rwu, rsd = d0.copy(), bu0.copy(), wu0.copy(), sd0.copy()
    ora.conv_backward(x, w, F, k, s, p, spec.activation, out, rd, rbu, rwu, rsd)
    t = lambda a: torch_cuda.from_numpy(a.copy()).cuda()  # noqa: E731
    got = []
    try:
        for mode in (True, False):
            hip.setBwdOverlap(mode)
            dx, dw, dout, dd, dbu, dwu, dsd = map(t, (x, w, out, d0, bu0, wu0, sd0))
            hip.convBackward(batch, C, H, H, dx, dw, F, k, s, p, 1, spec.activation, dout, dd, dbu,
                             dwu, None, dsd)
            hip.finish()
            got.append([a.cpu().numpy() for a in (dd, dbu, dwu, dsd)])
    finally:
        hip.setBwdOverlap(True)
    for g in got:
        for a, r in zip(g, (rd, rbu, rwu, rsd)):
            assert np.array_equal(a, r)


@pytest.mark.parametrize("idx", [10, 28, 45])
def test_conv_backward_derive_sums_fused(hip, torch_cuda, ora, idx):
    """TNS_OPT_DERIVE_SUMS = 1 (Derivative fused into addSums' chain pass,
    each derived term written back as it is staged): delta, bias_updates,
    weight_updates and state.delta bit-exact against the oracle."""
    from tensorium_amd.yolo import yolov3_conv_table
    spec = yolov3_conv_table()[idx]
    batch, C, H, F, k, s, p = 8, spec.c, spec.h, spec.filters, spec.size, spec.stride, spec.pad
    rng = np.random.default_rng(500 + idx)
    oh = (H + 2 * p - k) // s + 1
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.1, 0.1, F * C * k * k).astype(np.float32)
    out = rng.uniform(-1, 1, (batch, F, oh, oh)).astype(np.float32)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu0 = rng.uniform(-1, 1, F).astype(np.float32)
    wu0 = rng.uniform(-1, 1, F * C * k * k).astype(np.float32)
    sd0 = rng.uniform(-1, 1, x.shape).astype(np.float32)
    rd, rbu, rwu, rsd = d0.copy(), bu0.copy(), wu0.copy(), sd0.copy()
    ora.conv_backward(x, w, F, k, s, p, spec.activation, out, rd, rbu, rwu, rsd)
    t = lambda a: torch_cuda.from_numpy(a.copy()).cuda()  # noqa: E731
    dx, dw, dout, dd, dbu, dwu, dsd = map(t, (x, w, out, d0, bu0, wu0, sd0))
    try:
        hip.setDeriveSums(True)
        hip.convBackward(batch, C, H, H, dx, dw, F, k, s, p, 1, spec.activation, dout, dd, dbu,
                         dwu, None, dsd)
        hip.finish()
    finally:
        hip.setDeriveSums(False)
    for a, r in zip((dd, dbu, dwu, dsd), (rd, rbu, rwu, rsd)):
        assert np.array_equal(a.cpu().numpy(), r)


def test_conv_backward_pipelined_chain(hip, torch_cuda):
    """TNS_OPT_BWD_OVERLAP = 2 over a chain of YOLOv3 layers (43 .. 46, run
    in backward order, each layer's state.delta the delta of the layer below
    and its input that layer's output), two passes: every call's dW is left
    running on the side stream while the next calls' derive / bias sums /
    state.delta work proceeds, and pass 2's derivative of a layer waits for
    pass 1's dW that still reads that delta; every delta, bias / weight
    update and the chain's state.delta bit-identical to the sequential
    schedule (0)."""
    from tensorium_amd.yolo import yolov3_conv_table
    specs = [yolov3_conv_table()[i] for i in (43, 44, 45, 46)]
    B = 8
    rng = np.random.default_rng(4346)
    x0 = rng.uniform(0, 1, (B, specs[0].c, specs[0].h, specs[0].h)).astype(np.float32)
    outs = [rng.uniform(-1, 1, (B, s.filters, s.out_h, s.out_h)).astype(np.float32) for s in specs]
    deltas = [rng.uniform(-1, 1, o.shape).astype(np.float32) for o in outs]
    sd0 = np.zeros_like(x0)
    ws = [rng.uniform(-0.1, 0.1, (s.filters, s.K)).astype(np.float32) for s in specs]
    t = lambda a: torch_cuda.from_numpy(a.copy()).cuda()  # noqa: E731
    got = {}
    try:
        for mode in (0, 2):
            hip.setBwdOverlap(mode)
            X, O, D, W = t(x0), [t(o) for o in outs], [t(d) for d in deltas], [t(w) for w in ws]
            SD = t(sd0)
            BU = [torch_cuda.zeros(s.filters, device="cuda") for s in specs]
            WU = [torch_cuda.zeros(s.filters, s.K, device="cuda") for s in specs]
            for _ in range(2):  # (pass 2 rewrites the deltas pass 1's dW products read)
                for j in range(len(specs) - 1, -1, -1):
                    s = specs[j]
                    inp = X if j == 0 else O[j - 1]
                    sd = SD if j == 0 else D[j - 1]
                    hip.convBackward(B, s.c, s.h, s.h, inp, W[j], s.filters, s.size, s.stride,
                                     s.pad, 1, s.activation, O[j], D[j], BU[j], WU[j], None, sd)
            hip.finish()
            got[mode] = [a.cpu().numpy() for a in D + BU + WU + [SD]]
    finally:
        hip.setBwdOverlap(True)
    for a, b in zip(got[0], got[2]):
        assert np.array_equal(a, b)


def _residual_block_case(seed):
    """YOLOv3 layers 9, 10, 11 and the shortcut that adds layer 11's output
    to layer 9's (a darknet residual block at 52^2, batch 8): inputs,
    outputs, deltas, weights and the layers' update buffers."""
    from tensorium_amd.yolo import yolov3_conv_table
    specs = [yolov3_conv_table()[i] for i in (9, 10, 11)]
    B = 8
    rng = np.random.default_rng(seed)
    x0 = rng.uniform(0, 1, (B, specs[0].c, specs[0].h, specs[0].h)).astype(np.float32)
    outs = [rng.uniform(-1, 1, (B, s.filters, s.out_h, s.out_h)).astype(np.float32) for s in specs]
    deltas = [rng.uniform(-1, 1, o.shape).astype(np.float32) for o in outs]
    d_sc = rng.uniform(-1, 1, outs[2].shape).astype(np.float32)   # the shortcut layer's delta
    ws = [rng.uniform(-0.1, 0.1, (s.filters, s.K)).astype(np.float32) for s in specs]
    bs = [rng.uniform(-0.1, 0.1, s.filters).astype(np.float32) for s in specs]
    wus = [rng.uniform(-1, 1, w.shape).astype(np.float32) for w in ws]
    bus = [rng.uniform(-1, 1, s.filters).astype(np.float32) for s in specs]
    return specs, B, x0, outs, deltas, d_sc, ws, bs, wus, bus


def _residual_block_oracle(ora, specs, x0, outs, deltas, d_sc, ws, bs, wus, bus, lr, B, decay, mom):
    D, W, Bi, WU, BU = ([a.copy() for a in arr] for arr in (deltas, ws, bs, wus, bus))
    # TNet.backward (nnet.pas:332-366), i = 3 .. 0: the shortcut (TAddLayer,
    # linear: its delta added to layer 11's and to layer 9's, naddlayer.pas)
    D[2] += d_sc
    D[0] += d_sc
    inputs = [x0, outs[0], outs[1]]
    for j in (2, 1, 0):
        s = specs[j]
        ora.conv_backward(inputs[j], W[j].ravel(), s.filters, s.size, s.stride, s.pad, s.activation,
                          outs[j], D[j], BU[j], WU[j].ravel(), D[j - 1] if j else None)
    # TNet.update: every layer's TConvolutionalLayer.update, fused
    f32 = np.float32
    lrb = f32(f32(lr) / f32(B))
    ndb = f32(-f32(decay) * f32(B))
    for j in range(3):
        wflat, wuflat = W[j].reshape(-1), WU[j].reshape(-1)
        ora.sgd_update(wflat, wuflat, Bi[j], BU[j], None, None, float(lrb), float(ndb), mom)
    return D, W, Bi, WU, BU


@pytest.mark.parametrize("pipelined", [True, False])
def test_tnet_backward_order_through_tnnhip(hip, torch_cuda, ora, pipelined):
    """TNet.backward's loop (nnet.pas:332-366) replayed through TNNHip over a
    darknet residual block (YOLOv3 layers 9, 10, 11 + the shortcut) at batch
    8: the shortcut's backward (two addvv calls — a non-conv TNNHip call
    between the conv backward calls) first, then the conv layers from the top
    down, each taking the layer below's delta as state.delta (layer 9, the
    first, none), then TNet.update's sgdUpdate per layer — on the pipelined
    schedule initHIP selects (each conv layer's dW left on the side stream)
    and on the joined one; every delta, weight, bias and update bit-exact
    against the oracle's restated sequence."""
    specs, B, x0, outs, deltas, d_sc, ws, bs, wus, bus = _residual_block_case(911)
    lr, decay, mom = 1e-3, 5e-4, 0.9
    rD, rW, rB, rWU, rBU = _residual_block_oracle(ora, specs, x0, outs, deltas, d_sc, ws, bs, wus,
                                                  bus, lr, B, decay, mom)
    t = lambda a: torch_cuda.from_numpy(a.copy()).cuda()  # noqa: E731
    X, O, D, W = t(x0), [t(o) for o in outs], [t(d) for d in deltas], [t(w) for w in ws]
    Bi, WU, BU, DSC = [t(b) for b in bs], [t(w) for w in wus], [t(b) for b in bus], t(d_sc)
    try:
        hip.setBwdOverlap(2 if pipelined else 1)
        n = DSC.numel()
        hip.addvv(n, D[2], 0, 1, DSC, 0, 1, D[2], 0, 1)
        hip.addvv(n, D[0], 0, 1, DSC, 0, 1, D[0], 0, 1)
        inputs = [X, O[0], O[1]]
        for j in (2, 1, 0):
            s = specs[j]
            hip.convBackward(B, s.c, s.h, s.h, inputs[j], W[j], s.filters, s.size, s.stride, s.pad, 1,
                             s.activation, O[j], D[j], BU[j], WU[j], None, D[j - 1] if j else None)
        for j in range(3):
            hip.sgdUpdate(W[j], WU[j], Bi[j], BU[j], lr, B, decay, mom)
        hip.finish()
    finally:
        hip.setBwdOverlap(True)
    for got, ref in ((D, rD), (W, rW), (Bi, rB), (WU, rWU), (BU, rBU)):
        for g, r in zip(got, ref):
            assert np.array_equal(g.cpu().numpy(), r)


def test_pipelined_backward_get_stream_joins(hip, torch_cuda, ora):
    """A pipelined pass (TNS_OPT_BWD_OVERLAP = 2) leaves the dW products on
    the side stream; tns_hip_get_stream joins them before handing out the
    context's stream, so a torch read of weight_updates enqueued
    on that stream right after the pass — no finish — sees the finished sums."""
    specs, B, x0, outs, deltas, d_sc, ws, bs, wus, bus = _residual_block_case(912)
    rD, rWU, rBU = [d.copy() for d in deltas], [w.copy() for w in wus], [b.copy() for b in bus]
    inputs = [x0, outs[0], outs[1]]
    for j in (2, 1, 0):
        s = specs[j]
        ora.conv_backward(inputs[j], ws[j].ravel(), s.filters, s.size, s.stride, s.pad,
                          s.activation, outs[j], rD[j], rBU[j], rWU[j].ravel(),
                          rD[j - 1] if j else None)
    t = lambda a: torch_cuda.from_numpy(a.copy()).cuda()  # noqa: E731
    X, O, D, W = t(x0), [t(o) for o in outs], [t(d) for d in deltas], [t(w) for w in ws]
    WU, BU = [t(w) for w in wus], [t(b) for b in bus]
    try:
        hip.setBwdOverlap(2)
        hip.finish()
        ins = [X, O[0], O[1]]
        for j in (2, 1, 0):
            s = specs[j]
            hip.convBackward(B, s.c, s.h, s.h, ins[j], W[j], s.filters, s.size, s.stride, s.pad, 1,
                             s.activation, O[j], D[j], BU[j], WU[j], None, D[j - 1] if j else None)
        stream = torch_cuda.cuda.ExternalStream(hip.stream)   # (joins the pending dW)
        with torch_cuda.cuda.stream(stream):
            snap = [w.clone() for w in WU]
        stream.synchronize()
    finally:
        hip.setBwdOverlap(True)
    for g, r in zip(snap, rWU):
        assert np.array_equal(g.cpu().numpy(), r)


@pytest.mark.parametrize("idx", [3, 4, 9, 10, 11, 27, 28, 44, 45, 58])
def test_conv_backward_dx_yolov3_batch8(hip, torch_cuda, ora, idx):
    """state.delta at YOLOv3 layer shapes, batch 8, on the default path (the
    k-major-A conv tile where one applies, the parity-class transposed
    convolutions on the stride-2 layers 4 and 9; on the 1x1 layers 10, 27, 44, 58
    the product adds into state.delta in its epilogue, col2im's one add per
    pixel): bit-exact."""
    from tensorium_amd.yolo import yolov3_conv_table
    spec = yolov3_conv_table()[idx]
    got, ref = _dx_case(hip, torch_cuda, ora, 8, spec.c, spec.h, spec.filters, spec.size,
                        spec.stride, spec.pad, spec.activation, seed=idx)
    assert np.array_equal(got, ref)


DW_CASES = [(2, 64, 13, 64, 3, 1, 1, 9), (3, 128, 9, 64, 1, 1, 0, 4), (1, 64, 17, 128, 3, 1, 1, 1),
            (2, 16, 20, 64, 3, 2, 1, 9), (2, 128, 11, 128, 3, 1, 1, 9), (9, 64, 12, 64, 3, 1, 1, 9)]


def _dw_case(hip, torch, ora, batch, C, H, F, k, s, p, act, seed, dil=1, state_delta=False,
             workspace=False):
    rng = np.random.default_rng(seed)
    oh = ora.out_dim(H, p * dil, k, dil, s)
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.3, 0.3, F * C * k * k).astype(np.float32)
    out = rng.uniform(-1, 1, (batch, F, oh, oh)).astype(np.float32)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu0 = rng.uniform(-1, 1, F).astype(np.float32)
    wu0 = rng.uniform(-1, 1, F * C * k * k).astype(np.float32)
    rd, rbu, rwu = d0.copy(), bu0.copy(), wu0.copy()
    sd0 = rng.uniform(-1, 1, x.shape).astype(np.float32) if state_delta else None
    rsd = sd0.copy() if state_delta else None
    ora.conv_backward(x, w, F, k, s, p, act, out, rd, rbu, rwu, rsd, dil=dil)
    t = lambda a: torch.from_numpy(a.copy()).cuda()  # noqa: E731
    dx, dw, dout, dd, dbu, dwu = map(t, (x, w, out, d0, bu0, wu0))
    dsd = t(sd0) if state_delta else None
    ws = torch.zeros(batch * C * k * k * oh * oh, device="cuda") if workspace else None
    hip.convBackward(batch, C, H, H, dx, dw, F, k, s, p, dil, act, dout, dd, dbu, dwu, ws, dsd)
    hip.finish()
    if state_delta:
        assert np.array_equal(dsd.cpu().numpy(), rsd), "state_delta"
        assert np.array_equal(dbu.cpu().numpy(), rbu), "bias_updates"
    return dwu.cpu().numpy(), rwu


def test_conv_backward_dw_tiles(hip, torch_cuda, ora):
    """Every implicit-im2col dW tile (dw_tile.hip, TNS_OPT_DW_TILE = v: the
    im2col rows generated in the staging of the sdot-order product, all
    images in one launch, added in image order): weight_updates bit-exact
    against the reference's per-image im2col + beta = 1 sdot loop; 1x1 and
    3x3, stride 2, pixel counts off the 64-pixel tile and odd (scalar delta
    loads), batch 9; tiles that do not divide the layer report UNSUPPORTED."""
    from tensorium_amd._abi import TnsError
    nv = hip.convDwTiles()
    assert nv >= 3
    ran = 0
    try:
        for v in range(nv):
            hip.setDwTile(v)
            for i, case in enumerate(DW_CASES):
                try:
                    got, ref = _dw_case(hip, torch_cuda, ora, *case, seed=70 + i)
                except TnsError:
                    continue
                ran += 1
                assert np.array_equal(got, ref), (v, case)
    finally:
        hip.setDwTile(-1)
    assert ran >= 2 * nv


DWR_CASES = [(3, 128, 11, 128, 3, 1, 1, 9), (2, 64, 13, 64, 3, 1, 1, 9), (2, 64, 20, 128, 3, 2, 1, 1),
             (1, 128, 26, 256, 3, 1, 1, 9), (2, 64, 9, 64, 1, 1, 0, 4), (9, 64, 12, 64, 3, 1, 1, 9),
             (2, 128, 10, 128, 3, 1, 1, 9, 2), (1, 32, 48, 64, 3, 1, 1, 9), (2, 3, 20, 64, 3, 1, 1, 1),
             (1, 16, 72, 64, 3, 1, 1, 9), (2, 16, 144, 64, 3, 2, 1, 1), (1, 64, 20, 64, 3, 1, 1, 9),
             (1, 64, 30, 64, 3, 1, 1, 1)]


def test_conv_backward_dw_res_forms(hip, torch_cuda, ora):
    """Every residue-sequential dW form (dw_res.hip, TNS_OPT_DW_RES = v: the
    sdot order's eight residue chains run one after another per output tile
    over residue-major copies of delta and the im2col matrix, folded in sdot's
    order, images added in order): weight_updates (and state.delta, bias)
    bit-exact against the reference's per-image im2col + beta = 1 sdot loop;
    k = 100 .. 5184 pixels (chains of 13 .. 648 terms: ragged last k-tiles;
    the col' rows in one or two input bands), stride 2, dilation 2, a 1x1 layer (the input planes rearranged), batch 9,
    col rows off the column tile (N = 27, 288, 576: padded rows); forms whose
    row tile does not divide the filters report UNSUPPORTED."""
    from tensorium_amd._abi import TnsError
    nv = hip.convDwRes()
    assert nv >= 4
    ran = 0
    try:
        for v in range(nv):
            hip.setDwRes(v)
            for i, case in enumerate(DWR_CASES):
                dil = case[8] if len(case) > 8 else 1
                try:
                    got, ref = _dw_case(hip, torch_cuda, ora, *case[:8], seed=90 + i, dil=dil,
                                        state_delta=i % 2 == 0)
                except TnsError:
                    continue
                ran += 1
                assert np.array_equal(got, ref), (v, case)
    finally:
        hip.setDwRes(-1)
    assert ran >= 2 * nv


@pytest.mark.parametrize("dil", [1, 2])
def test_conv_backward_dw_auto_pick_dilated(hip, torch_cuda, ora, dil):
    """The shape dw_tile_pick selects by default (3x3, 256 filters over 128
    channels, batch 8) with dilation 2 (same padding, pad*dil geometry,
    nConvolutionLayer.pas:640) as well as 1: dW, bias and state.delta
    bit-exact on the automatic choice and on im2col + sdot."""
    try:
        for form in (-1, -2):
            hip.setDwTile(form)
            got, ref = _dw_case(hip, torch_cuda, ora, 8, 128, 14, 256, 3, 1, 1, 9, seed=91,
                                dil=dil, state_delta=True)
            assert np.array_equal(got, ref), form
    finally:
        hip.setDwTile(-1)


@pytest.mark.parametrize("overlap", [1, 0])
def test_conv_backward_caller_workspace(hip, torch_cuda, ora, overlap):
    """A caller-supplied workspace (batch * C*k*k * oH*oW floats, tns.h) with
    the dW/state.delta overlap on and off: the same bits either way."""
    try:
        hip.setBwdOverlap(bool(overlap))
        hip.setDwTile(-2)   # dW reads an im2col matrix: both chains need a col buffer
        got, ref = _dw_case(hip, torch_cuda, ora, 4, 32, 19, 64, 3, 1, 1, 9, seed=93,
                            state_delta=True, workspace=True)
        assert np.array_equal(got, ref)
    finally:
        hip.setBwdOverlap(True)
        hip.setDwTile(-1)


@pytest.mark.parametrize("idx", [1, 11, 28, 44, 45, 58])
def test_conv_backward_dw_rc_forms(hip, torch_cuda, ora, idx):
    """Every residue-register form of the dW product (sgemm_sdot_rc.hip,
    TNS_OPT_SDOT_FORM = 64 + v; per-image sums added in image order after
    the launch) gives the reference's per-image beta = 1 sdot loop bit for
    bit — 13^2 (K = 169 per image: unaligned rows, ragged k-tile), 255
    filters, 1x1 and stride-2 layers."""
    from tensorium_amd.yolo import yolov3_conv_table
    spec = yolov3_conv_table()[idx]
    batch, C, H, F, k, s, p = 8, spec.c, spec.h, spec.filters, spec.size, spec.stride, spec.pad
    rng = np.random.default_rng(100 + idx)
    oh = (H + 2 * p - k) // s + 1
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.1, 0.1, F * C * k * k).astype(np.float32)
    out = rng.uniform(-1, 1, (batch, F, oh, oh)).astype(np.float32)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu0 = rng.uniform(-1, 1, F).astype(np.float32)
    wu0 = rng.uniform(-1, 1, F * C * k * k).astype(np.float32)
    rd, rbu, rwu = d0.copy(), bu0.copy(), wu0.copy()
    ora.conv_backward(x, w, F, k, s, p, spec.activation, out, rd, rbu, rwu, None)
    t = lambda a: torch_cuda.from_numpy(a.copy()).cuda()  # noqa: E731
    dx, dw, dout = map(t, (x, w, out))
    try:
        for v in range(hip.sdotRcVariants()):
            hip.setSdotForm(64 + v)
            dd, dbu, dwu = map(t, (d0, bu0, wu0))
            hip.convBackward(batch, C, H, H, dx, dw, F, k, s, p, 1, spec.activation, dout, dd,
                             dbu, dwu)
            hip.finish()
            got = dwu.cpu().numpy()
            assert np.array_equal(got, rwu), (v, float(np.abs(got - rwu).max()))
            assert np.array_equal(dd.cpu().numpy(), rd)
    finally:
        hip.setSdotForm(-1)


@pytest.mark.parametrize("fused", [2, 0])
@pytest.mark.parametrize("batch,C,H,F,k,s,p,act", [
    (2, 8, 17, 12, 3, 1, 1, 9), (3, 64, 13, 100, 3, 1, 1, 1), (2, 68, 9, 40, 1, 1, 0, 4),
    (1, 32, 20, 16, 5, 1, 2, 9), (2, 16, 11, 24, 3, 1, 0, 9), (1, 132, 7, 65, 3, 1, 1, 0),
    (8, 512, 13, 1024, 3, 1, 1, 9), (8, 128, 52, 256, 3, 1, 1, 9), (8, 32, 208, 64, 3, 1, 1, 9)])
def test_conv_backward_state_delta_fused(hip, torch_cuda, ora, fused, batch, C, H, F, k, s, p,
                                         act):
    """state.delta of stride-1 layers: one kernel running each window tap's
    filter chain and adding it to the pixel in scol2im's order (no col
    matrix) and the reference's TN GEMM + col2im — both bit-exact: ragged
    channel / filter / pixel tiles, 1x1, 5x5, padding 0 (taps skipped at
    the border), YOLOv3 13x13 and 52x52 shapes at batch 8."""
    rng = np.random.default_rng(C * 7 + F + H)
    oh = (H + 2 * p - k) // s + 1
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.3, 0.3, F * C * k * k).astype(np.float32)
    out = rng.uniform(-1, 1, (batch, F, oh, oh)).astype(np.float32)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu0 = rng.uniform(-1, 1, F).astype(np.float32)
    wu0 = rng.uniform(-1, 1, F * C * k * k).astype(np.float32)
    sd0 = rng.uniform(-1, 1, x.shape).astype(np.float32)
    sd0[0, 0, 0, :2] = -0.0  # a pixel whose every skipped tap must stay skipped
    rd, rbu, rwu, rsd = d0.copy(), bu0.copy(), wu0.copy(), sd0.copy()
    ora.conv_backward(x, w, F, k, s, p, act, out, rd, rbu, rwu, rsd)
    t = lambda a: torch_cuda.from_numpy(a.copy()).cuda()  # noqa: E731
    dx, dw, dout, dd, dbu, dwu, dsd = map(t, (x, w, out, d0, bu0, wu0, sd0))
    hip.setDxFused(fused)
    try:
        hip.convBackward(batch, C, H, H, dx, dw, F, k, s, p, 1, act, dout, dd, dbu, dwu, None,
                         dsd)
        hip.finish()
    finally:
        hip.setDxFused(1)
    assert np.array_equal(dsd.cpu().numpy(), rsd)
    assert np.array_equal(dwu.cpu().numpy(), rwu)
    assert np.array_equal(dd.cpu().numpy(), rd)


def _t(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).copy()).cuda()


BN_CASES = [(2, 3, 17, 8, 3, 1, 1, 9, 1), (3, 5, 12, 7, 3, 2, 1, 9, 1), (2, 16, 9, 5, 1, 1, 0, 4, 1),
            (2, 6, 13, 33, 3, 1, 1, 0, 1), (2, 4, 15, 6, 3, 1, 1, 9, 2),
            # 65^2 = 4225-pixel planes: the 256-thread chain form with a tail;
            # 129^2 = 16641: the specialised-wave form with a tail
            (1, 2, 65, 3, 3, 1, 1, 9, 1), (1, 1, 129, 2, 3, 1, 1, 9, 1),
            # the fused batchNormBack's edges: 16^2 = 256 pixels (the first
            # plane past the short-plane finish), 127^2 = 16129 (the largest
            # fused plane), 128^2 = 16384 (the first on the separate passes)
            (2, 3, 16, 5, 3, 1, 1, 9, 1), (1, 1, 127, 2, 3, 1, 1, 9, 1),
            (1, 1, 128, 2, 3, 1, 1, 9, 1)]


@pytest.mark.parametrize("quirk", [0, 1])
@pytest.mark.parametrize("batch,C,H,F,k,s,p,act,dil", BN_CASES)
def test_conv_train_batchnorm_forward_backward(hip, torch_cuda, ora, batch, C, H, F, k, s, p, act,
                                               dil, quirk):
    """TConvolutionalLayer.forward (training, batch norm) and .backward with
    batchNormBack, bit-exact: output, x, x_norm, mean, variance, rolling
    statistics; delta, scale_updates, mean/variance_delta, weight_updates,
    state_delta — with and without the srss / sVarinceDelta lane drop."""
    T = torch_cuda
    rng = np.random.default_rng(batch * 7 + C + H + dil)
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.3, 0.3, F * C * k * k).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, F).astype(np.float32)
    b = rng.uniform(-0.2, 0.2, F).astype(np.float32)
    rm, rv = rng.uniform(-0.1, 0.1, F).astype(np.float32), rng.uniform(0.5, 2, F).astype(np.float32)
    R = [a.copy() for a in (rm, rv)]
    out, m, v, xs, xn = ora.conv_forward_train(x, w, F, k, s, p, act, sc, b, R[0], R[1], 0.1,
                                               True, dil=dil, quirk=quirk)
    dx, dw, dsc, db, drm, drv = (_t(T, a) for a in (x, w, sc, b, rm, rv))
    g = {n: T.zeros(a.shape, device="cuda") for n, a in
         (("out", out), ("m", m), ("v", v), ("xs", xs), ("xn", xn))}
    hip.setSrssQuirk(bool(quirk))
    try:
        hip.convForwardTrain(batch, C, H, H, dx, dw, F, k, s, p, dil, act, dsc, db, drm, drv, 0.1,
                             True, g["m"], g["v"], g["xs"], g["xn"], None, g["out"])
        hip.finish()
        for n, r in (("out", out), ("m", m), ("v", v), ("xs", xs), ("xn", xn)):
            assert np.array_equal(g[n].cpu().numpy(), r), n
        assert np.array_equal(drm.cpu().numpy(), R[0]) and np.array_equal(drv.cpu().numpy(), R[1])
        # backward with batchNormBack: its geometry is the layer's outH (no
        # dilation, nConvolutionLayer.pas:92-100), which differs from the
        # dilated forward's rows — the reference's dilated layer cannot run
        # forward and backward on one tensor, so that case stops here
        if ora.lib().ora_conv_backward_oh(H, k, s, p, dil) != out.shape[2]:
            return
        d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
        su0 = rng.uniform(-1, 1, F).astype(np.float32)
        wu0 = rng.uniform(-1, 1, w.size).astype(np.float32)
        sd0 = rng.uniform(-1, 1, x.shape).astype(np.float32)
        rd, rsu, rwu, rsd = d0.copy(), su0.copy(), wu0.copy(), sd0.copy()
        md, vd = ora.conv_backward_bn(x, w, F, k, s, p, act, out, rd, sc, xs, xn, m, v, rsu, rwu,
                                      rsd, dil=dil, quirk=quirk)
        dd, dsu, dwu, dsd = (_t(T, a) for a in (d0, su0, wu0, sd0))
        dmd, dvd = T.zeros(F, device="cuda"), T.zeros(F, device="cuda")
        hip.convBackwardBN(batch, C, H, H, dx, dw, F, k, s, p, dil, act, _t(T, out), dd, dsc,
                           _t(T, xs), _t(T, xn), _t(T, m), _t(T, v), dsu, dmd, dvd, dwu, None, dsd)
        hip.finish()
    finally:
        hip.setSrssQuirk(False)
    for n, gg, r in (("delta", dd, rd), ("scale_updates", dsu, rsu), ("mean_delta", dmd, md),
                     ("variance_delta", dvd, vd), ("weight_updates", dwu, rwu),
                     ("state_delta", dsd, rsd)):
        assert np.array_equal(gg.cpu().numpy(), r), n


@pytest.mark.parametrize("idx", [0, 1, 2, 11, 62, 74])
def test_conv_train_batchnorm_yolov3_batch8(hip, torch_cuda, ora, idx):
    """YOLOv3 shapes at batch 8 / 416 px: the training forward with batch norm
    (inference mode too) and the backward with batchNormBack, bit-exact."""
    from tensorium_amd.yolo import yolov3_conv_table
    T = torch_cuda
    spec = yolov3_conv_table()[idx]
    batch, C, H, F, k, s, p, act = 8, spec.c, spec.h, spec.filters, spec.size, spec.stride, \
        spec.pad, spec.activation
    x = ora.uniform(batch * C * H * H, 3, idx, 0.0, 1.0).reshape(batch, C, H, H)
    scl = float(np.sqrt(2.0 / (k * k * C)))
    w = ora.uniform(F * C * k * k, 30 + idx, idx, -scl, scl)
    sc, b = ora.uniform(F, 70, idx, 0.5, 1.5), ora.uniform(F, 71, idx, -0.1, 0.1)
    rm, rv = np.zeros(F, np.float32), np.ones(F, np.float32)
    R = [rm.copy(), rv.copy()]
    out, m, v, xs, xn = ora.conv_forward_train(x, w, F, k, s, p, act, sc, b, R[0], R[1], 0.1, True)
    dx, dw, dsc, db, drm, drv = (_t(T, a) for a in (x, w, sc, b, rm, rv))
    g = {n: T.zeros(a.shape, device="cuda") for n, a in
         (("out", out), ("m", m), ("v", v), ("xs", xs), ("xn", xn))}
    hip.convForwardTrain(batch, C, H, H, dx, dw, F, k, s, p, 1, act, dsc, db, drm, drv, 0.1, True,
                         g["m"], g["v"], g["xs"], g["xn"], None, g["out"])
    hip.finish()
    for n, r in (("out", out), ("m", m), ("v", v), ("xs", xs), ("xn", xn)):
        assert np.array_equal(g[n].cpu().numpy(), r), n
    assert np.array_equal(drm.cpu().numpy(), R[0]) and np.array_equal(drv.cpu().numpy(), R[1])
    # inference mode: rolling statistics
    inf, *_ = ora.conv_forward_train(x, w, F, k, s, p, act, sc, b, R[0].copy(), R[1].copy(), 0.1,
                                     False)
    gi = T.zeros(out.shape, device="cuda")
    hip.convForwardTrain(batch, C, H, H, dx, dw, F, k, s, p, 1, act, dsc, db, drm, drv, 0.1,
                         False, None, None, None, None, None, gi)
    hip.finish()
    assert np.array_equal(gi.cpu().numpy(), inf)
    rng = np.random.default_rng(idx)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    su0 = np.zeros(F, np.float32)
    wu0 = np.zeros(w.size, np.float32)
    rd, rsu, rwu = d0.copy(), su0.copy(), wu0.copy()
    md, vd = ora.conv_backward_bn(x, w, F, k, s, p, act, out, rd, sc, xs, xn, m, v, rsu, rwu)
    dd, dsu, dwu = (_t(T, a) for a in (d0, su0, wu0))
    dmd, dvd = T.zeros(F, device="cuda"), T.zeros(F, device="cuda")
    hip.convBackwardBN(batch, C, H, H, dx, dw, F, k, s, p, 1, act, _t(T, out), dd, dsc, _t(T, xs),
                       _t(T, xn), _t(T, m), _t(T, v), dsu, dmd, dvd, dwu)
    hip.finish()
    for n, gg, r in (("delta", dd, rd), ("scale_updates", dsu, rsu), ("mean_delta", dmd, md),
                     ("variance_delta", dvd, vd), ("weight_updates", dwu, rwu)):
        assert np.array_equal(gg.cpu().numpy(), r), n


def test_conv_backward_dilation_same_padding(hip, torch_cuda, ora):
    """Dilation 2 with k=3, p=1: the backward's padding*dilation im2col gives
    the layer's outH columns; bit-exact incl. col2im's dilation formula."""
    T = torch_cuda
    rng = np.random.default_rng(21)
    batch, C, H, F, k, s, p, d = 2, 3, 14, 5, 3, 1, 1, 2
    x = rng.uniform(-1, 1, (batch, C, H, H)).astype(np.float32)
    w = rng.uniform(-0.3, 0.3, F * C * k * k).astype(np.float32)
    out = rng.uniform(-1, 1, (batch, F, H, H)).astype(np.float32)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu0, wu0 = rng.uniform(-1, 1, F).astype(np.float32), rng.uniform(-1, 1, w.size).astype(np.float32)
    sd0 = rng.uniform(-1, 1, x.shape).astype(np.float32)
    rd, rbu, rwu, rsd = d0.copy(), bu0.copy(), wu0.copy(), sd0.copy()
    ora.conv_backward(x, w, F, k, s, p, 9, out, rd, rbu, rwu, rsd, dil=d)
    dd, dbu, dwu, dsd = (_t(T, a) for a in (d0, bu0, wu0, sd0))
    hip.convBackward(batch, C, H, H, _t(T, x), _t(T, w), F, k, s, p, d, 9, _t(T, out), dd, dbu, dwu,
                     None, dsd)
    hip.finish()
    for gg, r in ((dd, rd), (dbu, rbu), (dwu, rwu), (dsd, rsd)):
        assert np.array_equal(gg.cpu().numpy(), r)


def test_conv_backward_rejects_dilation(hip, torch_cuda):
    from tensorium_amd._abi import TnsError
    z = torch_cuda.zeros(4096, device="cuda")
    with pytest.raises(TnsError):
        hip.convBackward(1, 1, 9, 9, z, z, 1, 3, 1, 2, 2, 9, z, z, z, z, None, None)


TILE_CASES = [
    (2, 32, 17, 128, 3, 1, 1, 9, 1), (3, 32, 12, 64, 3, 2, 1, 9, 1), (2, 64, 9, 32, 1, 1, 0, 4, 1),
    (1, 96, 26, 128, 3, 2, 1, 1, 1), (2, 32, 13, 256, 3, 1, 1, 0, 1), (2, 32, 21, 64, 3, 1, 2, 9, 2),
    (1, 32, 40, 32, 3, 1, 1, 9, 1),
    # K % 64 == 0 (the 64-deep k-tiles of conv_tile4.hip), 1x1 and 3x3
    (2, 64, 13, 128, 3, 1, 1, 9, 1), (1, 128, 11, 256, 3, 2, 1, 1, 1), (2, 128, 9, 128, 1, 1, 0, 4, 1),
    (1, 64, 20, 64, 3, 1, 2, 9, 2)]


def test_conv_tile_variants_bit_exact(hip, torch_cuda, ora):
    """Every plane-sized conv tile (conv_tile.hip, TNS_OPT_CONV_VARIANT =
    100 + v): bounds-checked gather from unpadded images, 1x1 and 3x3,
    strides 1/2, dilation 2, ragged N, fused bias + leaky/linear/relu and the
    separate logistic pass; tiles whose rows do not divide the filter count
    report UNSUPPORTED."""
    from tensorium_amd._abi import TnsError
    ntiles = hip.convTileVariants()
    assert ntiles >= 4
    ran = 0
    try:
        for v in range(ntiles):
            hip.setConvVariant(100 + v)
            for i, (batch, C, H, F, k, s, p, act, d) in enumerate(TILE_CASES):
                try:
                    got, ref = conv_case(hip, torch_cuda, ora, batch, C, H, F, k, s, p, act, 3,
                                         seed=i, dil=d)
                except TnsError:
                    continue
                ran += 1
                assert np.array_equal(got, ref), (v, batch, C, H, F, k, s, p, act, d)
    finally:
        hip.setConvVariant(-1)
    assert ran >= 2 * ntiles


PP_CASES = TILE_CASES + [(2, 32, 9, 128, 1, 1, 0, 4, 1), (2, 64, 9, 128, 1, 1, 0, 4, 1),
                         (2, 64, 26, 512, 3, 1, 1, 9, 1), (1, 64, 13, 1024, 3, 1, 1, 1, 1)]


def test_conv_pp_variants_bit_exact(hip, torch_cuda, ora):
    """Every ping-pong conv tile (conv_pp.hip, TNS_OPT_CONV_VARIANT = 200 + v):
    two wave groups alternating compute and staging, staging loads issued a
    phase early; one, two and many k-tiles (the prologue, the peeled last
    tiles), 1x1 / 3x3, strides 1/2, dilation 2, ragged N, fused epilogues and
    the separate logistic pass — bit-identical to the oracle."""
    from tensorium_amd._abi import TnsError
    nv = hip.convPPVariants()
    if nv == 0:
        pytest.skip("measured-and-not-picked family: diagnostics build only (TNS_DIAG=1)")
    assert nv >= 3
    ran = 0
    try:
        for v in range(nv):
            hip.setConvVariant(200 + v)
            for i, (batch, C, H, F, k, s, p, act, d) in enumerate(PP_CASES):
                try:
                    got, ref = conv_case(hip, torch_cuda, ora, batch, C, H, F, k, s, p, act, 3,
                                         seed=100 + i, dil=d)
                except TnsError:
                    continue
                ran += 1
                assert np.array_equal(got, ref), (v, batch, C, H, F, k, s, p, act, d)
    finally:
        hip.setConvVariant(-1)
    assert ran >= 3 * nv


def test_conv_dma_variants_bit_exact(hip, torch_cuda, ora):
    """Every LDS-DMA-ring conv tile (conv_dma.hip, TNS_OPT_CONV_VARIANT =
    300 + v): B gathered into LDS by dword LDS-DMA (out-of-window taps land
    as 0 through the range check), A by 16-byte LDS-DMA into the swizzled
    slot image, three stages two tiles ahead; one, two, three and many
    k-tiles, 1x1 / 3x3, strides 1/2, dilation 2, ragged N, fused epilogues
    and the separate logistic pass — bit-identical to the oracle."""
    from tensorium_amd._abi import TnsError
    nv = hip.convDMAVariants()
    if nv == 0:
        pytest.skip("measured-and-not-picked family: diagnostics build only (TNS_DIAG=1)")
    assert nv >= 3
    ran = 0
    cases = PP_CASES + [(2, 96, 11, 128, 1, 1, 0, 9, 1), (3, 32, 7, 64, 3, 1, 1, 9, 1)]
    try:
        for v in range(nv):
            hip.setConvVariant(300 + v)
            for i, (batch, C, H, F, k, s, p, act, d) in enumerate(cases):
                try:
                    got, ref = conv_case(hip, torch_cuda, ora, batch, C, H, F, k, s, p, act, 3,
                                         seed=200 + i, dil=d)
                except TnsError:
                    continue
                ran += 1
                assert np.array_equal(got, ref), (v, batch, C, H, F, k, s, p, act, d)
    finally:
        hip.setConvVariant(-1)
    assert ran >= 3 * nv


PATCH_CASES = [(2, 32, 17, 128, 3, 1, 1, 9, 1), (2, 32, 13, 256, 3, 1, 1, 0, 1),
               (1, 64, 26, 128, 3, 1, 1, 1, 1), (3, 32, 52, 128, 3, 1, 1, 9, 1),
               (2, 64, 13, 1024, 3, 1, 1, 9, 1), (1, 32, 104, 128, 3, 1, 1, 4, 1),
               (2, 32, 7, 64, 3, 1, 1, 9, 1), (1, 32, 23, 128, 3, 1, 1, 9, 1)]


def test_conv_patch_variants_bit_exact(hip, torch_cuda, ora):
    """Every input-patch conv tile (conv_patch.hip, TNS_OPT_CONV_VARIANT =
    400 + v): whole output rows per tile (partial last row groups), the
    5-channel zero-halo patch by dword LDS-DMA, tap offsets from the per-tile
    table — bit-identical to the oracle; tiles that do not fit a plane
    report UNSUPPORTED."""
    from tensorium_amd._abi import TnsError
    nv = hip.convPatchVariants()
    if nv == 0:
        pytest.skip("measured-and-not-picked family: diagnostics build only (TNS_DIAG=1)")
    assert nv >= 3
    ran = 0
    try:
        for v in range(nv):
            hip.setConvVariant(400 + v)
            for i, (batch, C, H, F, k, s, p, act, d) in enumerate(PATCH_CASES):
                try:
                    got, ref = conv_case(hip, torch_cuda, ora, batch, C, H, F, k, s, p, act, 3,
                                         seed=300 + i, dil=d)
                except TnsError:
                    continue
                ran += 1
                assert np.array_equal(got, ref), (v, batch, C, H, F, k, s, p, act, d)
    finally:
        hip.setConvVariant(-1)
    assert ran >= 2 * nv


SLAB_CASES = [
    # (batch, C, H, F, k, s, p, act): YOLOv3 13^2 / 26^2 layers at batch 8
    # (layers 45, 43, 28, 26, 44) and ragged / small ones (N past the last
    # column tile, one and two k-tiles)
    (8, 512, 13, 1024, 3, 1, 1, 9), (8, 256, 26, 1024, 3, 2, 1, 9), (8, 256, 26, 512, 3, 1, 1, 9),
    (8, 256, 52, 512, 3, 2, 1, 9), (8, 1024, 13, 512, 1, 1, 0, 9), (3, 64, 7, 128, 3, 1, 1, 1),
    (2, 16, 9, 64, 3, 1, 1, 4), (1, 128, 5, 64, 1, 1, 0, 0)]


def test_conv_slab_forms_bit_exact(hip, torch_cuda, ora):
    """Every two-pass slab form (conv_slab.hip, TNS_OPT_CONV_VARIANT = 500 +
    v: the im2col matrix written in the GEMM's LDS slot order, B by LDS-DMA)
    at the YOLOv3 13^2 / 26^2 shapes and ragged small ones, fused bias +
    leaky/relu/linear and the separate logistic pass: bit-identical to the
    oracle; forms whose tiles do not divide the filters / k report
    UNSUPPORTED."""
    from tensorium_amd._abi import TnsError
    nv = hip.convSlabForms()
    assert nv >= 2
    ran = 0
    try:
        for v in range(nv):
            hip.setConvVariant(500 + v)
            for i, (batch, C, H, F, k, s, p, act) in enumerate(SLAB_CASES):
                try:
                    got, ref = conv_case(hip, torch_cuda, ora, batch, C, H, F, k, s, p, act, 3,
                                         seed=40 + i)
                except TnsError:
                    continue
                ran += 1
                assert np.array_equal(got, ref), (v, batch, C, H, F, k, s, p, act)
    finally:
        hip.setConvVariant(-1)
    assert ran >= 3 * nv


C1_CASES = [
    # (batch, C, H, F, act): YOLOv3 1x1 layers at batch 8 — 208^2 (2), 104^2
    # (5), 52^2 (10, 68: 384 channels, 74: the 255-filter head), 26^2 (27, 60,
    # 66: head) — and ragged small ones (N past the last column tile, one k-tile)
    (8, 64, 208, 32, 9), (8, 128, 104, 64, 9), (8, 256, 52, 128, 9), (8, 384, 52, 128, 9),
    (8, 256, 52, 255, 4), (8, 512, 26, 256, 9), (8, 768, 26, 256, 9), (8, 512, 26, 255, 4),
    (3, 64, 6, 48, 1), (1, 32, 2, 16, 0), (2, 128, 10, 40, 9)]


def test_conv1x1_forms_bit_exact(hip, torch_cuda, ora):
    """Every DMA-fed 1x1 form (conv1x1.hip, TNS_OPT_CONV_VARIANT = 600 + v:
    the input planes straight into LDS, interleaved fragment columns, 16-byte
    output stores) at the YOLOv3 1x1 shapes — filter counts that are not a
    multiple of the block (the 255-filter heads) included — and small ragged
    ones, fused bias + leaky/relu/linear and the separate logistic pass:
    bit-identical to the oracle; forms whose k-tile does not divide k report
    UNSUPPORTED."""
    from tensorium_amd._abi import TnsError
    nv = hip.conv1x1Forms()
    assert nv >= 2
    ran = 0
    try:
        for v in range(nv):
            hip.setConvVariant(600 + v)
            for i, (batch, C, H, F, act) in enumerate(C1_CASES):
                try:
                    got, ref = conv_case(hip, torch_cuda, ora, batch, C, H, F, 1, 1, 0, act, 3,
                                         seed=70 + i)
                except TnsError:
                    continue
                ran += 1
                assert np.array_equal(got, ref), (v, batch, C, H, F, act)
    finally:
        hip.setConvVariant(-1)
    assert ran >= 6 * nv
