"""A darknet training pass through the drop-in, in the reference's call order
(TNet.forward in training, then TNet.backward: nnet.pas:275-366), on the
pipelined backward schedule the Pascal binding selects (initHIP,
pipelineBackward = true) and on the joined one — bit-exact against the
oracle's restated pass (tests/_darknet_oracle.py).

The non-conv calls between conv layers (the shortcut's DeriveArray and two
addvv, a route's addvv, an upsample's accumulation, a yolo layer's axpy) join
the dW products pending on the side stream only when their operands meet a
pending dW's (tns.h, TNS_OPT_BWD_OVERLAP); the residual-block test asserts
the pipeline stays running across a shortcut."""
import numpy as np
import pytest

from tensorium_amd import darknet as dn

from _darknet_oracle import train_pass

pytestmark = pytest.mark.gpu


def _stage_cfg(batch):
    """YOLOv3's conv layers 9..13 (the stride-2 entry to the 52^2 stage and
    its first two residual blocks; yolov3.cfg), as a network of their own."""
    conv = ("[convolutional]\nbatch_normalize=1\nfilters={f}\nsize={k}\nstride={s}\npad=1\n"
            "activation=leaky\n")
    sc = "[shortcut]\nfrom=-3\nactivation=linear\n"
    return (f"[net]\nbatch={batch}\nwidth=104\nheight=104\nchannels=128\n" +
            conv.format(f=256, k=3, s=2) +
            conv.format(f=128, k=1, s=1) + conv.format(f=256, k=3, s=1) + sc +
            conv.format(f=128, k=1, s=1) + conv.format(f=256, k=3, s=1) + sc)


def _run(hip, torch, net, params, x, yd, mode, on_backward=None):
    model = dn.HipDarknetTrain(hip, net, params, torch)
    X = torch.from_numpy(x).cuda()
    try:
        hip.setBwdOverlap(mode)
        model.forward(X)
        model.set_yolo_deltas([torch.from_numpy(d).cuda() for d in yd])
        model.backward(X, on_backward)
        hip.finish()
    finally:
        hip.setBwdOverlap(True)
    return model


def _compare(net, model, outs, deltas, state):
    for l in net.layers:
        i = l.index
        assert np.array_equal(model.out[i].cpu().numpy(), outs[i]), f"output {i} ({l.kind})"
        assert np.array_equal(model.delta[i].cpu().numpy(), deltas[i]), f"delta {i} ({l.kind})"
        if l.kind != "convolutional":
            continue
        st, rs = model.conv[i], state[i]
        assert np.array_equal(st["wu"].cpu().numpy(), rs["wu"]), f"weight_updates {i}"
        if l.bn:
            for k in ("su", "md", "vd", "mean", "var", "rm", "rv"):
                assert np.array_equal(st[k].cpu().numpy(), rs[k]), f"{k} {i}"
        else:
            assert np.array_equal(st["bu"].cpu().numpy(), rs["bu"]), f"bias_updates {i}"


@pytest.mark.parametrize("mode", [2, 1])
def test_two_residual_blocks_train_pass(hip, torch_cuda, ora, mode):
    """YOLOv3 layers 9..13 + two shortcuts at 104^2 -> 52^2, batch 8: every
    output, delta, update and BN statistic bit-exact; on the pipelined
    schedule the two dW products of the upper block are still pending after
    the lower shortcut's DeriveArray + addvv calls (they write deltas no
    pending dW reads), and the count only grows until the final finish."""
    net = dn.Network(dn.parse_cfg(_stage_cfg(8)), 8)
    params = dn.random_params(net, seed=61)
    rng = np.random.default_rng(61)
    x = rng.uniform(0, 1, (8, 128, 104, 104)).astype(np.float32)
    # no yolo layer: the top shortcut's delta is what the layers above left
    seen = []
    top = net.layers[-1].index
    d_top = rng.uniform(-1, 1, 8 * net.layers[-1].out_size).astype(np.float32)
    outs_ref, deltas_ref, state_ref = train_pass(ora, net, params, x, [],
                                                 seed_delta={top: d_top})

    def probe(l):
        seen.append((l.index, l.kind, hip.pendingDw()))

    model = dn.HipDarknetTrain(hip, net, params, torch_cuda)
    X = torch_cuda.from_numpy(x).cuda()
    try:
        hip.setBwdOverlap(mode)
        model.forward(X)
        model.delta[top].copy_(torch_cuda.from_numpy(d_top).cuda())
        model.backward(X, probe)
        hip.finish()
    finally:
        hip.setBwdOverlap(True)
    assert hip.pendingDw() == 0
    _compare(net, model, outs_ref, deltas_ref, state_ref)
    counts = [c for _, _, c in seen]
    if mode == 2:
        # layers 6 (shortcut), 5, 4 (conv), 3 (shortcut), 2, 1, 0 (conv)
        assert [k for _, k, _ in seen] == ["shortcut", "convolutional", "convolutional",
                                           "shortcut", "convolutional", "convolutional",
                                           "convolutional"]
        assert counts == [0, 1, 2, 2, 3, 4, 5], seen
    else:
        assert counts == [0] * 7, seen


@pytest.mark.parametrize("mode", [2, 1])
def test_whole_yolov3_train_pass_small(hip, torch_cuda, ora, mode):
    """The whole YOLOv3 plan (75 conv, 23 shortcut, 4 route, 2 upsample, 3
    yolo layers) at 64 px, batch 2: training forward, synthetic yolo deltas,
    TNet.backward through every layer — every output, delta, update and BN
    statistic bit-exact against the oracle, pipelined and joined."""
    net = dn.Network(dn.parse_cfg(dn.yolov3_cfg(64)), 2)
    params = dn.random_params(net, seed=62)
    rng = np.random.default_rng(62)
    x = rng.uniform(0, 1, (2, 3, 64, 64)).astype(np.float32)
    yd = [rng.uniform(-0.1, 0.1, 2 * l.out_size).astype(np.float32)
          for l in net.layers if l.kind == "yolo"]
    outs, deltas, state = train_pass(ora, net, params, x, yd)
    model = _run(hip, torch_cuda, net, params, x, yd, mode)
    _compare(net, model, outs, deltas, state)


def test_scratch_cap_takes_dw_fallback(hip, torch_cuda, ora):
    """when the residue-major dW buffers cannot be had (here: a
    scratch cap below their size), the conv backward clears the error and
    takes the workspace-only dW path — bit-exact, and the next call without
    the cap runs the residue form again (nothing sticky left behind)."""
    from tensorium_amd.yolo import yolov3_conv_table
    s = yolov3_conv_table()[11]          # 52^2, 128 -> 256 3x3 (dw_res by shape)
    B = 2
    rng = np.random.default_rng(63)
    x = rng.uniform(0, 1, (B, s.c, s.h, s.h)).astype(np.float32)
    w = rng.uniform(-0.1, 0.1, (s.filters, s.K)).astype(np.float32)
    out = rng.uniform(-1, 1, (B, s.filters, s.out_h, s.out_h)).astype(np.float32)
    d0 = rng.uniform(-1, 1, out.shape).astype(np.float32)
    bu0 = rng.uniform(-1, 1, s.filters).astype(np.float32)
    wu0 = rng.uniform(-1, 1, s.filters * s.K).astype(np.float32)
    sd0 = rng.uniform(-1, 1, x.shape).astype(np.float32)
    rd, rbu, rwu, rsd = d0.copy(), bu0.copy(), wu0.copy(), sd0.copy()
    ora.conv_backward(x, w.ravel(), s.filters, s.size, s.stride, s.pad, s.activation, out, rd,
                      rbu, rwu, rsd)
    t = lambda a: torch_cuda.from_numpy(a.copy()).cuda()  # noqa: E731
    ws = torch_cuda.zeros(B * s.K * s.out_h * s.out_h, device="cuda")
    for cap in (2_000_000, 0):
        dx, dw, dout, dd, dbu, dwu, dsd = map(t, (x, w, out, d0, bu0, wu0, sd0))
        try:
            hip.setScratchCap(cap)
            hip.convBackward(B, s.c, s.h, s.h, dx, dw, s.filters, s.size, s.stride, s.pad, 1,
                             s.activation, dout, dd, dbu, dwu, ws, dsd)
            hip.finish()
        finally:
            hip.setScratchCap(0)
        assert np.array_equal(dwu.cpu().numpy(), rwu), cap
        assert np.array_equal(dsd.cpu().numpy(), rsd), cap
        assert np.array_equal(dd.cpu().numpy(), rd), cap
        assert np.array_equal(dbu.cpu().numpy(), rbu), cap
