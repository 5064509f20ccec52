"""Darknet plan (cfg parsing, shapes), .weights I/O and BN folding on the CPU;
the whole YOLOv3 forward (convolutions + shortcut / route / upsample / yolo)
on the GPU against the oracle.

Bar: every layer bit-exact (the yolo layers' logistic evaluates exp in double
and rounds once, as the oracle does)."""
import numpy as np
import pytest

from tensorium_amd import darknet as dn
from tensorium_amd.yolo import yolov3_conv_table


def test_yolov3_cfg_plan_matches_conv_table():
    net = dn.Network(dn.parse_cfg(dn.yolov3_cfg(416)), 8)
    kinds = [l.kind for l in net.layers]
    assert len(net.layers) == 107
    assert (kinds.count("convolutional"), kinds.count("shortcut"), kinds.count("route"),
            kinds.count("upsample"), kinds.count("yolo")) == (75, 23, 4, 2, 3)
    assert [l.index for l in net.layers if l.kind == "yolo"] == [82, 94, 106]
    for l, t in zip(net.convs(), yolov3_conv_table()):
        assert (l.c, l.h, l.filters, l.size, l.stride, l.pad, l.activation, l.bn) == \
            (t.c, t.h, t.filters, t.size, t.stride, t.pad, t.activation, t.batch_normalize)
    assert net.layers[86].inputs == (85, 61) and net.layers[86].out_c == 768
    assert net.layers[83].inputs == (79,)


def test_cfg_parser_rejects_and_comments():
    with pytest.raises(ValueError):
        dn.parse_cfg("[convolutional]\nfilters=3\n")
    secs = dn.parse_cfg("# c\n[net]\nwidth=32 \n; x\nheight=32\n[convolutional]\nfilters=4\n"
                        "size=3\nstride=2\npad=1\nactivation=leaky\n")
    net = dn.Network(secs, 2)
    assert (net.layers[0].out_h, net.layers[0].out_c, net.layers[0].pad) == (16, 4, 1)
    with pytest.raises(ValueError):
        dn.Network(dn.parse_cfg("[net]\nwidth=8\nheight=8\n[maxpoolx]\n"))


@pytest.mark.parametrize("major,minor", [(0, 2), (0, 1)])
def test_weights_round_trip(tmp_path, major, minor):
    net = dn.Network(dn.parse_cfg(dn.yolov3_cfg(64)), 1)
    ps = dn.random_params(net, seed=7)
    path = tmp_path / "w.weights"
    dn.write_weights(path, net, ps, major=major, minor=minor, seen=12345)
    got, seen = dn.load_weights(path, net)
    assert seen == 12345
    for a, b in zip(got, ps):
        assert np.array_equal(a.biases, b.biases) and np.array_equal(a.weights, b.weights)
        if b.scales is not None:
            assert np.array_equal(a.rolling_var, b.rolling_var)
    with pytest.raises(ValueError):
        (tmp_path / "short.weights").write_bytes(path.read_bytes()[:1000])
        dn.load_weights(tmp_path / "short.weights", net)


def test_fuse_batchnorm_matches_oracle():
    from oracle import oracle as ora
    net = dn.Network(dn.parse_cfg(dn.yolov3_cfg(64)), 1)
    l = net.convs()[1]
    p = dn.random_params(net, seed=9)[1]
    f = dn.fuse_batchnorm(l, p)
    w, b = p.weights.ravel().copy(), p.biases.copy()
    ora.lib().ora_fuse_batchnorm(l.filters, l.c * 9, ora._p(w), ora._p(b), ora._p(p.scales),
                                 ora._p(p.rolling_mean), ora._p(p.rolling_var))
    assert np.array_equal(f.weights.ravel(), w) and np.array_equal(f.biases, b)


def test_oracle_layers_small():
    from oracle import oracle as ora
    x = ora.uniform(2 * 3 * 4 * 5, 11, 0)
    up = ora.upsample(x, 6, 4, 5, 2).reshape(6, 8, 10)
    assert np.array_equal(up, np.repeat(np.repeat(x.reshape(6, 4, 5), 2, 1), 2, 2))
    y = ora.yolo_forward(x, 1, 2, 1, 10)  # 2 anchors x 6 entries x 10
    e = y.reshape(2, 6, 10)
    assert np.array_equal(e[:, 2:4], x.reshape(2, 6, 10)[:, 2:4])
    assert np.allclose(e[:, [0, 1, 4, 5]], 1 / (1 + np.exp(-x.reshape(2, 6, 10)[:, [0, 1, 4, 5]])))


@pytest.mark.gpu
@pytest.mark.parametrize("size,batch", [(64, 2), (96, 1)])
def test_yolov3_network_forward_vs_oracle(hip, torch_cuda, ora, size, batch):
    net = dn.Network(dn.parse_cfg(dn.yolov3_cfg(size)), batch)
    ps = dn.random_params(net, seed=size + batch)
    x = ora.uniform(batch * 3 * size * size, 3, size, 0.0, 1.0)
    ref = ora.darknet_forward(net, ps, x)
    model = dn.HipDarknet(hip, net, ps, torch_cuda)
    outs = model.forward(torch_cuda.from_numpy(x).cuda())
    hip.finish()
    for l, o, r in zip(net.layers, outs, ref):
        assert np.array_equal(o.cpu().numpy(), r), (l.index, l.kind)


@pytest.mark.gpu
def test_upsample_shortcut_yolo_ops(hip, torch_cuda, ora):
    T = torch_cuda
    x = ora.uniform(3 * 7 * 9, 12, 0)
    out = T.empty(3 * 14 * 18, device="cuda")
    hip.upSample(1, 3, 7, 9, T.from_numpy(x).cuda(), 2, 1, 1.0, out)
    hip.finish()
    assert np.array_equal(out.cpu().numpy(), ora.upsample(x, 3, 7, 9, 2))
    # backward direction (isForward = 0): in += scale*out over each pixel's
    # stride x stride block, row-major (nupsamplelayer.pas:101-110)
    for zero, scale, s in ((0, 1.0, 2), (1, 0.5, 2), (0, 0.3, 3)):
        g = ora.uniform(3 * 7 * s * 9 * s, 15, s)
        base = ora.uniform(3 * 7 * 9, 16, s)
        dev_in = T.from_numpy(base.copy()).cuda()
        hip.upSample(1, 3, 7, 9, dev_in, s, 0, scale, T.from_numpy(g).cuda(), zero)
        hip.finish()
        ref = np.zeros_like(base) if zero else base.copy()
        g4 = g.reshape(3, 7, s, 9, s)
        sc = np.float32(scale)
        for dy in range(s):
            for dx in range(s):
                ref = (ref + (sc * g4[:, :, dy, :, dx]).reshape(-1)).astype(np.float32)
        assert np.array_equal(dev_in.cpu().numpy(), ref), (zero, scale, s)
    for n in (1000, 1001):  # float4 and scalar forms
        a, b = ora.uniform(n, 13, 0), ora.uniform(n, 13, 1)
        o = T.empty(n, device="cuda")
        for act in (4, 9, 1):
            hip.shortcut(n, T.from_numpy(a).cuda(), 0, T.from_numpy(b).cuda(), 0, o, 0, act)
            hip.finish()
            assert np.array_equal(o.cpu().numpy(), ora.shortcut(a, b, act)), (n, act)
    y = ora.uniform(2 * 3 * 85 * 13, 14, 0, -4.0, 4.0)
    oy = T.empty(y.size, device="cuda")
    hip.yoloForward(2, 3, 80, 13, T.from_numpy(y).cuda(), oy)
    hip.finish()
    r = ora.yolo_forward(y, 2, 3, 80, 13)
    assert np.array_equal(oy.cpu().numpy(), r)
