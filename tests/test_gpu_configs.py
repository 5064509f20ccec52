"""BASELINE configs 3 and 4 at their real sizes on the GPU.

Config 4 — 1024 independent 1024^3 fp32 GEMMs (12.9 GB of operands, one
MI355X): sampled rows of sampled GEMMs bit-exact against the oracle's
restated sgemm_nn (saxpy FMA chains, ntensors.pas:2061-2157); every one of the
1024 products checked by a checksum-linearity property (column sums of C_b
against colsum(A_b) @ B_b in float64, componentwise bound
1e-4 * colsum(|A_b|) @ |B_b|); and the shards of world sizes 1, 2 and 8
(tensorium_amd.shard.shard_range, the contiguous blocks each rank runs) give
bit-identical products to the single call.

Config 3 — YOLOv3-416 nConvolutionLayer.forward at batch 8: all 75
convolutions (BN folded, leaky / linear) bit-exact against the oracle's
restated layer (im2col + sgemm_nn + forwardBias + activate), each fed its own
synthetic input (teacher forcing); and the whole 107-layer network
at 416 px, batch 2, every layer bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free(torch):
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def test_config4_1024_gemms_1024cubed(hip, torch_cuda, ora):
    from tensorium_amd.shard import shard_range
    torch = torch_cuda
    G, n = 1024, 1024
    g = torch.Generator(device="cuda").manual_seed(4)
    A = torch.rand(G, n, n, device="cuda", generator=g) * 2 - 1
    B = torch.rand(G, n, n, device="cuda", generator=g) * 2 - 1
    C = torch.empty(G, n, n, device="cuda")
    hip.gemmStridedBatched(False, False, n, n, n, 1.0, A, 0, n, n * n, B, 0, n, n * n, 0.0, C, 0,
                           n, n * n, G)
    hip.finish()
    # the shards of every world size reproduce the single call bit for bit
    # (beta = 0 is 0*C as in the reference, so the sentinel must be finite;
    # a shard that is never written keeps it and fails the comparison)
    Cs = torch.empty_like(C)
    for world in (2, 8):
        Cs.fill_(12345.0)
        for r in range(world):
            s, e = shard_range(G, r, world)
            hip.gemmStridedBatched(False, False, n, n, n, 1.0, A, s * n * n, n, n * n, B,
                                   s * n * n, n, n * n, 0.0, Cs, s * n * n, n, n * n, e - s)
        hip.finish()
        assert torch.equal(Cs, C), world
    del Cs
    # sampled rows bit-exact vs the restated reference
    for b in (0, 1, 511, 1023):
        a, bb = A[b].cpu().numpy(), B[b].cpu().numpy()
        for r in (0, 517, 1023):
            ref = np.zeros((1, n), np.float32)
            ora.sgemm(False, False, 1, n, n, 1.0, a[r:r + 1].copy(), n, bb, n, 0.0, ref, n)
            assert np.array_equal(C[b, r].cpu().numpy(), ref[0]), (b, r)
    # checksum linearity on all 1024 products (float64 checker)
    for s in range(0, G, 64):
        a64 = A[s:s + 64].double()
        b64 = B[s:s + 64].double()
        lhs = C[s:s + 64].double().sum(dim=1)
        rhs = torch.bmm(a64.sum(dim=1, keepdim=True), b64)[:, 0]
        bound = torch.bmm(a64.abs().sum(dim=1, keepdim=True), b64.abs())[:, 0]
        assert bool(((lhs - rhs).abs() <= 1e-4 * bound + 1e-30).all()), s
        del a64, b64, lhs, rhs, bound
    del A, B, C
    _free(torch)


@pytest.mark.parametrize("idx", range(75))
def test_yolov3_layer_batch8_416(hip, torch_cuda, ora, idx):
    from tensorium_amd.yolo import yolov3_conv_table
    from test_gpu_conv import conv_case
    spec = yolov3_conv_table()[idx]
    got, ref = conv_case(hip, torch_cuda, ora, 8, spec.c, spec.h, spec.filters, spec.size,
                         spec.stride, spec.pad, spec.activation, True, seed=spec.index)
    assert np.array_equal(got, ref), spec


def test_yolov3_network_416_batch2(hip, torch_cuda, ora):
    from tensorium_amd import darknet as dn
    size, batch = 416, 2
    net = dn.Network(dn.parse_cfg(dn.yolov3_cfg(size)), batch)
    ps = dn.random_params(net, seed=size + batch)
    x = ora.uniform(batch * 3 * size * size, 3, size, 0.0, 1.0)
    ref = ora.darknet_forward(net, ps, x)
    model = dn.HipDarknet(hip, net, ps, torch_cuda)
    outs = model.forward(torch_cuda.from_numpy(x).cuda())
    hip.finish()
    bad = [(l.index, l.kind) for l, o, r in zip(net.layers, outs, ref)
           if not np.array_equal(o.cpu().numpy(), r)]
    assert not bad, bad
