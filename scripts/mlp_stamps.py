#!/usr/bin/env python3
"""Stage timing of the fused MLP train step from a diagnostic build
(TNS_EXTRA_CFLAGS=-DTNS_MLP_STAMPS, loaded with TNS_LIB=...): s_memtime
stamps written after the packed buffer.  Prints cycles per stage."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402

widths, acts, B = [784, 64, 64, 64, 64, 32, 10], [1, 1, 1, 1, 1, 4], 32
hip = TNNHip(0)
n = TNNHip.mlpBufferFloats(widths, True, B)
buf = torch.zeros(n + 256, device="cuda")
off = 0
for l in range(len(widths) - 1):
    I, O = widths[l], widths[l + 1]
    buf[off:off + I * O] = (torch.rand(I * O, device="cuda") * 2 - 1) * (2.0 / I) ** 0.5
    off += 2 * I * O + 2 * O
    buf[off:off + O] = 1.0
    off += 4 * O + 4 * B * O + 4 * O
X = torch.rand(B, 784, device="cuda")
T = torch.zeros(B, 10, device="cuda")
T[torch.arange(B), torch.randint(0, 10, (B,))] = 1.0
cost = torch.zeros(1, device="cuda")
for _ in range(20):
    hip.mlpTrainStep(widths, acts, True, B, X, T, 1e-3, 0.9, 1e-4, buf, cost)
torch.cuda.synchronize()
st = buf[n:n + 256].cpu().numpy().view(np.uint32).astype(np.uint64)
t = st[0::2] | (st[1::2] << 32)
names = {0: "start"}
names.update({1 + l: f"fwd{l}" for l in range(6)})
names[20] = "softmax"
names.update({21 + l: f"bwd{l}" for l in range(6)})
names[40] = "update"
names.update({50 + 2 * l: f"bwd{l}.stage" for l in range(6)})
names.update({51 + 2 * l: f"bwd{l}.chan" for l in range(6)})
order = [0] + [1 + l for l in range(6)] + [20]
for l in reversed(range(6)):
    order += [50 + 2 * l, 51 + 2 * l, 21 + l]  # stage, column pass, gemms
order += [40]
prev = None
for i in order:
    if prev is not None:
        print(f"{names[i]:8s} {int(t[i]) - int(t[prev]):8d} cycles")
    prev = i
print(f"total    {int(t[order[-1]]) - int(t[0]):8d} cycles (s_memtime ticks)")

m = t[64:128]
def mk(i): return int(m[i])
fw = ["prefetch issued", "gemm done", "after barrier", "fold done", "after barrier",
      "chains done", "after barrier", "element pass done", "after barrier"]
print("forward layer 1 (wave 0 marks, cycles since the previous mark):")
for i in range(1, 9):
    print(f"  {fw[i]:20s} {mk(i) - mk(i - 1):8d}")
bw = {11: "B1 done", 12: "after barrier", 13: "chains done", 14: "after barrier",
      15: "normalizeDelta done", 16: "after barrier", 17: "dW task done",
      18: "(dX) loop done", 19: "after barrier"}
print("backward stage 2:")
for i in range(11, 20):
    print(f"  {bw[i]:20s} {mk(i) - mk(i - 1):8d}")
gm = {20: "gemm: start", 21: "operand loads issued", 22: "stored to LDS", 23: "after barrier",
      24: "MFMAs issued", 25: "after barrier", 26: "partials stored"}
print("forward layer 1 gemm (wave 0, cycles since the layer's mark 0):")
for i in range(20, 27):
    print(f"  {gm[i]:22s} {mk(i) - mk(0):8d}")
