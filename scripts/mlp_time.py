#!/usr/bin/env python3
"""µs per fused MNIST train step (bench.py's mnist leg alone), for A/B runs
between library builds: TNS_LIB=ab/<name>/libtensorium_hip.so python scripts/mlp_time.py"""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402

widths, acts, B = [784, 64, 64, 64, 64, 32, 10], [1, 1, 1, 1, 1, 4], 32
hip = TNNHip(0)
n = TNNHip.mlpBufferFloats(widths, True, B)
g = torch.Generator(device="cuda").manual_seed(5)
buf = torch.zeros(n + 256, device="cuda")
off = 0
for l in range(len(widths) - 1):
    I, O = widths[l], widths[l + 1]
    buf[off:off + I * O] = (torch.rand(I * O, device="cuda", generator=g) * 2 - 1) * (2.0 / I) ** 0.5
    off += 2 * I * O + 2 * O
    buf[off:off + O] = 1.0
    off += 4 * O + 4 * B * O + 4 * O
X = torch.rand(B, 784, device="cuda", generator=g)
T = torch.zeros(B, 10, device="cuda")
T[torch.arange(B), torch.randint(0, 10, (B,), device="cuda", generator=g)] = 1.0
cost = torch.zeros(1, device="cuda")
step = lambda: hip.mlpTrainStep(widths, acts, True, B, X, T, 1e-3, 0.9, 1e-4, buf, cost)  # noqa
res = []
for r in range(5):
    for _ in range(50):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(300):
        step()
    torch.cuda.synchronize()
    res.append((time.perf_counter() - t0) / 300 * 1e6)
print(json.dumps({"lib": str(hip.lib_path) if hasattr(hip, "lib_path") else None,
                  "us_per_step": [round(x, 2) for x in res], "cost": float(cost.item())}))
