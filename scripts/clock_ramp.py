#!/usr/bin/env python3
"""Per-launch duration of the 4096^3 SGEMM over a long back-to-back run
(clock ramp / steady state), HIP events on the kernel's stream.

  python scripts/clock_ramp.py [--reps 400]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--reps", type=int, default=400)
a = ap.parse_args()
hip = TNNHip(0)
n = a.n
A = torch.rand(n, n, device="cuda") * 2 - 1
B = torch.rand(n, n, device="cuda") * 2 - 1
C = torch.zeros(n, n, device="cuda")
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
      for _ in range(a.reps)]
torch.cuda.synchronize()
for e0, e1 in ev:
    e0.record()
    hip.gemm(False, False, n, n, n, 1.0, A, 0, n, B, 0, n, 0.0, C, 0, n)
    e1.record()
torch.cuda.synchronize()
ms = [e0.elapsed_time(e1) for e0, e1 in ev]
blk = 20
print(json.dumps({"block_means_ms": [round(sum(ms[i:i + blk]) / blk, 4)
                                     for i in range(0, len(ms), blk)],
                  "first": [round(x, 3) for x in ms[:10]], "min": round(min(ms), 4)}))
