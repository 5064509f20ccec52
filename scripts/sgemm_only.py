#!/usr/bin/env python3
"""Run one SGEMM shape repeatedly (for rocprofv3 counter passes)."""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--variant", type=int, default=-1)
a = ap.parse_args()
hip = TNNHip(0)
n = a.n
A = torch.rand(n, n, device="cuda") * 2 - 1
B = torch.rand(n, n, device="cuda") * 2 - 1
C = torch.zeros(n, n, device="cuda")
for _ in range(a.reps):
    hip.gemmVariant(a.variant, False, False, n, n, n, 1.0, A, 0, n, 0, B, 0, n, 0, 0.0, C, 0, n, 0)
hip.finish()
print("done")
