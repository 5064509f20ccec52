#!/usr/bin/env python3
"""A few 4096^3 NN SGEMMs (the headline kernel) for counter passes.

  rocprofv3 --pmc ... -- python3 scripts/sgemm_one.py [--reps 5]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--n", type=int, default=4096)
a = ap.parse_args()
hip = TNNHip(0)
n = a.n
A = torch.rand(n, n, device="cuda") * 2 - 1
B = torch.rand(n, n, device="cuda") * 2 - 1
C = torch.empty(n, n, device="cuda")
for _ in range(a.reps):
    hip.gemm(False, False, n, n, n, 1.0, A, 0, n, B, 0, n, 0.0, C, 0, n)
torch.cuda.synchronize()
print("ok")
