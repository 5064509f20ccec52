#!/usr/bin/env python3
"""One sdot-order NT shape on one form, for counter passes:
  python scripts/sdot_one.py M N K batch form [reps]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402

M, N, K, batch, form = (int(x) for x in sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
hip = TNNHip(0)
A = torch.rand(batch, M, K, device="cuda") * 2 - 1
B = torch.rand(batch, N, K, device="cuda") * 2 - 1
C = torch.zeros(batch, M, N, device="cuda")
hip.setSdotForm(form)
for _ in range(reps):
    hip.gemmStridedBatched(False, True, M, N, K, 1.0, A, 0, K, M * K, B, 0, K, N * K, 0.0, C, 0, N,
                           M * N, batch)
torch.cuda.synchronize()
print("ok")
