#!/usr/bin/env python3
"""Vendor-library fp32 GEMM on the same box, for context beside the bench's
SGEMM: torch.mm (hipBLASLt / rocBLAS, TF32 off) at M=N=K=4096, timed like
bench.py (30 warm-up, 50 timed, HIP events).  One JSON line."""
import json

import torch

torch.backends.cuda.matmul.allow_tf32 = False
n = 4096
A = torch.rand(n, n, device="cuda") * 2 - 1
B = torch.rand(n, n, device="cuda") * 2 - 1
C = torch.empty(n, n, device="cuda")
for _ in range(30):
    torch.mm(A, B, out=C)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    torch.mm(A, B, out=C)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 50
print(json.dumps({"op": "torch.mm fp32 4096^3 (allow_tf32=False)", "ms": round(ms, 4),
                  "tflops": round(2 * n ** 3 / ms / 1e9, 2), "torch": torch.__version__}))
