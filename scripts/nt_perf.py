#!/usr/bin/env python3
"""gemm(NoTrans, Trans) throughput in the reference's sdot order against the
plain ascending-k MFMA kernel, and the addSums-order backward bias, on the
shapes the reference runs them at (FC forward at batch 32, conv dW per
image, a 4096^3 square).  One JSON line to stdout.

  python scripts/nt_perf.py
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    hip = TNNHip(0)
    out = {}
    for M, N, K in [(32, 4096, 4096), (32, 1024, 9216), (256, 1152, 2704), (1024, 4608, 169),
                    (4096, 4096, 4096)]:
        A = torch.rand(M, K, device="cuda") * 2 - 1
        B = torch.rand(N, K, device="cuda") * 2 - 1
        C = torch.zeros(M, N, device="cuda")
        run = lambda: hip.gemm(False, True, M, N, K, 1.0, A, 0, K, B, 0, K, 0.0, C, 0, N)  # noqa
        row = {}
        for name, on in (("sdot", True), ("plain", False)):
            hip.setNtSdot(on)
            ms = timed(run, 5 if M * N * K > 1e10 else 20)
            row[name] = {"ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9, 2)}
        hip.setNtSdot(True)
        out[f"nt_{M}x{N}x{K}"] = row
    for F, bs, batch in [(32, 173056, 8), (256, 2704, 8), (1024, 169, 8)]:
        src = torch.rand(batch * F * bs, device="cuda")
        dst = torch.zeros(F, device="cuda")
        ms = timed(lambda: hip.backwardBias(F, dst, src.numel(), src, 0, 1, batch))
        out[f"addsums_{F}x{bs}x{batch}"] = {"ms": round(ms, 4),
                                             "gbs": round(src.numel() * 4 / ms / 1e6, 1)}
    nw = 4096 * 4096
    W, dW = torch.rand(nw, device="cuda"), torch.rand(nw, device="cuda")
    b, db = torch.rand(4096, device="cuda"), torch.rand(4096, device="cuda")
    ms = timed(lambda: hip.sgdUpdate(W, dW, b, db, 1e-3, 32, 1e-4, 0.9))
    out["sgd_update_16M"] = {"ms": round(ms, 4), "gbs": round(16 * nw / ms / 1e6, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
