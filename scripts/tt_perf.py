#!/usr/bin/env python3
"""gemm(Trans, Trans) throughput: the reference-order VALU kernel
(sgemm_tt.hip, bit-exact) against the fp32 MFMA kernel (TNS_OPT_TT_EXACT = 0).
One JSON line to stdout.

  python scripts/tt_perf.py
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from nt_perf import timed  # noqa: E402


def main():
    hip = TNNHip(0)
    out = {}
    for M, N, K in [(256, 256, 256), (1024, 1024, 1024), (4096, 4096, 4096), (512, 4608, 169)]:
        A = torch.rand(K, M, device="cuda") * 2 - 1
        B = torch.rand(N, K, device="cuda") * 2 - 1
        C = torch.zeros(M, N, device="cuda")
        run = lambda: hip.gemm(True, True, M, N, K, 1.0, A, 0, M, B, 0, K, 0.0, C, 0, N)  # noqa
        row = {}
        for name, on in (("exact_valu", True), ("mfma", False)):
            hip.setTtExact(on)
            ms = timed(run, 5 if M * N * K > 1e10 else 20)
            row[name] = {"ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9, 2)}
        hip.setTtExact(True)
        out[f"tt_{M}x{N}x{K}"] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main()
