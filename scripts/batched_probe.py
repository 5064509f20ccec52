#!/usr/bin/env python3
"""Config 4 (1024 independent 1024^3 GEMMs, bench.py bench_batched) timed
under variations that isolate the per-block C traffic: strict beta = 0 (the
reference's 0*C: C read), BLAS beta = 0 (C not read), beta = 1, and fewer /
more GEMMs per launch.  One JSON line.

  python scripts/batched_probe.py [--steps 3]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--n-gemm", type=int, default=1024)
    a = ap.parse_args()
    hip = TNNHip(0)
    n, nb = 1024, a.n_gemm
    A = torch.rand(nb, n, n, device="cuda") * 2 - 1
    B = torch.rand(nb, n, n, device="cuda") * 2 - 1
    C = torch.rand(nb, n, n, device="cuda") * 2 - 1

    def timed(beta, cnt):
        def step():
            hip.gemmStridedBatched(False, False, n, n, n, 1.0, A, 0, n, n * n, B, 0, n, n * n, beta,
                                   C, 0, n, n * n, cnt)
        step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        return {"ms": round(ms, 4), "tflops": round(2.0 * n ** 3 * cnt / ms / 1e9, 2)}

    row = {"strict_beta0": timed(0.0, nb), "beta1": timed(1.0, nb)}
    hip.lib.tns_set_option(0, 0)
    row["blas_beta0"] = timed(0.0, nb)
    hip.lib.tns_set_option(0, 1)
    row["strict_beta0_256"] = timed(0.0, 256)
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
