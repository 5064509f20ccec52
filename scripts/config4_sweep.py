#!/usr/bin/env python3
"""Config 4 (1024 independent 1024^3 NN GEMMs, strict beta = 0) on each
large-NN SGEMM form (TNS gemm variants *_nn_big, forced), interleaved rounds,
the default pick beside them; C compared bit for bit with the default's.

  python scripts/config4_sweep.py [--rounds 2] [--steps 3]
"""
import argparse
import hashlib
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--n-gemm", type=int, default=1024)
a = ap.parse_args()
hip = TNNHip(0)
names = TNNHip.gemmVariants()
vs = [-1] + [i for i, nm in enumerate(names) if nm.endswith("nn_big")]
n, nb = 1024, a.n_gemm
g = torch.Generator(device="cuda").manual_seed(4)
A = torch.rand(nb, n, n, device="cuda", generator=g) * 2 - 1
B = torch.rand(nb, n, n, device="cuda", generator=g) * 2 - 1
C = torch.zeros(nb, n, n, device="cuda")


def step(v):
    if v < 0:
        hip.gemmStridedBatched(False, False, n, n, n, 1.0, A, 0, n, n * n, B, 0, n, n * n, 0.0, C, 0,
                               n, n * n, nb)
    else:
        hip.gemmVariant(v, False, False, n, n, n, 1.0, A, 0, n, n * n, B, 0, n, n * n, 0.0, C, 0, n,
                        n * n, nb)


res = {}
for r in range(a.rounds):
    for v in vs:
        name = "default" if v < 0 else names[v]
        try:
            step(v)
        except Exception as e:  # noqa: BLE001
            res[name] = {"error": str(e)[:120]}
            continue
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            step(v)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        sha = hashlib.sha1(C[::97].cpu().numpy().tobytes()).hexdigest()[:10]
        res.setdefault(name, {"ms": [], "sha": sha})["ms"].append(round(ms, 3))
for k, v in res.items():
    if "ms" in v:
        v["tflops"] = round(2.0 * n ** 3 * nb / min(v["ms"]) / 1e9, 1)
        v["frac"] = round(v["tflops"] / 157.3, 4)
print(json.dumps(res))
