#!/usr/bin/env python3
"""A/B of the large-NN SGEMM variants at one size: interleaved rounds of
warm-up + timed launches (HIP events), outputs compared bit for bit.

  python scripts/nn_big_ab.py [--n 4096] [--rounds 5] [--variants 0,3]
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
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--variants", default="0,3")
a = ap.parse_args()
hip = TNNHip(0)
names = TNNHip.gemmVariants()
base = [i for i, nm in enumerate(names) if nm.endswith("nn_big")][0]
vs = [base + int(v) for v in a.variants.split(",")]
n = a.n
g = torch.Generator(device="cuda").manual_seed(1)
A = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
B = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
outs = {}
res = {names[v]: [] for v in vs}


def run(v, C):
    hip.gemmVariant(v, False, False, n, n, n, 1.0, A, 0, n, 0, B, 0, n, 0, 0.0, C, 0, n, 0)


for v in vs:
    C = torch.zeros(n, n, device="cuda")
    run(v, C)
    torch.cuda.synchronize()
    outs[v] = C
for r in range(a.rounds):
    for v in vs:
        C = outs[v]
        for _ in range(30):
            run(v, C)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run(v, C)
        e1.record()
        torch.cuda.synchronize()
        res[names[v]].append(e0.elapsed_time(e1) / a.reps)
ref = outs[vs[0]]
out = {}
for v in vs:
    ms = sorted(res[names[v]])
    out[names[v]] = {"ms_median": ms[len(ms) // 2], "ms_min": ms[0],
                     "tflops_median": 2 * n ** 3 / ms[len(ms) // 2] / 1e9,
                     "bit_exact_vs_first": bool(torch.equal(outs[v], ref))}
print(json.dumps(out, indent=1))
