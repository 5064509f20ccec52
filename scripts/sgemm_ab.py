#!/usr/bin/env python3
"""Interleaved A/B of the 4096^3 NN SGEMM between library builds (each run in
its own process with TNS_LIB pointing at one build, rounds alternating):
kernel mean by HIP events over 50 launches after 30 warm-up, and a checksum
of C (the builds must agree bit for bit).

  python scripts/sgemm_ab.py [--rounds 4] lib_a.so lib_b.so ...
"""
import argparse
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

CHILD = r"""
import sys, json, torch, hashlib
sys.path.insert(0, %r)
from tensorium_amd.nnhip import TNNHip
n = %d
hip = TNNHip(0)
g = torch.Generator(device="cuda").manual_seed(7)
A = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
B = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
C = torch.zeros(n, n, device="cuda")
run = lambda: hip.gemm(False, False, n, n, n, 1.0, A, 0, n, B, 0, n, 0.0, C, 0, n)
for _ in range(30): run()
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
for a, b in ev:
    a.record(); run(); b.record()
torch.cuda.synchronize()
ms = sorted(a.elapsed_time(b) for a, b in ev)
h = hashlib.sha1(C.cpu().numpy().tobytes()).hexdigest()[:12]
print(json.dumps({"mean_ms": sum(ms) / len(ms), "median_ms": ms[len(ms) // 2], "sha": h}))
"""

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("libs", nargs="+")
a = ap.parse_args()
res = {l: [] for l in a.libs}
for r in range(a.rounds):
    for lib in a.libs:
        env = dict(os.environ, TNS_LIB=str(Path(lib).resolve()))
        out = subprocess.run([sys.executable, "-c", CHILD % (str(ROOT), a.n)], env=env,
                             capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(out.stderr[-2000:], file=sys.stderr)
            sys.exit(1)
        res[lib].append(json.loads(out.stdout.strip().splitlines()[-1]))
print(json.dumps({lib: {"mean_ms": [round(x["mean_ms"], 4) for x in v],
                        "sha": sorted({x["sha"] for x in v})} for lib, v in res.items()}))
