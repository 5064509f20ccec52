#!/usr/bin/env python3
"""Tile-shape sweep for the MFMA SGEMM (interleaved rounds in one process,
methodology rule 24).  Writes gpurun_out/sgemm_sweep.json.

  python scripts/sgemm_sweep.py [--sizes 4096,2048] [--yolo] [--rounds 5]
      [--tn "M,N,K,batch;..."]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402


_warned = set()


def time_variant(hip, v, prob, reps):
    M, N, K, batch, A, B, C = prob[:7]
    if len(prob) > 7:  # TN: A stored K x M (conv backward's W^T . delta), shared
        call = lambda: hip.gemmVariant(v, True, False, M, N, K, 1.0, A, 0, M, 0, B, 0, N,  # noqa
                                       K * N, 0.0, C, 0, N, M * N, batch)
        return _time(call, v, reps)
    sA = M * K if A.dim() == 3 else 0  # batched: own A per GEMM; yolo: shared weights
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        hip.gemmVariant(v, False, False, M, N, K, 1.0, A, 0, K, sA, B, 0, N,
                        K * N, 0.0, C, 0, N, M * N, batch)
    except Exception as e:
        if v not in _warned:
            _warned.add(v)
            print(f"variant {v}: {e}", flush=True)
        return None
    torch.cuda.synchronize()
    ev0.record()
    for _ in range(reps):
        hip.gemmVariant(v, False, False, M, N, K, 1.0, A, 0, K, sA, B, 0, N, K * N, 0.0, C, 0, N,
                        M * N, batch)
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / reps


def _time(call, v, reps):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        call()
    except Exception as e:
        if v not in _warned:
            _warned.add(v)
            print(f"variant {v}: {e}", flush=True)
        return None
    torch.cuda.synchronize()
    ev0.record()
    for _ in range(reps):
        call()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096")
    ap.add_argument("--yolo", action="store_true")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="")
    ap.add_argument("--batched", default="", help="n:batch strided-batched n^3 GEMMs")
    ap.add_argument("--shapes", default="", help="M,N,K[;M,N,K...] plain NN GEMMs")
    ap.add_argument("--tn", default="", help="M,N,K,batch[;...] TN GEMMs, shared A")
    args = ap.parse_args()
    hip = TNNHip(0)
    names = TNNHip.gemmVariants()
    vs = [int(x) for x in args.variants.split(",")] if args.variants else list(range(len(names)))
    probs = {}
    for n in [int(s) for s in args.sizes.split(",") if s]:
        A = torch.rand(n, n, device="cuda") * 2 - 1
        B = torch.rand(n, n, device="cuda") * 2 - 1
        C = torch.zeros(n, n, device="cuda")
        probs[f"sq{n}"] = (n, n, n, 1, A, B, C)
    for shp in [x for x in args.shapes.split(";") if x]:
        M, N, K = (int(v) for v in shp.split(","))
        A = torch.rand(M, K, device="cuda") * 2 - 1
        B = torch.rand(K, N, device="cuda") * 2 - 1
        C = torch.zeros(M, N, device="cuda")
        probs[f"g{M}x{N}x{K}"] = (M, N, K, 1, A, B, C)
    for shp in [x for x in args.tn.split(";") if x]:
        M, N, K, nb = (int(v) for v in shp.split(","))
        A = torch.rand(K, M, device="cuda") * 0.2 - 0.1
        B = torch.rand(nb, K, N, device="cuda") * 2 - 1
        C = torch.zeros(nb, M, N, device="cuda")
        probs[f"tn{M}x{N}x{K}b{nb}"] = (M, N, K, nb, A, B, C, "tn")
    if args.batched:
        n, nb = (int(v) for v in args.batched.split(":"))
        A = torch.rand(nb, n, n, device="cuda") * 2 - 1
        B = torch.rand(nb, n, n, device="cuda") * 2 - 1
        C = torch.zeros(nb, n, n, device="cuda")
        probs[f"batched{n}x{nb}"] = (n, n, n, nb, A, B, C)
    if args.yolo:
        seen = set()
        for s in yolov3_conv_table():
            key = (s.M, s.N, s.K)
            if key in seen:
                continue
            seen.add(key)
            A = torch.rand(s.M, s.K, device="cuda") * 0.2 - 0.1
            B = torch.rand(8, s.K, s.N, device="cuda")
            C = torch.zeros(8, s.M, s.N, device="cuda")
            probs[f"yolo_{s.M}x{s.N}x{s.K}"] = (s.M, s.N, s.K, 8, A, B, C)
    res = {p: {names[v]: [] for v in vs} for p in probs}
    res_h = {p: [] for p in probs}
    for r in range(args.rounds):
        for p, prob in probs.items():
            M, N, K, batch = prob[:4]
            reps = max(3, min(50, int(2e11 / (2 * M * N * K * batch))))
            t = time_variant(hip, -1, prob, reps)
            res_h[p].append(t)
            for v in vs:
                t = time_variant(hip, v, prob, reps)
                if t is not None:
                    res[p][names[v]].append(t)
    out = {}
    for p, prob in probs.items():
        M, N, K, batch = prob[:4]
        flop = 2.0 * M * N * K * batch
        row = {"heuristic": None}
        if res_h[p] and res_h[p][0] is not None:
            ms = float(np.median(res_h[p]))
            row["heuristic"] = {"ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 2)}
        for name, ts in res[p].items():
            if ts:
                ms = float(np.median(ts))
                row[name] = {"ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 2),
                             "min_ms": round(float(np.min(ts)), 4)}
        out[p] = row
        best = max(((k, v["tflops"]) for k, v in row.items() if v), key=lambda kv: kv[1])
        print(f"{p:28s} heuristic={row['heuristic']}  best={best}", flush=True)
    Path("gpurun_out").mkdir(exist_ok=True)
    Path("gpurun_out/sgemm_sweep.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
