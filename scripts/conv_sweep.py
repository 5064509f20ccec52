#!/usr/bin/env python3
"""Per-layer conv schedule sweep over the YOLOv3 conv table at batch B:
im2col + fused-epilogue SGEMM (schedule 2) vs implicit GEMM (schedule 3) for
every implicit tile shape.  Interleaved rounds in one process.  Writes
gpurun_out/conv_sweep.json.

  python scripts/conv_sweep.py [--batch 8] [--rounds 3]
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

IMPLICIT_VARIANTS = [int(v) for v in __import__('os').environ.get('CONV_VARIANTS', '6,12,13,14,15,18,19,20,21,22').split(',')]


def time_conv(hip, layer, mode, variant, reps, pad=-1):
    s, x, w, b, ws, out, batch = layer
    hip.setConvVariant(variant)
    hip.setConvPad(pad)
    run = lambda: hip.convForward(batch, s.c, s.h, s.h, x, w, b, s.filters, s.size, s.stride,
                                  s.pad, 1, s.activation, ws, out, fused=mode)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    hip.setConvVariant(-1)
    hip.setConvPad(-1)
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    hip = TNNHip(0)
    names = TNNHip.gemmVariants()
    layers, seen = {}, set()
    for s in yolov3_conv_table():
        key = (s.c, s.h, s.filters, s.size, s.stride)
        if key in seen:
            continue
        seen.add(key)
        x = torch.rand(args.batch, s.c, s.h, s.h, device="cuda")
        w = torch.rand(s.filters, s.K, device="cuda") * 0.2 - 0.1
        b = torch.rand(s.filters, device="cuda") * 0.2 - 0.1
        ws = torch.empty(args.batch * s.K * s.N, device="cuda")
        out = torch.empty(args.batch, s.filters, s.N, device="cuda")
        layers[f"L{s.index}_c{s.c}_h{s.h}_f{s.filters}_k{s.size}s{s.stride}"] = (
            (s, x, w, b, ws, out, args.batch), s)
    cfgs = [("im2col", 2, -1, -1), ("implicit_auto", 3, -1, -1)] + \
        [(f"implicit_{names[v]}", 3, v, -1) for v in IMPLICIT_VARIANTS]
    res = {k: {c[0]: [] for c in cfgs} for k in layers}
    for _ in range(args.rounds):
        for k, (layer, s) in layers.items():
            flop = 2.0 * s.M * s.N * s.K * args.batch
            reps = max(3, min(40, int(2e10 / flop)))
            for name, mode, v, pad in cfgs:
                res[k][name].append(time_conv(hip, layer, mode, v, reps, pad))
    out = {}
    tot = {c[0]: 0.0 for c in cfgs}
    best_tot = 0.0
    for k, (layer, s) in layers.items():
        flop = 2.0 * s.M * s.N * s.K * args.batch
        row = {n: {"ms": round(float(np.median(ts)), 4),
                   "tflops": round(flop / float(np.median(ts)) / 1e9, 2)}
               for n, ts in res[k].items()}
        cnt = sum(1 for t in yolov3_conv_table()
                  if (t.c, t.h, t.filters, t.size, t.stride) == (s.c, s.h, s.filters, s.size,
                                                                   s.stride))
        row["count"] = cnt
        for n in tot:
            tot[n] += row[n]["ms"] * cnt
        best = min(((n, v["ms"]) for n, v in row.items() if n != "count"), key=lambda t: t[1])
        best_tot += best[1] * cnt
        out[k] = row
        print(f"{k:34s} x{cnt} im2col={row['im2col']['ms']:.4f} "
              f"auto={row['implicit_auto']['ms']:.4f} best={best}", flush=True)
    out["_totals_ms"] = {**{n: round(v, 3) for n, v in tot.items()}, "best": round(best_tot, 3)}
    print(json.dumps(out["_totals_ms"]), flush=True)
    Path("gpurun_out").mkdir(exist_ok=True)
    Path("gpurun_out/conv_sweep.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
