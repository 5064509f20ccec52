#!/usr/bin/env python3
"""Compact perf probe for A/B runs of alternative builds (TNS_LIB=...):
SGEMM 4096^3 NN (median kernel ms), 256 x 1024^3 strided-batched GEMMs, and
the YOLOv3 conv-forward batch (ms per distinct layer x count).  One JSON line.

  TNS_LIB=ab/x/libtensorium_hip.so python scripts/quick_perf.py [--tag x]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ts]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default=os.environ.get("TNS_LIB", "tree"))
    ap.add_argument("--yolo-only", action="store_true")
    args = ap.parse_args()
    hip = TNNHip(0)
    res = {"tag": args.tag}
    if not args.yolo_only:
        n = 4096
        A = torch.rand(n, n, device="cuda") * 2 - 1
        B = torch.rand(n, n, device="cuda") * 2 - 1
        C = torch.empty(n, n, device="cuda")
        ms = timed(lambda: hip.gemm(False, False, n, n, n, 1.0, A, 0, n, B, 0, n, 0.0, C, 0, n), 30)
        res["sgemm4096_ms"] = round(ms, 4)
        res["sgemm4096_tflops"] = round(2 * n ** 3 / ms / 1e9, 2)
        del A, B, C
        nb, m = 256, 1024
        A = torch.rand(nb, m, m, device="cuda") * 2 - 1
        B = torch.rand(nb, m, m, device="cuda") * 2 - 1
        C = torch.empty(nb, m, m, device="cuda")
        ms = timed(lambda: hip.gemmStridedBatched(False, False, m, m, m, 1.0, A, 0, m, m * m, B, 0,
                                                  m, m * m, 0.0, C, 0, m, m * m, nb), 5)
        res["batched_tflops"] = round(2 * m ** 3 * nb / ms / 1e9, 2)
        del A, B, C
        torch.cuda.empty_cache()
    batch = 8
    layers, seen = [], {}
    for s in yolov3_conv_table():
        key = (s.c, s.h, s.filters, s.size, s.stride)
        seen[key] = seen.get(key, 0) + 1
        if seen[key] > 1:
            continue
        x = torch.rand(batch, s.c, s.h, s.h, device="cuda")
        w = torch.rand(s.filters, s.K, device="cuda") * 0.2 - 0.1
        b = torch.rand(s.filters, device="cuda") * 0.2 - 0.1
        out = torch.empty(batch, s.filters, s.N, device="cuda")
        layers.append((key, s, x, w, b, out))
    total, per = 0.0, {}
    for key, s, x, w, b, out in layers:
        ms = timed(lambda: hip.convForward(batch, s.c, s.h, s.h, x, w, b, s.filters, s.size,
                                           s.stride, s.pad, 1, s.activation, None, out, fused=True),
                   10)
        per[f"L{s.index}"] = round(ms, 4)
        total += ms * seen[key]
    flop = sum(s.flops for s in yolov3_conv_table()) * batch
    res["yolo_ms"] = round(total, 3)
    res["yolo_tflops"] = round(flop / total / 1e9, 2)
    res["yolo_layers_ms"] = per
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
