#!/usr/bin/env python3
"""bench.py's yolo leg (75 conv layers, batch 8, independent synthetic inputs)
for a kernel trace: --steps passes after --warmup, wall time per pass printed.
  rocprofv3 --kernel-trace --output-format csv -- python3 scripts/yolo_fwd_once.py"""
import argparse
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--per-layer", action="store_true", help="HIP events around every layer (in sequence)")
a = ap.parse_args()
hip = TNNHip(0)
batch, layers, mx = 8, [], 1
for s in yolov3_conv_table():
    x = torch.rand(batch, s.c, s.h, s.h, device="cuda")
    w = (torch.rand(s.filters, s.K, device="cuda") * 2 - 1) * (2.0 / s.K) ** 0.5
    b = torch.rand(s.filters, device="cuda") * 0.2 - 0.1
    layers.append((s, x, w, b, torch.empty(batch, s.filters, s.out_h, s.out_h, device="cuda")))
    mx = max(mx, batch * s.col_elems)
ws = torch.empty(mx, device="cuda")


def step():
    for s, x, w, b, out in layers:
        hip.convForward(batch, s.c, s.h, s.h, x, w, b, s.filters, s.size, s.stride, s.pad, 1,
                        s.activation, ws, out, fused=True)


if a.per_layer:
    import json
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(layers) + 1)]
    acc = [0.0] * len(layers)
    for rep in range(a.warmup + a.steps):
        ev[0].record()
        for j, (s, x, w, b, out) in enumerate(layers):
            hip.convForward(batch, s.c, s.h, s.h, x, w, b, s.filters, s.size, s.stride, s.pad, 1,
                            s.activation, ws, out, fused=True)
            ev[j + 1].record()
        torch.cuda.synchronize()
        if rep >= a.warmup:
            for j in range(len(layers)):
                acc[j] += ev[j].elapsed_time(ev[j + 1]) / a.steps
    print(json.dumps({"sum_ms": round(sum(acc), 4),
                      "layers": [[s.index, round(t, 4)] for (s, *_), t in zip(layers, acc)]}))
    sys.exit(0)
for _ in range(a.warmup):
    step()
torch.cuda.synchronize()
for i in range(a.steps):
    time.sleep(0.005)  # (a gap between passes in the trace)
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    print(f"pass {i}: {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)
