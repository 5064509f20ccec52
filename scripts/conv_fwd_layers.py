#!/usr/bin/env python3
"""Per-layer YOLOv3-416 conv forward at batch 8 (the bench's `yolo` field,
TConvolutionalLayer.forward after fuseBatchNorm: nConvolutionLayer.pas:457-569),
each layer timed alone with HIP events on the driver's stream.  One JSON line:
per layer the shape, ms, TFLOP/s and its share of the sum; run under
`rocprofv3 --kernel-trace --stats` for the kernel (tile) each layer launches.

  python scripts/conv_fwd_layers.py [--batch 8] [--reps 10]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--pad", type=int, default=-1, help="TNS_OPT_CONV_PAD (-1: heuristic)")
    ap.add_argument("--variant", type=int, default=-1, help="TNS_OPT_CONV_VARIANT (-1: heuristic)")
    ap.add_argument("--layers", default="", help="comma-separated layer indices (default: all)")
    ap.add_argument("--warm-ms", type=float, default=0.0,
                    help="run each layer back-to-back this long before timing it")
    a = ap.parse_args()
    hip = TNNHip(0)
    hip.setConvPad(a.pad)
    hip.setConvVariant(a.variant)
    only = {int(v) for v in a.layers.split(",") if v}
    rows, total = [], 0.0
    for s in yolov3_conv_table():
        if only and s.index not in only:
            continue
        x = torch.rand(a.batch, s.c, s.h, s.h, device="cuda")
        w = torch.rand(s.filters, s.K, device="cuda") * 0.2 - 0.1
        b = torch.rand(s.filters, device="cuda") * 0.2 - 0.1
        ws = torch.empty(a.batch * s.K * s.N if s.needs_im2col else 1, device="cuda")
        out = torch.empty(a.batch, s.filters, s.N, device="cuda")
        run = lambda: hip.convForward(a.batch, s.c, s.h, s.h, x, w, b, s.filters, s.size,  # noqa
                                      s.stride, s.pad, 1, s.activation, ws, out)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        if a.warm_ms > 0:  # hold the GPU busy first: the clock ramps over ~20 ms of load
            t_end = time.perf_counter() + a.warm_ms / 1e3
            while time.perf_counter() < t_end:
                for _ in range(10):
                    run()
                torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        total += ms
        gf = s.flops * a.batch / 1e9
        rows.append({"layer": s.index, "shape": f"{s.c}x{s.h} k{s.size}s{s.stride}->{s.filters}",
                     "M": s.M, "N": s.N * a.batch, "K": s.K, "ms": round(ms, 4),
                     "tflops": round(gf / ms, 1)})
    for r in rows:
        r["share"] = round(r["ms"] / total, 4)
    print(json.dumps({"batch": a.batch, "sum_ms": round(total, 3), "layers": rows}))


if __name__ == "__main__":
    main()
