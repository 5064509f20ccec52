#!/usr/bin/env python3
"""The bench's 75-layer YOLOv3 conv backward (batch 8, bench.py
bench_conv_backward) timed five ways: per-call launches with the dW / dX
overlap on (1), off (0) and pipelined (2: each dW left on the side stream),
and the same call sequence captured once into a HIP graph and replayed
(overlap 1 / 0).  The graph replays the very kernels the calls
launch, with the same arguments; the replay's weight_updates, bias_updates
and state.delta are checked bit-identical to the per-call pass from the same
starting state.  One JSON line.

  python scripts/bwd_graph.py [--steps 5] [--rounds 3]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    cap = torch.cuda.Stream()
    hip = TNNHip(0, stream=cap.cuda_stream)
    specs = yolov3_conv_table()
    B = 8
    gen = torch.Generator(device="cuda")
    layers, max_ws = [], 0
    for s in specs:
        gen.manual_seed(7000 + s.index)
        x = torch.rand(B, s.c, s.h, s.h, device="cuda", generator=gen)
        sc = float(np.sqrt(2.0 / (s.size * s.size * s.c)))
        w = (torch.rand(s.filters, s.K, device="cuda", generator=gen) * 2 - 1) * sc
        out = torch.rand(B, s.filters, s.out_h, s.out_h, device="cuda", generator=gen) * 2 - 1
        delta = torch.rand(B, s.filters, s.out_h, s.out_h, device="cuda", generator=gen) * 2 - 1
        bu = torch.zeros(s.filters, device="cuda")
        wu = torch.zeros(s.filters, s.K, device="cuda")
        sd = torch.zeros(B, s.c, s.h, s.h, device="cuda") if s.index > 0 else None
        layers.append([s, x, w, out, delta, bu, wu, sd])
        max_ws = max(max_ws, B * s.K * s.out_h * s.out_h)
    ws = torch.empty(max_ws, device="cuda")

    def step():
        for s, x, w, out, delta, bu, wu, sd in layers:
            hip.convBackward(B, s.c, s.h, s.h, x, w, s.filters, s.size, s.stride, s.pad, 1,
                             s.activation, out, delta, bu, wu, ws, sd)

    def state():
        return [[t.clone() for t in L[4:] if t is not None] for L in layers]

    def restore(snap):
        for L, sv in zip(layers, snap):
            for t, v in zip([t for t in L[4:] if t is not None], sv):
                t.copy_(v)

    def timed(fn, join=False):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cap)
        for _ in range(a.steps):
            fn()
        if join:  # the pipelined schedule's last dW products inside the region
            hip.finish()
        e1.record(cap)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.steps

    row = {"layers": len(specs), "batch": B, "steps": a.steps}
    with torch.cuda.stream(cap):
        for ov in (1, 0, 2):  # every scratch buffer and the side stream exist
            hip.setBwdOverlap(ov)
            step()
            hip.finish()
        torch.cuda.synchronize()
        graphs = {}
        for ov in (True, False):
            hip.setBwdOverlap(ov)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap):
                step()
            graphs[ov] = g
        torch.cuda.synchronize()
        # bit-identity of the replay against the per-call pass
        snap = state()
        hip.setBwdOverlap(True)
        step()
        torch.cuda.synchronize()
        ref = state()
        for ov in (True, False):
            restore(snap)
            graphs[ov].replay()
            torch.cuda.synchronize()
            got = state()
            same = all(torch.equal(p, q) for r1, r2 in zip(ref, got) for p, q in zip(r1, r2))
            row[f"graph_overlap{int(ov)}_bit_identical"] = bool(same)
        # the pipelined schedule (2) per call against the same reference
        restore(snap)
        hip.setBwdOverlap(2)
        step()
        hip.finish()
        torch.cuda.synchronize()
        got = state()
        row["calls_overlap2_bit_identical"] = bool(
            all(torch.equal(p, q) for r1, r2 in zip(ref, got) for p, q in zip(r1, r2)))
        times = {k: [] for k in ("calls_overlap1", "calls_overlap0", "calls_overlap2",
                                 "calls_overlap2_derive_fused", "graph_overlap1",
                                 "graph_overlap0")}
        for _ in range(a.rounds):
            for ov in (True, False):
                hip.setBwdOverlap(ov)
                times[f"calls_overlap{int(ov)}"].append(timed(step))
                times[f"graph_overlap{int(ov)}"].append(timed(graphs[ov].replay))
            hip.setBwdOverlap(2)
            times["calls_overlap2"].append(timed(step, join=True))
            hip.setDeriveSums(True)
            times["calls_overlap2_derive_fused"].append(timed(step, join=True))
            hip.setDeriveSums(False)
        hip.setBwdOverlap(True)
    for k, v in times.items():
        row[k + "_ms"] = round(min(v), 3)
        row[k + "_all"] = [round(t, 3) for t in v]
    print(json.dumps(row))


if __name__ == "__main__":
    main()
