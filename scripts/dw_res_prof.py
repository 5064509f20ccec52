#!/usr/bin/env python3
"""Time the conv backward's dW forms on one YOLOv3 layer (batch 8, no
state.delta, so the call is derive + bias + dW only): every residue-
sequential form (dw_res.hip), the implicit-im2col tiles and the default
pick, each call timed by HIP events after a warm-up.  Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split.  One JSON line.

  python scripts/dw_res_prof.py --layer 11 [--reps 10]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd._abi import TnsError  # noqa: E402
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", type=int, default=11)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    hip = TNNHip(0)
    s = yolov3_conv_table()[a.layer]
    B = 8
    x = torch.rand(B, s.c, s.h, s.h, device="cuda")
    w = torch.rand(s.filters, s.K, device="cuda") * 0.1
    o = torch.rand(B, s.filters, s.out_h, s.out_h, device="cuda")
    d = torch.rand_like(o)
    bu, wu = torch.zeros(s.filters, device="cuda"), torch.zeros(s.filters, s.K, device="cuda")

    def timed():
        def run():
            hip.convBackward(B, s.c, s.h, s.h, x, w, s.filters, s.size, s.stride, s.pad, 1,
                             s.activation, o, d, bu, wu)
        run()
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / a.reps, 4)

    # a warm clock before the first timed form (~100 ms of the default)
    for _ in range(100):
        hip.convBackward(B, s.c, s.h, s.h, x, w, s.filters, s.size, s.stride, s.pad, 1,
                         s.activation, o, d, bu, wu)
    torch.cuda.synchronize()
    row = {"layer": a.layer, "shape": f"{s.c}x{s.h} k{s.size}s{s.stride}->{s.filters}"}
    try:
        hip.setDwRes(-2)
        row["off"] = timed()
    finally:
        hip.setDwRes(-1)
    row["default"] = timed()
    for v in range(hip.convDwRes()):
        try:
            hip.setDwRes(v)
            row[f"dwres{v}"] = timed()
        except TnsError:
            pass
        finally:
            hip.setDwRes(-1)
    print(json.dumps(row))


if __name__ == "__main__":
    main()
