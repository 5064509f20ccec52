#!/usr/bin/env python3
"""Conv backward without state.delta (derive, bias sums, im2col, dW) per
unique YOLOv3 batch-8 layer shape under each sdot form (TNS_OPT_SDOT_FORM:
-1 by shape, 0 the one-class-per-wave MFMA kernel, 64 + v the
residue-register forms).  HIP-event time of the whole call, so the batched
forms' in-order accumulate pass is included.  One JSON line.

  python scripts/dw_forms.py [--forms -1,64,65] [--layers 11,28,45]
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

ap = argparse.ArgumentParser()
ap.add_argument("--forms", default="")
ap.add_argument("--layers", default="")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
hip = TNNHip(0)
forms = [int(t) for t in a.forms.split(",")] if a.forms else \
    [-1, 0] + [64 + v for v in range(hip.sdotRcVariants())]
batch = 8
seen, rows = set(), []
for s in yolov3_conv_table():
    key = (s.c, s.h, s.size, s.stride, s.filters)
    if a.layers and str(s.index) not in a.layers.split(","):
        continue
    if not a.layers and key in seen:
        continue
    seen.add(key)
    x = torch.rand(batch, s.c, s.h, s.h, device="cuda")
    w = torch.rand(s.filters, s.K, device="cuda") * 0.1
    o = torch.rand(batch, s.filters, s.out_h, s.out_h, device="cuda")
    d = torch.rand_like(o)
    bu, wu = torch.zeros(s.filters, device="cuda"), torch.zeros(s.filters, s.K, device="cuda")
    run = lambda: hip.convBackward(batch, s.c, s.h, s.h, x, w, s.filters, s.size, s.stride,  # noqa
                                   s.pad, 1, s.activation, o, d, bu, wu, None, None)
    res = {}
    for f in forms:
        hip.setSdotForm(f)
        try:
            run()
        except TnsError:
            continue
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / a.reps)
        res[str(f)] = round(best, 4)
    hip.setSdotForm(-1)
    rows.append({"layer": s.index, "shape": f"{s.c}x{s.h} k{s.size}s{s.stride}->{s.filters}",
                 "ms": res, "best": min(res, key=res.get)})
    print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
print(json.dumps(rows))
