#!/usr/bin/env python3
"""Time one YOLOv3 conv layer shape (batch 8) under forced conv variants.

  TNS_LIB=... python scripts/conv_one.py --layer 11 --variants -1,100,300
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
ap.add_argument("--layer", type=int, default=11)
ap.add_argument("--variants", default="-1,100,300")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
hip = TNNHip(0)
s = yolov3_conv_table()[a.layer]
x = torch.rand(8, s.c, s.h, s.h, device="cuda")
w = torch.rand(s.filters, s.K, device="cuda") * 0.2 - 0.1
b = torch.rand(s.filters, device="cuda") * 0.2 - 0.1
out = torch.empty(8, s.filters, s.N, device="cuda")
res = {}
for _ in range(a.rounds):
    for v in [int(t) for t in a.variants.split(",")]:
        hip.setConvVariant(v)
        run = lambda: hip.convForward(8, s.c, s.h, s.h, x, w, b, s.filters, s.size, s.stride,  # noqa
                                      s.pad, 1, s.activation, None, out)
        try:
            run()
        except TnsError:
            continue
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(v, []).append(e0.elapsed_time(e1) / a.reps)
hip.setConvVariant(-1)
gf = s.flops * 8 / 1e9
print(json.dumps({str(v): {"ms": round(min(t), 4), "tf": round(gf / min(t), 1)} for v, t in res.items()}))
