#!/usr/bin/env python3
"""Run one YOLOv3-416 conv layer's backward (batch 8, with state.delta) a few
times — the command the r04 counter passes profile (scripts/gpu_r4_evidence.sh).

  python scripts/conv_bwd_one.py --layer 11 [--reps 5]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layer", type=int, default=11)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
hip = TNNHip(0)
s = yolov3_conv_table()[a.layer]
B = 8
x = torch.rand(B, s.c, s.h, s.h, device="cuda")
w = torch.rand(s.filters, s.K, device="cuda") * 0.2 - 0.1
out = torch.rand(B, s.filters, s.out_h, s.out_h, device="cuda") * 2 - 1
delta = torch.rand(B, s.filters, s.out_h, s.out_h, device="cuda") * 2 - 1
bu = torch.zeros(s.filters, device="cuda")
wu = torch.zeros(s.filters, s.K, device="cuda")
sd = torch.zeros(B, s.c, s.h, s.h, device="cuda")
ws = torch.empty(max(B * s.K * s.out_h * s.out_h, 1), device="cuda")
for _ in range(a.reps):
    hip.convBackward(B, s.c, s.h, s.h, x, w, s.filters, s.size, s.stride, s.pad, 1, s.activation,
                     out, delta, bu, wu, ws, sd)
torch.cuda.synchronize()
print("ok", a.layer)
