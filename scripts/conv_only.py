#!/usr/bin/env python3
"""Run one YOLOv3 conv layer repeatedly (for rocprofv3 counter passes)."""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layer", type=int, default=45)
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--mode", type=int, default=3)
ap.add_argument("--variant", type=int, default=-1)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
s = yolov3_conv_table()[a.layer]
hip = TNNHip(0)
x = torch.rand(a.batch, s.c, s.h, s.h, device="cuda")
w = torch.rand(s.filters, s.K, device="cuda") * 0.2 - 0.1
b = torch.rand(s.filters, device="cuda") * 0.2 - 0.1
ws = torch.empty(a.batch * s.K * s.N, device="cuda")
out = torch.empty(a.batch, s.filters, s.N, device="cuda")
hip.setConvVariant(a.variant)
for _ in range(a.reps):
    hip.convForward(a.batch, s.c, s.h, s.h, x, w, b, s.filters, s.size, s.stride, s.pad, 1,
                    s.activation, ws, out, fused=a.mode)
hip.finish()
print("done", s)
