#!/usr/bin/env python3
"""YOLOv3-416 batch-8 training backward as the drop-in runs it
(darknet.HipDarknetTrain, bench.py's yolo_train_backward) for a kernel trace:
one training forward, then --passes backward passes (deltas reset between
them), pipelined (TNS_OPT_BWD_OVERLAP = 2) unless --joined.

  rocprofv3 --kernel-trace --stats -- python3 scripts/train_bwd_once.py
"""
import argparse
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd import darknet as dn  # noqa: E402
from tensorium_amd.nnhip import TNNHip  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--passes", type=int, default=3)
ap.add_argument("--joined", action="store_true")
a = ap.parse_args()
hip = TNNHip(0)
net = dn.Network(dn.parse_cfg(dn.yolov3_cfg(416)), 8)
model = dn.HipDarknetTrain(hip, net, dn.random_params(net, seed=3), torch)
g = torch.Generator(device="cuda").manual_seed(7)
x = torch.rand(8, 3, 416, 416, device="cuda", generator=g)
model.forward(x)
yd = [torch.rand(8 * l.out_size, device="cuda", generator=g) * 0.2 - 0.1
      for l in net.layers if l.kind == "yolo"]
hip.setBwdOverlap(1 if a.joined else 2)
for p in range(a.passes + 1):
    hip.finish()
    for d in model.delta:
        d.zero_()
    model.set_yolo_deltas(yd)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.backward(x)
    hip.finish()
    torch.cuda.synchronize()
    print(f"pass {p}: {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)
