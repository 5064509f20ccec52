#!/usr/bin/env python3
"""HBM rates of the elementwise kernels on the YOLOv3-416 batch-8 layer
shapes: im2col (strided batched), bias add (forwardBias) and leaky
activation (ActivateArray), each timed alone with HIP events over repeated
launches on the kernel's stream.  Algorithmic bytes: im2col reads the images
and writes the col matrix; bias and activation read and write every output
element.  One JSON line to stdout.

  python scripts/elementwise_perf.py
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402
from nt_perf import timed  # noqa: E402


def main():
    hip = TNNHip(0)
    batch = 8
    specs = yolov3_conv_table()
    rows = []
    tot = {"im2col": [0.0, 0.0], "col2im": [0.0, 0.0], "bias": [0.0, 0.0],
           "leaky": [0.0, 0.0]}
    col = torch.empty(max(s.col_elems for s in specs) * batch, device="cuda")
    for s in specs:
        x = torch.rand(batch * s.c * s.h * s.h, device="cuda")
        out = torch.rand(batch * s.filters * s.out_h * s.out_h, device="cuda")
        b = torch.rand(s.filters, device="cuda")
        row = {"layer": s.index, "shape": f"{s.c}x{s.h}x{s.h} k{s.size}s{s.stride}->{s.filters}"}
        if s.needs_im2col:
            ms = timed(lambda: hip.im2colStridedBatched(
                s.c, s.h, s.h, s.size, s.size, s.pad, s.pad, s.stride, s.stride, 1, 1, x,
                s.c * s.h * s.h, 0, col, s.col_elems, 0, batch), 10)
            by = (s.col_elems + s.c * s.h * s.h) * batch * 4
            row["im2col_gbs"] = round(by / ms / 1e6, 1)
            tot["im2col"][0] += by
            tot["im2col"][1] += ms
            # col2im: reads the col matrix, reads and writes the image
            ms = timed(lambda: hip.col2imStridedBatched(
                s.c, s.h, s.h, s.size, s.size, s.pad, s.pad, s.stride, s.stride, 1, 1, col,
                s.col_elems, 0, x, s.c * s.h * s.h, 0, batch), 10)
            by = (s.col_elems + 2 * s.c * s.h * s.h) * batch * 4
            row["col2im_gbs"] = round(by / ms / 1e6, 1)
            tot["col2im"][0] += by
            tot["col2im"][1] += ms
        by = 2 * out.numel() * 4
        ms = timed(lambda: hip.forwardBias(out.numel(), out, 0, s.filters, b, 1, batch), 10)
        row["bias_gbs"] = round(by / ms / 1e6, 1)
        tot["bias"][0] += by
        tot["bias"][1] += ms
        ms = timed(lambda: hip.ActivateArray(out.numel(), out, 0, 9), 10)  # LEAKY
        row["leaky_gbs"] = round(by / ms / 1e6, 1)
        tot["leaky"][0] += by
        tot["leaky"][1] += ms
        rows.append(row)
        del x, out
    res = {k: {"bytes": v[0], "ms": round(v[1], 4), "gbs": round(v[0] / v[1] / 1e6, 1)}
           for k, v in tot.items()}
    big = sorted(rows, key=lambda r: -r.get("im2col_gbs", 0))[:3]
    print(json.dumps({"totals_batch8": res, "layers": rows, "best_im2col_layers": big}))


if __name__ == "__main__":
    main()
