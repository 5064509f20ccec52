#!/usr/bin/env python3
"""Per-layer split of the YOLOv3 batch-8 conv backward (telemetry: GEMM =
dW sdot batch + dX TN, im2col, col2im).  One JSON line.

  python scripts/conv_bwd_layers.py
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402
from tensorium_amd._abi import TNS_OP_GEMM, TNS_OP_IM2COL, TNS_OP_COL2IM  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--dx-fused", type=int, default=1, help="TNS_OPT_DX_FUSED")
    ap.add_argument("--dw-tile", type=int, default=-1, help="TNS_OPT_DW_TILE")
    ap.add_argument("--dx-tile", type=int, default=-1, help="TNS_OPT_DX_TILE")
    ap.add_argument("--layers", default="", help="comma-separated layer indices (default: all)")
    a = ap.parse_args()
    hip = TNNHip(0)
    hip.setDxFused(a.dx_fused)
    hip.setDwTile(a.dw_tile)
    hip.setDxTile(a.dx_tile)
    only = {int(v) for v in a.layers.split(",") if v}
    batch = 8
    out = []
    for s in yolov3_conv_table():
        if only and s.index not in only:
            continue
        x = torch.rand(batch, s.c, s.h, s.h, device="cuda")
        w = torch.rand(s.filters, s.K, device="cuda") * 0.1
        o = torch.rand(batch, s.filters, s.out_h, s.out_h, device="cuda")
        d = torch.rand_like(o)
        bu, wu = torch.zeros(s.filters, device="cuda"), torch.zeros(s.filters, s.K, device="cuda")
        sd = torch.zeros_like(x)
        run = lambda: hip.convBackward(batch, s.c, s.h, s.h, x, w, s.filters, s.size, s.stride,  # noqa
                                       s.pad, 1, s.activation, o, d, bu, wu, None, sd)
        run()
        hip.setTelemetry(True)
        run()
        g, i, c = hip.opMs(TNS_OP_GEMM), hip.opMs(TNS_OP_IM2COL), hip.opMs(TNS_OP_COL2IM)
        hip.setTelemetry(False)
        # dW alone (no state.delta: no dX GEMM, no col2im)
        run_dw = lambda: hip.convBackward(batch, s.c, s.h, s.h, x, w, s.filters, s.size,  # noqa
                                          s.stride, s.pad, 1, s.activation, o, d, bu, wu, None,
                                          None)
        run_dw()
        hip.setTelemetry(True)
        run_dw()
        gw = hip.opMs(TNS_OP_GEMM)
        hip.setTelemetry(False)
        # whole backward call (derive, bias sums, im2col, dW incl. any
        # accumulate pass, dX, col2im) by HIP events
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run()
        e1.record()
        torch.cuda.synchronize()
        call_ms = e0.elapsed_time(e1) / 5
        out.append({"layer": s.index, "shape": f"{s.c}x{s.h} k{s.size}s{s.stride}->{s.filters}",
                    "gemm_ms": round(g, 3), "dw_ms": round(gw, 3), "dx_ms": round(g - gw, 3), "tf": round(2 * s.flops * batch / g / 1e9, 1),
                    "im2col_ms": round(i, 3), "col2im_ms": round(c, 3),
                    "call_ms": round(call_ms, 4)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
