#!/usr/bin/env python3
"""YOLOv3 batch-8 conv forward per distinct layer shape: the default choice,
the previous shape heuristic (TNS_OPT_CONV_VARIANT = 99: sgemm_kernel.hpp
tiles on zero-padded copies) and every plane-sized conv tile (100 + v) and ping-pong tile (200 + v),
interleaved rounds in one process.  One JSON line; per-shape lines on stderr.

  python scripts/conv_tile_sweep.py [--rounds 3]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd._abi import TnsError  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--only", default="", help="comma list of forced variants to time")
    a = ap.parse_args()
    hip = TNNHip(0)
    nt = hip.convTileVariants()
    names = {100 + v: hip.lib.tns_conv_tile_variant_name(v).decode() for v in range(nt)}
    names.update({200 + v: hip.lib.tns_conv_pp_variant_name(v).decode()
                  for v in range(hip.convPPVariants())})
    names.update({300 + v: hip.lib.tns_conv_dma_variant_name(v).decode()
                  for v in range(hip.convDMAVariants())})
    names.update({400 + v: hip.lib.tns_conv_patch_variant_name(v).decode()
                  for v in range(hip.convPatchVariants())})
    if a.only:
        names = {k: v for k, v in names.items() if str(k) in a.only.split(",")}
    forms = [-1, 99] + list(names)
    layers, seen = [], {}
    for s in yolov3_conv_table():
        key = (s.c, s.h, s.filters, s.size, s.stride)
        seen[key] = seen.get(key, 0) + 1
        if seen[key] > 1:
            continue
        x = torch.rand(a.batch, s.c, s.h, s.h, device="cuda")
        w = torch.rand(s.filters, s.K, device="cuda") * 0.2 - 0.1
        b = torch.rand(s.filters, device="cuda") * 0.2 - 0.1
        out = torch.empty(a.batch, s.filters, s.N, device="cuda")
        layers.append((s, key, x, w, b, out))
    res = {key: {f: [] for f in forms} for _, key, *_ in layers}
    for _ in range(a.rounds):
        for s, key, x, w, b, out in layers:
            run = lambda: hip.convForward(a.batch, s.c, s.h, s.h, x, w, b, s.filters, s.size,  # noqa
                                          s.stride, s.pad, 1, s.activation, None, out)
            for f in forms:
                hip.setConvVariant(f)
                try:
                    run()
                except TnsError:
                    continue
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    run()
                e1.record()
                torch.cuda.synchronize()
                res[key][f].append(e0.elapsed_time(e1) / 5)
            hip.setConvVariant(-1)
    rows = []
    for s, key, *_ in layers:
        gf = s.flops * a.batch / 1e9
        ms = {str(f): round(float(np.median(v)), 4) for f, v in res[key].items() if v}
        best = min(ms, key=ms.get)
        row = {"layer": s.index, "count": seen[key],
               "shape": f"{s.c}x{s.h} k{s.size}s{s.stride}->{s.filters}", "gflop": round(gf, 3),
               "ms": ms, "best": best, "default_tf": round(gf / ms["-1"], 1),
               "legacy_tf": round(gf / ms["99"], 1), "best_tf": round(gf / ms[best], 1)}
        rows.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    tot = {k: round(sum(r["count"] * r["ms"].get(k, 0) for r in rows), 3) for k in ("-1", "99")}
    tot["best"] = round(sum(r["count"] * r["ms"][r["best"]] for r in rows), 3)
    print(json.dumps({"names": names, "sum_ms": tot, "rows": rows}))


if __name__ == "__main__":
    main()
