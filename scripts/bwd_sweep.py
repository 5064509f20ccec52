#!/usr/bin/env python3
"""Sweep the conv backward's kernel forms per YOLOv3 layer (batch 8, with
state.delta): every dW form (im2col + the sdot kernels: MFMA, VALU chain
variants, residue-register variants; the implicit-im2col dw_tile forms) and
every dX form (TN GEMM, k-major conv tiles, fused dX + col2im).  Each call
timed by HIP events after a warm-up; all forms give the same bits (the GPU
tests check that), so the fastest is a free choice.  One JSON line.

  python scripts/bwd_sweep.py --layers 0,1,2,3 [--what dw,dx]
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
    ap.add_argument("--layers", default="0,1,2,3,4,5,6,9,10,11")
    ap.add_argument("--what", default="dw,dx")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    hip = TNNHip(0)
    n_chain, n_rc, n_dw, n_dx = (hip.sdotChainsVariants(), hip.sdotRcVariants(), hip.convDwTiles(),
                                 hip.convDxTiles())
    B = 8
    res = {}
    for s in yolov3_conv_table():
        if s.index not in {int(v) for v in a.layers.split(",")}:
            continue
        x = torch.rand(B, s.c, s.h, s.h, device="cuda")
        w = torch.rand(s.filters, s.K, device="cuda") * 0.1
        o = torch.rand(B, s.filters, s.out_h, s.out_h, device="cuda")
        d = torch.rand_like(o)
        bu, wu = torch.zeros(s.filters, device="cuda"), torch.zeros(s.filters, s.K, device="cuda")
        sd = torch.zeros_like(x)

        def run():
            hip.convBackward(B, s.c, s.h, s.h, x, w, s.filters, s.size, s.stride, s.pad, 1,
                             s.activation, o, d, bu, wu, None, sd)

        def timed():
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

        for _ in range(50):  # a warm clock before the first timed form (~50 calls)
            run()
        torch.cuda.synchronize()
        row = {"shape": f"{s.c}x{s.h} k{s.size}s{s.stride}->{s.filters}", "default": timed()}
        if "dw" in a.what:
            forms = ([("sdot", f) for f in [0] + [1 + v for v in range(n_chain)] +
                      [64 + v for v in range(n_rc)]] + [("dwtile", v) for v in range(n_dw)] +
                     [("dwres", v) for v in range(hip.convDwRes())])
            for kind, f in forms:
                try:
                    if kind == "sdot":
                        hip.setDwTile(-2)
                        hip.setDwRes(-2)
                        hip.setSdotForm(f)
                    elif kind == "dwtile":
                        hip.setDwTile(f)
                    else:
                        hip.setDwRes(f)
                    row[f"{kind}{f}"] = timed()
                except TnsError:
                    pass
                finally:
                    hip.setDwTile(-1)
                    hip.setDwRes(-1)
                    hip.setSdotForm(-1)
        if "dx" in a.what:
            for f in [-2] + list(range(n_dx)):
                try:
                    hip.setDxTile(f)
                    row[f"dxtile{f}"] = timed()
                except TnsError:
                    pass
                finally:
                    hip.setDxTile(-1)
            for f in [-2] + list(range(hip.convDxConvs())):
                try:
                    hip.setDxConv(f)
                    row[f"dxconv{f}"] = timed()
                except TnsError:
                    pass
                finally:
                    hip.setDxConv(-1)
            for f in (0, 2):
                try:
                    hip.setDxFused(f)
                    row[f"dxfused{f}"] = timed()
                except TnsError:
                    pass
                finally:
                    hip.setDxFused(1)
        best = min((v, k) for k, v in row.items() if isinstance(v, float))
        row["best"] = best[1]
        res[s.index] = row
        print(json.dumps({s.index: row}), file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
