#!/usr/bin/env python3
"""Conv dW products of the YOLOv3 batch-8 backward (nConvolutionLayer.pas:
636-640: weight_updates += delta_b . col_b^T per image, sdot order) timed on
every sdot-order NT kernel: the MFMA kernel (form 0) and each VALU chain
variant (form 1 + v), as the strided-batched launch the driver issues.  One
JSON line: per distinct layer shape the ms of each form, the default pick and
its ms.

  python scripts/sdot_forms.py [--all]     (--all: every chain variant)
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    hip = TNNHip(0)
    batch = 8
    nv = hip.sdotChainsVariants()
    forms = list(range(nv + 1)) if "--all" in sys.argv else [0, 1, 2, 3, 4, 5, 6, 9]
    seen, rows = set(), []
    for s in yolov3_conv_table():
        M, N, K = s.filters, s.K, s.out_h * s.out_h
        if (M, N, K) in seen:
            continue
        seen.add((M, N, K))
        A = torch.rand(batch, M, K, device="cuda") * 2 - 1
        B = torch.rand(batch, N, K, device="cuda") * 2 - 1
        C = torch.zeros(batch, M, N, device="cuda")
        run = lambda: hip.gemmStridedBatched(False, True, M, N, K, 1.0, A, 0, K, M * K, B, 0,  # noqa
                                             K, N * K, 0.0, C, 0, N, M * N, batch)
        reps = 5 if batch * M * N * K > 3e9 else 20
        row = {"layer": s.index, "M": M, "N": N, "K": K, "ms": {}}
        ref = None
        for f in forms + [-1]:
            hip.setSdotForm(f)
            ms = timed(run, reps)
            if f >= 0:
                row["ms"][f] = round(ms, 4)
            else:
                row["default_ms"] = round(ms, 4)
            if ref is None:
                ref = C.clone()
            elif not torch.equal(ref, C):
                row.setdefault("mismatch", []).append(f)
        hip.setSdotForm(-1)
        best = min(row["ms"], key=row["ms"].get)
        row["best"] = best
        row["gflop"] = round(2 * batch * M * N * K / 1e9, 3)
        rows.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    names = {f + 1: hip.lib.tns_sdot_chains_variant_name(f).decode() for f in range(nv)}
    print(json.dumps({"forms": names, "rows": rows}))


if __name__ == "__main__":
    main()
