#!/usr/bin/env python3
"""Rates of the batch-norm forward kernels (meansAndVars in the reference's
lane orders, normalize, forwardScaleAdd) on conv-layer BN shapes of YOLOv3
at batch 8 ([groups=8][channels][H*W]) and the MNIST FC shape.  Algorithmic
bytes: meansAndVars reads x (twice: mean then variance pass), normalize and
scale+bias read and write x; meansAndVarsDelta reads delta and x once
(both lane chains run off one staged tile); addDots reads both operands, addSums
one.  One JSON line.

  python scripts/bn_perf.py
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from nt_perf import timed  # noqa: E402


def main():
    hip = TNNHip(0)
    out = {}
    for groups, N, bs in [(8, 32, 173056), (8, 64, 43264), (8, 256, 2704), (8, 1024, 169),
                          (32, 64, 1)]:
        n = groups * N * bs
        x = torch.rand(n, device="cuda")
        m, v = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
        s, b = torch.ones(N, device="cuda"), torch.zeros(N, device="cuda")
        row = {}
        ms = timed(lambda: hip.meansAndVars(n, N, groups, x, 0, m, v), 10)
        row["means_vars_ms"] = round(ms, 4)
        row["means_vars_gbs"] = round(2 * n * 4 / ms / 1e6, 1)
        ms = timed(lambda: hip.normalize(N, n, groups, m, 1, v, 1, x, 0), 10)
        row["normalize_gbs"] = round(2 * n * 4 / ms / 1e6, 1)
        ms = timed(lambda: hip.forwardScaleAdd(n, x, 0, N, s, b, 1, groups), 10)
        row["scale_add_gbs"] = round(2 * n * 4 / ms / 1e6, 1)
        d = torch.rand(n, device="cuda")
        md, vd = torch.zeros(N, device="cuda"), torch.zeros(N, device="cuda")
        ms = timed(lambda: hip.meansAndVarsDelta(n, N, groups, d, x, 0, m, v, md, vd), 5)
        row["means_vars_delta_ms"] = round(ms, 4)
        row["means_vars_delta_gbs"] = round(2 * n * 4 / ms / 1e6, 1)
        dsc = torch.zeros(N, device="cuda")
        ms = timed(lambda: hip.addDots(n, N, groups, d, x, 0, dsc), 5)
        row["add_dots_ms"] = round(ms, 4)
        row["add_dots_gbs"] = round(2 * n * 4 / ms / 1e6, 1)
        ms = timed(lambda: hip.backwardBias(N, dsc, n, d, 0, 1, groups), 5)
        row["add_sums_ms"] = round(ms, 4)
        row["add_sums_gbs"] = round(n * 4 / ms / 1e6, 1)
        out[f"{groups}x{N}x{bs}"] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main()
