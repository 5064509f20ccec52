#!/usr/bin/env python3
"""Measured HBM ceilings on this GPU for the traffic mixes of the elementwise
kernels: write-only (tns_hip_fill), read+write 1:1 (tns_hip_copy; torch
copy_), read-only (torch sum).  GB/s of algorithmic bytes, HIP events.

  python scripts/hbm_ceiling.py
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
    for mb in (64, 400, 1600):
        n = mb * 1024 * 1024 // 4
        x = torch.rand(n, device="cuda")
        y = torch.empty_like(x)
        r = {}
        ms = timed(lambda: hip.fill(n, y, 0, 1.5, 1), 10)
        r["fill_write_only"] = round(n * 4 / ms / 1e6, 1)
        ms = timed(lambda: torch.fill_(y, 2.0), 10)
        r["torch_fill"] = round(n * 4 / ms / 1e6, 1)
        ms = timed(lambda: hip.copy(n, x, 0, 1, y, 0, 1), 10)
        r["copy_r1w1"] = round(2 * n * 4 / ms / 1e6, 1)
        ms = timed(lambda: y.copy_(x), 10)
        r["torch_copy"] = round(2 * n * 4 / ms / 1e6, 1)
        ms = timed(lambda: x.sum(), 10)
        r["torch_sum_read_only"] = round(n * 4 / ms / 1e6, 1)
        out[f"{mb}MiB"] = r
        del x, y
    print(json.dumps(out))


if __name__ == "__main__":
    main()
