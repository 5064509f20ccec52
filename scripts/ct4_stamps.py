#!/usr/bin/env python3
"""Per-phase cycle sums of conv_tile4's wave 0 (diagnostic build with
-DTNS_CT4_STAMPS, loaded with TNS_LIB=...): tile top (loads issued), groups
before the stores, the stores, up to the barrier, the barrier wait, and the
rest (last group + loop).  Mean cycles per k-tile over the blocks.

  TNS_LIB=ab/ct4s/libtensorium_hip.so python scripts/ct4_stamps.py --layer 11 --variant 106
"""
import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd._abi import load  # noqa: E402
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layer", default="11", help="layer index or comma list")
ap.add_argument("--variant", type=int, default=-1, help="-1: the heuristic")
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--warm-ms", type=float, default=0.0, help="load before the stamped run")
a = ap.parse_args()
hip = TNNHip(0)
lib = load()
stamps = torch.zeros(32 * 65536, dtype=torch.int32, device="cuda")
fn = lib.tns_debug_ct4_stamps
fn.argtypes = [ctypes.c_void_p]
for layer in map(int, a.layer.split(",")):
    s = yolov3_conv_table()[layer]
    x = torch.rand(a.batch, s.c, s.h, s.h, device="cuda")
    w = torch.rand(s.filters, s.K, device="cuda") * 0.2 - 0.1
    b = torch.rand(s.filters, device="cuda") * 0.2 - 0.1
    out = torch.empty(a.batch, s.filters, s.N, device="cuda")
    hip.setConvVariant(a.variant)
    run = lambda: hip.convForward(a.batch, s.c, s.h, s.h, x, w, b, s.filters, s.size, s.stride,  # noqa
                                  s.pad, 1, s.activation, None, out)
    for _ in range(20):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < a.warm_ms:
        for _ in range(10):
            run()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    layer_ms = e0.elapsed_time(e1) / 20
    stamps.zero_()
    fn(stamps.data_ptr())
    run()
    torch.cuda.synchronize()
    fn(None)
    st = stamps.cpu().numpy().view(np.uint32).reshape(-1, 32).astype(np.float64)
    st = st[st[:, 7] > 0]
    # block timeline (100 MHz realtime): entry relative to the first block's,
    # prologue (entry -> loop start), loop, epilogue (loop end -> wave 0's
    # stores done), end relative to the first entry
    ent = st[:, 8] + st[:, 9] * 2.0 ** 32
    ent = (ent - ent.min()) / 100.0  # us
    pro = st[:, 10] / 100.0
    loop_us = (st[:, 12] - st[:, 10]) / 100.0
    epi = (st[:, 11] - st[:, 12]) / 100.0
    end = ent + st[:, 11] / 100.0
    q = lambda v: [round(float(np.percentile(v, x)), 2) for x in (0, 50, 100)]  # noqa: E731
    timeline = {"entry_us_min_med_max": q(ent), "prologue_us": q(pro), "loop_us": q(loop_us),
                "epilogue_us": q(epi), "end_us": q(end)}
    # tile 8's barrier: each wave's arrival (s_memtime cycles) after the
    # block's first arrival; mean lateness per wave index, and how often each
    # wave is the last to arrive
    arr = st[:, 16:32]
    nw = int((arr[0] > 0).sum()) if len(arr) else 0
    if nw > 1 and int(st[0, 7]) & 0xff > 8:
        a_ = arr[:, :nw]
        late = a_ - a_.min(axis=1, keepdims=True)
        timeline["barrier8_late_cycles_by_wave"] = [round(float(v), 1) for v in late.mean(axis=0)]
        last = np.bincount(a_.argmax(axis=1), minlength=nw)
        timeline["barrier8_last_counts_by_wave"] = [int(v) for v in last]
    nt = st[:, 7].astype(np.uint64) & 0xff
    rt = (st[:, 7].astype(np.uint64) >> 8).astype(np.float64)  # 100 MHz ticks
    nt = nt.astype(np.float64)
    names = ["top_loads", "groups_before_store", "stores", "to_barrier", "barrier_wait", "last_group_loop"]
    per_tile = {n: round(float(np.mean(st[:, i] / nt)), 1) for i, n in enumerate(names)}
    per_tile["total"] = round(float(np.mean(st[:, 6] / nt)), 1)
    clock_ghz = round(float(np.median(st[:, 6] / np.maximum(rt, 1) * 0.1)), 3)
    print(json.dumps({"layer": layer, "variant": a.variant, "blocks": int(len(st)),
                      "k_tiles": int(nt[0]), "layer_ms": round(layer_ms, 4), "cycles_per_tile_wave0": per_tile,
                      "clock_ghz_median": clock_ghz, "timeline": timeline}))
