#!/usr/bin/env python3
"""Block timeline of one implicit-conv / GEMM launch from a diagnostic build
(TNS_EXTRA_CFLAGS=-DTNS_GEMM_STAMPS, loaded with TNS_LIB=...): per block
start/end s_memtime and its CU.  Reports the kernel span, block durations by
how many blocks shared the CU, and CU occupancy over time.

  TNS_LIB=ab/gstamps/libtensorium_hip.so python scripts/gemm_timeline.py --layer 11
"""
import argparse
import ctypes
import json
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd._abi import load  # noqa: E402
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layer", type=int, default=11)
ap.add_argument("--variant", type=int, default=-1)
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--gemm", default="", help="M,N,K plain NN GEMM instead of a conv layer")
a = ap.parse_args()
hip = TNNHip(0)
lib = load()
stamps = torch.zeros(8 * 65536, dtype=torch.int32, device="cuda")
fn = lib.tns_debug_gemm_stamps
fn.argtypes = [ctypes.c_void_p]
if a.gemm:
    M, N, K = (int(x) for x in a.gemm.split(","))
    A = torch.rand(M, K, device="cuda")
    B = torch.rand(K, N, device="cuda")
    Cm = torch.empty(M, N, device="cuda")
    run = lambda: hip.gemmVariant(a.variant, False, False, M, N, K, 1.0, A, 0, K, 0, B, 0, N, 0,
                                  0.0, Cm, 0, N, 0, 1)
    flop = 2.0 * M * N * K
else:
    s = yolov3_conv_table()[a.layer]
    x = torch.rand(a.batch, s.c, s.h, s.h, device="cuda")
    w = torch.rand(s.filters, s.K, device="cuda") * 0.2 - 0.1
    b = torch.rand(s.filters, device="cuda") * 0.2 - 0.1
    out = torch.empty(a.batch, s.filters, s.N, device="cuda")
    hip.setConvVariant(a.variant)
    run = lambda: hip.convForward(a.batch, s.c, s.h, s.h, x, w, b, s.filters, s.size, s.stride,
                                  s.pad, 1, s.activation, None, out, fused=3)
    flop = float(s.flops) * a.batch
for _ in range(5):
    run()
torch.cuda.synchronize()
fn(stamps.data_ptr())
run()
torch.cuda.synchronize()
fn(None)
st = stamps.cpu().numpy().view(np.uint32).reshape(-1, 8).astype(np.uint64)
used = st[:, 2] != 0
st = st[used]
t0 = st[:, 0] | (st[:, 1] << 32)
t1 = st[:, 2] | (st[:, 3] << 32)
hw, xcc = st[:, 4].astype(np.int64), st[:, 5].astype(np.int64)
cu = (xcc & 0xf) * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 50 + ((hw >> 8) & 0xf)
# s_memtime counters are per XCD (not synchronised across dies): every XCD's
# timeline starts at its own first block
t0i = np.zeros(len(t0), np.int64)
t1i = np.zeros(len(t0), np.int64)
for x in np.unique(xcc & 0xf):
    sel = (xcc & 0xf) == x
    base = int(t0[sel].min())
    t0i[sel] = (t0[sel] - base).astype(np.int64)
    t1i[sel] = (t1[sel] - base).astype(np.int64)
t0, t1 = t0i, t1i
span = int(t1.max())
dur = t1 - t0
# concurrency of each block: mean number of blocks on its CU during its life
conc = np.zeros(len(t0))
bycu = defaultdict(list)
for i, c in enumerate(cu):
    bycu[int(c)].append(i)
for c, idx in bycu.items():
    for i in idx:
        ov = 0
        for j in idx:
            ov += max(0, min(t1[i], t1[j]) - max(t0[i], t0[j]))
        conc[i] = ov / max(dur[i], 1)
res = {"blocks": int(len(t0)), "cus": len(bycu), "span_ticks": span,
       "tflops_at_span_2.1GHz": round(flop / (span / 2.1e9) / 1e12, 1),
       "dur_mean": int(dur.mean()), "dur_min": int(dur.min()), "dur_max": int(dur.max()),
       "start_max": int(t0.max()), "end_min": int(t1.min())}
for k in sorted(set(np.round(conc).astype(int))):
    sel = np.round(conc).astype(int) == k
    res[f"dur_at_conc{k}"] = [int(sel.sum()), int(dur[sel].mean())]
# busy CUs over time (10 buckets)
edges = np.linspace(0, span, 11)
occ = []
for lo, hi in zip(edges[:-1], edges[1:]):
    mid = (lo + hi) / 2
    alive = (t0 <= mid) & (t1 >= mid)
    occ.append([int(len(set(cu[alive]))), int(alive.sum())])
res["cus_and_blocks_alive_by_decile"] = occ
blocks_per_cu = [len(v) for v in bycu.values()]
res["blocks_per_cu_hist"] = {int(k): int(v) for k, v in zip(*np.unique(blocks_per_cu,
                                                                       return_counts=True))}
print(json.dumps(res))
