#!/usr/bin/env python3
"""Driver for the counter-based HBM traffic of the elementwise path
(VERDICT r01 item 6).  Runs each elementwise kernel of the conv / batch-norm
path REPS times at a YOLOv3-416 batch-8 shape, plus two calibration kernels
whose byte counts are known (a 4-byte-per-lane strided copy and the float4
SGD update), so that FETCH_SIZE can be corrected per access width as
MI355X_MICROARCH.md §HBM asks ("calibrate on a known byte count in your own
access pattern").  Meant to run under rocprofv3 (scripts/profile_elementwise.sh):

  pass 1  --kernel-trace --stats     durations
  pass 2  --pmc FETCH_SIZE           memory-side read requests
  pass 3  --pmc WRITE_SIZE           memory-side write requests

and summarised by scripts/summarize_elementwise.py.  Prints the algorithmic
byte count of every kernel (one JSON line) so the summary can divide.
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tensorium_amd.nnhip import TNNHip  # noqa: E402
from tensorium_amd.yolo import yolov3_conv_table  # noqa: E402

REPS = 5


def main():
    hip = TNNHip(0)
    T = torch
    cuda = "cuda"
    alg = {}
    sep = T.zeros(1, device=cuda)

    def run(name, fn, nbytes):
        # one fill_kernel launch opens each op's segment of the dispatch list
        hip.fill(1, sep, 0, float(len(alg)), 1)
        for _ in range(REPS):
            fn()
        hip.finish()
        alg[name] = nbytes

    # calibration: 1 GiB read + 1 GiB written with 4-byte lanes (copy), and
    # 16-byte lanes (sgd_update<4>: w, dw read and written)
    n = 1 << 28
    a, b = T.rand(n, device=cuda), T.empty(n, device=cuda)
    run("calib_copy_b32", lambda: hip.copy(n, a, 0, 1, b, 0, 1), {"read": 4 * n, "write": 4 * n})
    w, dw = T.rand(n, device=cuda), T.rand(n, device=cuda)
    bb, db = T.zeros(1, device=cuda), T.zeros(1, device=cuda)
    run("calib_sgd_b128", lambda: hip.sgdUpdate(w, dw, bb, db, 1e-3, 8, 1e-4, 0.9),
        {"read": 8 * n, "write": 8 * n})
    del a, b, w, dw
    T.cuda.empty_cache()

    specs = yolov3_conv_table()
    batch = 8
    s = specs[3]  # 32 x 208 x 208, 3x3 s1 -> 64 filters: the largest col matrix of a 3x3 layer
    x = T.rand(batch * s.c * s.h * s.h, device=cuda)
    col = T.empty(batch * s.col_elems, device=cuda)
    img = batch * s.c * s.h * s.h
    run("im2col", lambda: hip.im2colStridedBatched(
        s.c, s.h, s.h, s.size, s.size, s.pad, s.pad, s.stride, s.stride, 1, 1, x,
        s.c * s.h * s.h, 0, col, s.col_elems, 0, batch),
        {"read": 4 * img, "write": 4 * batch * s.col_elems, "layer": s.index})
    run("col2im", lambda: hip.col2imStridedBatched(
        s.c, s.h, s.h, s.size, s.size, s.pad, s.pad, s.stride, s.stride, 1, 1, col,
        s.col_elems, 0, x, s.c * s.h * s.h, 0, batch),
        {"read": 4 * (batch * s.col_elems + img), "write": 4 * img, "layer": s.index})
    del col
    out = T.rand(batch * s.filters * s.out_h * s.out_h, device=cuda)
    bias = T.rand(s.filters, device=cuda)
    no = out.numel()
    run("forward_bias", lambda: hip.forwardBias(no, out, 0, s.filters, bias, 1, batch),
        {"read": 4 * no, "write": 4 * no, "layer": s.index})
    run("activate_leaky", lambda: hip.ActivateArray(no, out, 0, 9),
        {"read": 4 * no, "write": 4 * no, "layer": s.index})
    del out, x
    # batch norm over the first layer's output: 8 x 32 x 173056 (the widest
    # blocks) — the lane-chain reductions and the fused train-time apply
    G, N, bs = batch, 32, 416 * 416
    ne = G * N * bs
    y = T.rand(ne, device=cuda)
    d = T.rand(ne, device=cuda)
    m, v = T.zeros(N, device=cuda), T.ones(N, device=cuda)
    md, vd, dsc = T.zeros(N, device=cuda), T.zeros(N, device=cuda), T.zeros(N, device=cuda)
    run("means_and_vars", lambda: hip.meansAndVars(ne, N, G, y, 0, m, v),
        {"read": 2 * 4 * ne, "write": 0, "shape": [G, N, bs]})
    run("means_and_vars_delta",
        lambda: hip.meansAndVarsDelta(ne, N, G, d, y, 0, m, v, md, vd),
        {"read": 2 * 4 * ne, "write": 0, "shape": [G, N, bs]})
    run("add_dots", lambda: hip.addDots(ne, N, G, y, d, 0, dsc),
        {"read": 2 * 4 * ne, "write": 0, "shape": [G, N, bs]})
    run("add_sums", lambda: hip.backwardBias(N, dsc, ne, d, 0, 1, G),
        {"read": 4 * ne, "write": 0, "shape": [G, N, bs]})
    run("normalize", lambda: hip.normalize(N, ne, G, m, 1, v, 1, y, 0),
        {"read": 4 * ne, "write": 4 * ne, "shape": [G, N, bs]})
    run("normalize_delta", lambda: hip.normalizeDelta(ne, N, G, d, y, 0, m, v, md, vd),
        {"read": 2 * 4 * ne, "write": 4 * ne, "shape": [G, N, bs]})
    print(json.dumps({"reps": REPS, "algorithmic_bytes": alg}), flush=True)


if __name__ == "__main__":
    main()
