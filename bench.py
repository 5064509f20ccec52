#!/usr/bin/env python3
"""bench.py — fp32 SGEMM (M=N=K=4096) on MI355X via libtensorium_hip.so, plus
YOLOv3-416 conv-forward images/s, per BASELINE.json's metric.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N ... bench.py --gpus N      (one process per GPU)

A "step" is one pass of the hot path over one batch of synthetic input: one
NN SGEMM 4096^3 (alpha=1, beta=0; BASELINE configs[1]) on operands already
resident in HBM.  With N GPUs every rank runs its own independent GEMM per
step (independent units, no data-path collective — SURVEY §8e), so scaling is
weak and `value` = total FLOP of all ranks / max-over-ranks time.  The
headline is timed after the secondary workloads below, at the clock the chip
holds under sustained load (a cold GPU ramps over its first ~20 launches).

Extra fields on the single JSON line:
  roofline     — dominant kernel (sgemm_mfma) vs the fp32 MFMA peak, its
                 duration taken live with HIP events on the stream the kernel
                 is launched on; `traffic` from the committed PMC pass
                 (profiles/, FETCH_SIZE doubled per the gfx950 guide) or null.
  cpu_baseline — the oracle's restated sgemm_nn (reference: ntensors.pas
                 cblas_sgemm -> sgemm_nn -> saxpy_avx2) on the host cores, rank
                 0 at N=1 only, on a bounded sample of rows of the same product.
  yolo         — YOLOv3-416 conv forward, batch 8 per GPU, 75 conv layers
                 (BASELINE configs[2]); images/s over all ranks.
  yolo_network — the whole YOLOv3-416 network (convolutions chained through
                 shortcut / route / upsample / yolo layers), batch 8 per GPU.
  yolo_conv_backward  — the 75 conv layers' backward (no BN) back to back.
  yolo_train_backward — TNet.backward over the whole network as the drop-in
                 runs it in training (BN conv layers, shortcut / route /
                 upsample / yolo backward calls between them).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_F32_TFLOPS = 157.3   # MI355X fp32 MFMA (= vector) peak, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=30,
                    help="untimed steps; the GPU clock ramps over the first ~20 launches "
                         "(profiles/r01_clock_ramp.json)")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--yolo-steps", type=int, default=5)
    ap.add_argument("--no-yolo", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-batched", action="store_true")
    ap.add_argument("--no-mnist", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target CPU-baseline sample duration")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check: start the ranks, rendezvous over gloo, print the "
                         "JSON line with n_gpus and the ranks seen; no GPU work")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def profiler_preloaded(env) -> bool:
    """rocprofv3 / roctracer injected into this process (LD_PRELOAD)."""
    preload = env.get("LD_PRELOAD", "")
    return any(tag in preload for tag in ("rocprof", "roctracer", "rocprofiler"))


def launch_ranks(args) -> int | None:
    """One process per GPU.  Returns None when this process is a rank (the
    caller goes on to benchmark), else the launcher's exit code.

    * WORLD_SIZE set (torchrun / the driver): it must equal --gpus, else exit
      non-zero — a mismatch would report a world the run did not have.
    * WORLD_SIZE unset and --gpus N > 1: start N copies of this script as
      child processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, before
      this process touches torch or the GPU; wait for them, stop the rest if
      one fails, and exit with the first non-zero status (rank 0 prints the
      JSON line).
    """
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}; refusing to report a "
                  f"world the run does not have", file=sys.stderr, flush=True)
            return 2
        return None
    if args.gpus <= 1:
        return None
    # A profiler's preloaded library has already initialised the GPU in this
    # process: starting ranks from here would be a spawn after GPU init.
    # Profile a multi-GPU run through torchrun (WORLD_SIZE set) instead.
    if profiler_preloaded(os.environ):
        print("bench.py: a profiler library is preloaded; refusing to start rank processes "
              "from a profiled launcher (run the ranks under torchrun)", file=sys.stderr,
              flush=True)
        return 2
    import signal
    import subprocess
    port = str(_free_port())
    procs = []
    rc = 0

    def stop(signum, _frame):   # a timeout or Ctrl-C of the launcher stops the ranks
        raise KeyboardInterrupt(signum)

    old = {sig: signal.signal(sig, stop) for sig in (signal.SIGTERM, signal.SIGHUP)}
    try:
        for r in range(args.gpus):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                       LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=port)
            procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] +
                                          sys.argv[1:], env=env))
        alive = list(procs)
        while alive:
            for p in list(alive):
                code = p.poll()
                if code is None:
                    continue
                alive.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the "
                          f"other ranks", file=sys.stderr, flush=True)
                    for q in alive:
                        q.terminate()
            time.sleep(0.05)
    except KeyboardInterrupt:
        rc = rc or 130
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        for sig, h in old.items():
            signal.signal(sig, h)
    return rc


def dry_run(args):
    """Launcher rehearsal (no GPU): every rank joins a gloo group, the ranks
    are gathered, rank 0 prints one JSON line."""
    from tensorium_amd import dist as tdist
    if os.environ.get("TNS_DRYRUN_FAIL_RANK") == os.environ.get("RANK", "0"):
        sys.exit(3)   # test hook: a rank that dies before the rendezvous
    if os.environ.get("TNS_DRYRUN_HANG_DIR"):   # test hook: ranks that never finish
        Path(os.environ["TNS_DRYRUN_HANG_DIR"], f"rank{os.environ.get('RANK', '0')}").write_text(
            str(os.getpid()))
        time.sleep(3600)
    ctx = tdist.init("gloo", use_gpu=False)
    ranks = ctx.gather_floats([float(ctx.rank), float(os.getpid())])
    t = ctx.max(float(ctx.rank))
    ctx.barrier()
    if ctx.rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": ctx.world, "gpus_arg": args.gpus,
                          "ranks": [int(r[0]) for r in ranks],
                          "pids": [int(r[1]) for r in ranks], "max_rank": t}), flush=True)
    ctx.close()


def synthetic(torch, shape, seed, lo=-1.0, hi=1.0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.rand(shape, generator=g, device="cuda", dtype=torch.float32) * (hi - lo) + lo


def bench_sgemm(torch, hip, ctx, rank, n, steps, warmup):
    A = synthetic(torch, (n, n), 2 * 1000 + rank)
    B = synthetic(torch, (n, n), 2 * 1000 + 500 + rank)
    Cm = torch.zeros((n, n), device="cuda", dtype=torch.float32)

    def step():
        hip.gemm(False, False, n, n, n, 1.0, A, 0, n, B, 0, n, 0.0, Cm, 0, n)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    # per-launch kernel duration with HIP events on the kernel's own stream
    # (TNNHip attaches torch's current stream, so torch.cuda.Event records there)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        ev[i][0].record()
        step()
        ev[i][1].record()
    torch.cuda.synchronize()
    ctx.barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    return wall, float(np.mean(kern_ms)), float(np.min(kern_ms))


def bench_yolo(torch, hip, ctx, rank, steps, warmup=4):
    from tensorium_amd.yolo import yolov3_conv_table
    specs = yolov3_conv_table()
    batch = 8
    layers = []
    max_ws = 0
    for s in specs:
        x = synthetic(torch, (batch, s.c, s.h, s.h), 3 * 100000 + rank * 1000 + s.index, 0.0, 1.0)
        sc = float(np.sqrt(2.0 / (s.size * s.size * s.c)))
        w = synthetic(torch, (s.filters, s.K), 3 * 200000 + s.index, -sc, sc)
        b = synthetic(torch, (s.filters,), 3 * 300000 + s.index, -0.1, 0.1)
        out = torch.empty((batch, s.filters, s.out_h, s.out_h), device="cuda")
        layers.append((s, x, w, b, out))
        max_ws = max(max_ws, batch * s.col_elems)
    ws = torch.empty(max(max_ws, 1), device="cuda")

    def step():
        for s, x, w, b, out in layers:
            hip.convForward(batch, s.c, s.h, s.h, x, w, b, s.filters, s.size, s.stride, s.pad, 1,
                            s.activation, ws, out, fused=True)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ctx.barrier()
    wall = (time.perf_counter() - t0) / steps
    # per-op split with telemetry (synchronous per op, separate passes):
    # the fused schedule (implicit GEMM; its only other op is the zero-border
    # copy of padded images), then the reference's three stages (im2col,
    # GEMM, bias+activation) for the elementwise kernels' HBM rates
    from tensorium_amd._abi import TNS_OP_GEMM, TNS_OP_IM2COL, TNS_OP_BIAS
    hip.setTelemetry(True)
    step()
    gemm_ms, pad_ms = hip.opMs(TNS_OP_GEMM), hip.opMs(TNS_OP_IM2COL)
    hip.setTelemetry(False)
    hip.setTelemetry(True)
    for s, x, w, b, out in layers:
        hip.convForward(batch, s.c, s.h, s.h, x, w, b, s.filters, s.size, s.stride, s.pad, 1,
                        s.activation, ws, out, fused=False)
    i2c_ms, bias_ms = hip.opMs(TNS_OP_IM2COL), hip.opMs(TNS_OP_BIAS)
    hip.setTelemetry(False)
    gflop = sum(s.flops for s in specs) * batch / 1e9
    # im2col: writes the col matrix, reads the image (layers that need one)
    col_bytes = sum(s.col_elems for s in specs) * batch * 4
    in_bytes = sum(s.c * s.h * s.h for s in specs if s.needs_im2col) * batch * 4
    # bias+activation: reads and writes every output element
    out_bytes = sum(2 * s.filters * s.out_h * s.out_h for s in specs) * batch * 4
    return {
        "batch_per_gpu": batch, "ms_per_batch": wall * 1e3, "gflop_per_batch": gflop,
        "gemm_ms": gemm_ms, "pad_copy_ms": pad_ms,
        "gemm_tflops": gflop / gemm_ms if gemm_ms > 0 else None,
        "unfused_im2col_ms": i2c_ms,
        "im2col_gbs": (col_bytes + in_bytes) / (i2c_ms * 1e6) if i2c_ms > 0 else None,
        "unfused_bias_act_ms": bias_ms,
        "bias_act_gbs": out_bytes / (bias_ms * 1e6) if bias_ms > 0 else None,
        "hbm_peak_gbs": 8000.0,
        "rates_note": "unfused rates from per-op synchronous telemetry over all 75 layers "
                      "(launch/sync gaps included; the 13x13 layers are ~20 us launches); "
                      "per-kernel rates: scripts/elementwise_perf.py",
    }


def bench_yolo_dp(torch, hip, ctx, steps):
    """Config 3 data-parallel over the ranks: the batch of 8
    images is split by image (tensorium_amd.shard.shard_range), every rank
    runs the 75 conv layers on its images.  The weights and biases of all 75
    layers (247.6 MB) exist on rank 0 only and reach the others through ONE
    RCCL broadcast of a packed buffer, outside the timed region (timed on
    its own).  images/s = 8 / max-over-ranks time per batch."""
    from tensorium_amd.dist import pack_flat, unpack_flat
    from tensorium_amd.shard import shard_range
    from tensorium_amd.yolo import yolov3_conv_table
    specs = yolov3_conv_table()
    batch = 8
    lo, hi = shard_range(batch, ctx.rank, ctx.world)
    mine = hi - lo
    params = []
    for s in specs:
        sc = float(np.sqrt(2.0 / (s.size * s.size * s.c)))
        if ctx.rank == 0:
            params.append(synthetic(torch, (s.filters, s.K), 3 * 200000 + s.index, -sc, sc))
            params.append(synthetic(torch, (s.filters,), 3 * 300000 + s.index, -0.1, 0.1))
        else:
            params.append(torch.empty((s.filters, s.K), device="cuda"))
            params.append(torch.empty((s.filters,), device="cuda"))
    flat, meta = pack_flat(torch, params, "cuda")
    del params
    torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    ctx.broadcast(flat, src=0)
    torch.cuda.synchronize()
    bcast_ms = ctx.max((time.perf_counter() - t0) * 1e3)
    views = unpack_flat(flat, meta)
    # this rank's images: global image index -> its own synthetic plane stack
    layers = []
    max_ws = 0
    for i, s in enumerate(specs):
        x = torch.empty((max(mine, 1), s.c, s.h, s.h), device="cuda")
        for j, g in enumerate(range(lo, hi)):
            x[j] = synthetic(torch, (s.c, s.h, s.h), 3 * 400000 + g * 1000 + s.index, 0.0, 1.0)
        out = torch.empty((max(mine, 1), s.filters, s.out_h, s.out_h), device="cuda")
        layers.append((s, x, views[2 * i], views[2 * i + 1], out))
        max_ws = max(max_ws, max(mine, 1) * s.col_elems)
    ws = torch.empty(max(max_ws, 1), device="cuda")

    def step():
        if mine == 0:
            return
        for s, x, w, b, out in layers:
            hip.convForward(mine, s.c, s.h, s.h, x, w, b, s.filters, s.size, s.stride, s.pad, 1,
                            s.activation, ws, out, fused=True)

    step()
    torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ctx.barrier()
    ms = ctx.max((time.perf_counter() - t0) / steps * 1e3)
    # every image of the batch computed exactly once across the ranks
    covered = ctx.sum(float(mine))
    wbytes = int(flat.numel()) * 4
    del layers, ws, flat, views
    torch.cuda.empty_cache()
    return {"batch_total": batch, "images_per_rank_max": -(-batch // ctx.world),
            "images_covered": int(covered), "ms_per_batch": round(ms, 4),
            "images_per_s_total": round(batch / (ms / 1e3), 2),
            "weights_bytes": wbytes, "weights_broadcast_ms": round(bcast_ms, 3),
            "collective": "one RCCL broadcast of the packed weights (untimed in ms_per_batch)"
                          if ctx.world > 1 else "none (one rank)",
            "scaling": "strong (fixed batch of 8 split by image)"}


def bench_elementwise_roofline(torch, hip, reps=10):
    """Per-kernel HBM roofline of the elementwise path at YOLOv3 batch-8
    shapes (the ops of scripts/elementwise_traffic.py): durations live with
    HIP events on the kernel's stream; achieved = algorithmic bytes /
    duration against 8 TB/s; `traffic` = the counter-measured bytes per
    launch (FETCH_SIZE / WRITE_SIZE, calibrated per access width) from the
    committed PMC pass, profiles/*_elementwise_traffic.json."""
    from tensorium_amd.yolo import yolov3_conv_table
    cands = sorted(ROOT.glob("profiles/*_elementwise_traffic.json"))
    pmc = json.loads(cands[-1].read_text())["ops"] if cands else {}
    s = yolov3_conv_table()[3]
    batch = 8
    x = torch.rand(batch * s.c * s.h * s.h, device="cuda")
    col = torch.empty(batch * s.col_elems, device="cuda")
    img = batch * s.c * s.h * s.h
    out = torch.rand(batch * s.filters * s.out_h * s.out_h, device="cuda")
    bias = torch.rand(s.filters, device="cuda")
    no = out.numel()
    G, N, bs = batch, 32, 416 * 416
    ne = G * N * bs
    y, d = torch.rand(ne, device="cuda"), torch.rand(ne, device="cuda")
    m, v = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
    md, vd, dsc = (torch.zeros(N, device="cuda") for _ in range(3))
    ops = {
        "im2col": (lambda: hip.im2colStridedBatched(
            s.c, s.h, s.h, s.size, s.size, s.pad, s.pad, s.stride, s.stride, 1, 1, x,
            s.c * s.h * s.h, 0, col, s.col_elems, 0, batch), 4 * (img + batch * s.col_elems)),
        "col2im": (lambda: hip.col2imStridedBatched(
            s.c, s.h, s.h, s.size, s.size, s.pad, s.pad, s.stride, s.stride, 1, 1, col,
            s.col_elems, 0, x, s.c * s.h * s.h, 0, batch), 4 * (2 * img + batch * s.col_elems)),
        "forward_bias": (lambda: hip.forwardBias(no, out, 0, s.filters, bias, 1, batch), 8 * no),
        "activate_leaky": (lambda: hip.ActivateArray(no, out, 0, 9), 8 * no),
        "means_and_vars": (lambda: hip.meansAndVars(ne, N, G, y, 0, m, v), 8 * ne),
        "means_and_vars_delta": (lambda: hip.meansAndVarsDelta(ne, N, G, d, y, 0, m, v, md, vd),
                                 8 * ne),
        "add_dots": (lambda: hip.addDots(ne, N, G, y, d, 0, dsc), 8 * ne),
        "normalize_delta": (lambda: hip.normalizeDelta(ne, N, G, d, y, 0, m, v, md, vd), 12 * ne),
    }
    res = {}
    for name, (fn, nbytes) in ops.items():
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        gbs = nbytes / (ms * 1e-3) / 1e9
        p = pmc.get(name, {})
        tr = (p.get("traffic_read_bytes") or 0) + (p.get("traffic_write_bytes") or 0) or None
        res[name] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
                     "traffic": tr, "algorithmic_bytes": nbytes, "ms": round(ms, 4)}
    res["_note"] = ("YOLOv3 batch 8: im2col/col2im/bias/activation on layer 3 (32x208x208 k3), "
                    "batch-norm reductions on 8x32x173056; traffic from " +
                    (str(cands[-1].relative_to(ROOT)) if cands else "none"))
    del x, col, out, y, d
    torch.cuda.empty_cache()
    return res


def bench_config1(steps=20):
    """BASELINE config 1: TSingleTensor.matMul 256x256x256 (beta = One,
    ntensors.pas:8059-8140) through the op-table drop-in (host pointers, HIP
    SGEMM) beside the restated CPU path (oracle sgemm_nn, host cores)."""
    from oracle import oracle as ora
    from tensorium_amd.ntensors import matMul
    n = 256
    a = ora.uniform(n * n, 1, 0).reshape(n, n)
    b = ora.uniform(n * n, 1, 1).reshape(n, n)
    c0 = np.zeros((n, n), np.float32)
    c = c0.copy()
    matMul(a, b, c)
    ref = c0.copy()
    ora.sgemm(False, False, n, n, n, 1.0, a, n, b, n, 1.0, ref, n)
    same = bool(np.array_equal(c, ref))
    t0 = time.perf_counter()
    for _ in range(steps):
        matMul(a, b, c)
    hip_ms = (time.perf_counter() - t0) / steps * 1e3
    t0 = time.perf_counter()
    for _ in range(steps):
        ora.sgemm(False, False, n, n, n, 1.0, a, n, b, n, 1.0, ref, n)
    cpu_ms = (time.perf_counter() - t0) / steps * 1e3
    flop = 2.0 * n ** 3
    return {"workload": "TSingleTensor.matMul 256x256x256 (beta=1)", "bit_exact_vs_cpu": same,
            "hip_op_table_ms": round(hip_ms, 4),
            "hip_op_table_gflops": round(flop / hip_ms / 1e6, 2),
            "cpu_port_ms": round(cpu_ms, 4), "cpu_port_gflops": round(flop / cpu_ms / 1e6, 2),
            "cpu_threads": ora.lib().ora_get_threads(),
            "note": "host pointers: both include nothing but the call; the HIP path moves "
                    "768 KB over PCIe per call"}


def host_cpus():
    """CPUs this process may use: the cgroup CPU quota (cpu.max) when set,
    else the affinity mask.  os.cpu_count() is the whole machine (on the GPU
    box many times the box's share)."""
    info = {"machine_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "cgroup_quota_cpus": None}
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = max(1, int(int(q) // int(period)))
    except Exception:
        pass
    info["threads_used"] = info["cgroup_quota_cpus"] or info["affinity_cpus"]
    return info


def bench_conv_backward(torch, hip, ctx, rank, steps=2):
    """Row f-2: TConvolutionalLayer.backward over the 75 YOLOv3-416 conv
    layers at batch 8 (tns_hip_conv_backward: derive, addSums, im2col,
    per-image NT dW in the sdot order, TN dX + col2im), synthetic delta.
    Work = dW for every layer + dX for layers 1..74: the first layer gets no
    state delta, as TNNet.Propagate leaves it (state := Default(TNNetState),
    nnet.pas:328-337 / 414-426), so its dX and col2im are skipped, as in
    nConvolutionLayer.pas:642 ("if assigned(state.delta)")."""
    from tensorium_amd.yolo import yolov3_conv_table
    specs = yolov3_conv_table()
    batch = 8
    layers = []
    max_ws = 0
    for s in specs:
        g = 5 * 100000 + rank * 1000 + s.index
        x = synthetic(torch, (batch, s.c, s.h, s.h), g, 0.0, 1.0)
        sc = float(np.sqrt(2.0 / (s.size * s.size * s.c)))
        w = synthetic(torch, (s.filters, s.K), g + 1, -sc, sc)
        out = synthetic(torch, (batch, s.filters, s.out_h, s.out_h), g + 2, -1.0, 1.0)
        delta = synthetic(torch, (batch, s.filters, s.out_h, s.out_h), g + 3, -1.0, 1.0)
        bu = torch.zeros(s.filters, device="cuda")
        wu = torch.zeros((s.filters, s.K), device="cuda")
        sd = torch.zeros((batch, s.c, s.h, s.h), device="cuda") if s.index > 0 else None
        layers.append((s, x, w, out, delta, bu, wu, sd))
        max_ws = max(max_ws, batch * s.K * s.out_h * s.out_h)
    ws = torch.empty(max(max_ws, 1), device="cuda")

    def step():
        for s, x, w, out, delta, bu, wu, sd in layers:
            hip.convBackward(batch, s.c, s.h, s.h, x, w, s.filters, s.size, s.stride, s.pad, 1,
                             s.activation, out, delta, bu, wu, ws, sd)

    def timed_pass(mode):
        # TNS_OPT_BWD_OVERLAP: 2 = pipelined (each layer's dW left running on
        # the context's side stream under the next layers' work; the device
        # synchronize below waits for all of it), 1 = dW and state.delta
        # concurrent within each call, joined before it returns
        hip.setBwdOverlap(mode)
        step()
        torch.cuda.synchronize()
        ctx.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        ctx.barrier()
        return ctx.max((time.perf_counter() - t0) / steps)

    wall_joined = timed_pass(1)
    wall = timed_pass(2)
    hip.setBwdOverlap(1)
    hip.finish()
    from tensorium_amd._abi import TNS_OP_GEMM, TNS_OP_IM2COL, TNS_OP_COL2IM
    hip.setTelemetry(True)
    step()
    split = {"gemm_ms": round(hip.opMs(TNS_OP_GEMM), 3),
             "im2col_ms": round(hip.opMs(TNS_OP_IM2COL), 3),
             "col2im_ms": round(hip.opMs(TNS_OP_COL2IM), 3)}
    hip.setTelemetry(False)
    gflop = sum(s.flops * (2 if s.index > 0 else 1) for s in specs) * batch / 1e9
    del layers, ws
    torch.cuda.empty_cache()
    return {"layers": len(specs), "batch_per_gpu": batch, "ms_per_batch": round(wall * 1e3, 3),
            "schedule": "pipelined (TNS_OPT_BWD_OVERLAP = 2: each layer's dW on the side "
                        "stream under the following layers' work) — the schedule the Pascal "
                        "drop-in selects (pascal/nnHip.pas initHIP, pipelineBackward = true); "
                        "ms_per_batch_joined: the C library's default (1)",
            "ms_per_batch_joined": round(wall_joined * 1e3, 3),
            "gflop_per_batch": round(gflop, 2), "tflops": round(gflop / wall / 1e3, 2),
            "images_per_s_total": round(ctx.world * batch / wall, 1),
            "telemetry_split": split}


def bench_train_backward(torch, hip, ctx, steps=3):
    """The backward the drop-in runs in YOLOv3-416 training, batch 8:
    TNet.backward over all 107 layers in the reference's order
    (darknet.HipDarknetTrain: the 72 batch-normalized conv layers on
    tns_hip_conv_backward_bn — Derivative, addDots, forwardScale,
    MeansAndVarsDelta, normalizeDelta, dW, state.delta — the 3 heads on
    tns_hip_conv_backward, each shortcut's DeriveArray + two addvv, the
    routes' addvv, the upsamples' accumulation and the yolo layers' axpy),
    after one training forward (BN statistics of the batch) with synthetic
    yolo deltas (the yolo loss is out of scope).  Each pass starts from the
    same deltas (reset outside the timed region); wall time from the first
    call to a device synchronize after the last, pipelined (the Pascal
    binding's default) and joined."""
    from tensorium_amd import darknet as dn
    net = dn.Network(dn.parse_cfg(dn.yolov3_cfg(416)), 8)
    model = dn.HipDarknetTrain(hip, net, dn.random_params(net, seed=3), torch)
    x = synthetic(torch, (8, 3, 416, 416), 7 * 100000 + ctx.rank, 0.0, 1.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.forward(x)
    torch.cuda.synchronize()
    fwd_ms = (time.perf_counter() - t0) * 1e3
    ys = [l for l in net.layers if l.kind == "yolo"]
    yd = [synthetic(torch, (8 * l.out_size,), 7 * 200000 + l.index, -0.1, 0.1) for l in ys]

    def reset():
        hip.finish()
        for d in model.delta:
            d.zero_()
        model.set_yolo_deltas(yd)
        torch.cuda.synchronize()

    def timed(mode):
        hip.setBwdOverlap(mode)
        reset()
        model.backward(x)          # (warm: scratch sized, k-tables built)
        ts = []
        for _ in range(steps):
            reset()
            ctx.barrier()
            t0 = time.perf_counter()
            model.backward(x)
            hip.finish()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return ctx.max(float(np.mean(ts)))

    joined = timed(1)
    piped = timed(2)
    # which calls drained the pipeline (untimed pass: a ctypes query per layer)
    reset()
    trace = []
    model.backward(x, lambda l: trace.append((l.index, l.kind, hip.pendingDw())))
    hip.finish()
    hip.setBwdOverlap(1)
    drains = [(i, k) for (i, k, n), (_, _, m) in zip(trace[1:], trace[:-1])
              if n < m and k != "convolutional"]
    convs = net.convs()
    gflop = sum(2 * l.filters * l.out_h * l.out_w * l.c * l.size * l.size * (2 if l.index else 1)
                for l in convs) * 8 / 1e9
    del model
    torch.cuda.empty_cache()
    return {"layers": len(net.layers), "conv_layers": len(convs),
            "bn_conv_layers": sum(1 for l in convs if l.bn), "batch_per_gpu": 8,
            "ms_per_batch": round(piped * 1e3, 3), "ms_per_batch_joined": round(joined * 1e3, 3),
            "conv_gflop_per_batch": round(gflop, 2),
            "tflops_conv": round(gflop / piped / 1e3, 2),
            "images_per_s_total": round(ctx.world * 8 / piped, 1),
            "training_forward_ms": round(fwd_ms, 3),
            "max_pending_dw": max(n for _, _, n in trace),
            "non_conv_calls_that_joined": drains,
            "schedule": "pipelined (TNS_OPT_BWD_OVERLAP = 2, pascal/nnHip.pas initHIP default); "
                        "ms_per_batch_joined: 1 (each call joined before it returns)",
            "data": "synthetic input, random-init parameters, synthetic yolo deltas U[-0.1,0.1)"}


def bench_yolo_network(torch, hip, ctx, steps):
    """The whole YOLOv3-416 network (yolov3.cfg plan: 75 convolutions chained
    through shortcut / route / upsample / yolo, darknet.HipDarknet), batch 8
    per GPU, BN-folded synthetic parameters."""
    from tensorium_amd import darknet as dn
    net = dn.Network(dn.parse_cfg(dn.yolov3_cfg(416)), 8)
    model = dn.HipDarknet(hip, net, dn.random_params(net, seed=3), torch)
    x = synthetic(torch, (8, 3, 416, 416), 3 * 100000 + ctx.rank, 0.0, 1.0)
    model.forward(x)
    torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        model.forward(x)
    torch.cuda.synchronize()
    ctx.barrier()
    ms = ctx.max((time.perf_counter() - t0) / steps * 1e3)
    return {"layers": len(net.layers), "batch_per_gpu": 8, "ms_per_batch": round(ms, 4),
            "images_per_s": round(ctx.world * 8 / (ms / 1e3), 2)}


def bench_batched(torch, hip, ctx, n_gemm=1024, n=1024, steps=3):
    """Config 4: n_gemm independent n^3 GEMMs, contiguous shard per rank, one
    strided-batched launch per step, operands generated on each device."""
    from tensorium_amd.shard import shard_range
    lo, hi = shard_range(n_gemm, ctx.rank, ctx.world)
    mine = hi - lo
    A = synthetic(torch, (mine, n, n), 4 * 1000 + lo)
    B = synthetic(torch, (mine, n, n), 4 * 2000 + lo)
    Cm = torch.empty((mine, n, n), device="cuda")

    def step():
        hip.gemmStridedBatched(False, False, n, n, n, 1.0, A, 0, n, n * n, B, 0, n, n * n, 0.0,
                               Cm, 0, n, n * n, mine)

    step()
    torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ctx.barrier()
    wall = ctx.max((time.perf_counter() - t0) / steps)
    del A, B, Cm
    torch.cuda.empty_cache()
    flop = 2.0 * n ** 3 * n_gemm
    return {"gemms_total": n_gemm, "gemm_size": n, "gemms_per_rank_max": -(-n_gemm // ctx.world),
            "ms_per_batch": round(wall * 1e3, 4), "tflops_total": round(flop / wall / 1e12, 3),
            "scaling": "strong (fixed 1024 GEMMs split over ranks)"}


def bench_host_api(n, steps=3):
    """Boundary A (host pointers, the reference's `gemm` op-table slot):
    tns_cblas_sgemm on pageable numpy arrays: H2D of A and B, the kernel and
    D2H of C inside each call, pipelined by row chunks of C over a copy
    stream (strict beta = 0 is 0*C, so C is uploaded too: 268 MB per call).
    Reported as the PCIe-inclusive rate beside `value`, never as `value`."""
    from tensorium_amd.ntensors import bind_hip_op_table
    ops = bind_hip_op_table()
    rng = np.random.default_rng(6)
    A = rng.uniform(-1, 1, (n, n)).astype(np.float32)
    B = rng.uniform(-1, 1, (n, n)).astype(np.float32)
    C = np.zeros((n, n), np.float32)

    def call():
        ops.gemm(101, 111, 111, n, n, n, 1.0, A.ctypes.data, n, B.ctypes.data, n, 0.0,
                 C.ctypes.data, n)

    call()
    t0 = time.perf_counter()
    for _ in range(steps):
        call()
    ms = (time.perf_counter() - t0) / steps * 1e3
    return {"entry": "tns_cblas_sgemm (host pointers, pageable)", "ms_per_call": round(ms, 3),
            "gflops_pcie_inclusive": round(2.0 * n ** 3 / ms / 1e6, 1),
            "bytes_moved_per_call": 4 * n * n * 4,
            "pcie_bound_ms": round(4 * n * n * 4 / 56e9 * 1e3, 3),
            "pcie_note": "56 GB/s per direction and total on the box (profiles/r02_pcie.json)"}


def bench_mnist(torch, hip, ctx, steps=200):
    """Config 5: fused connected-network train step (784-64x4-32-10, BN,
    softmax), batch 32, replicas per rank."""
    from tensorium_amd.nnhip import TNNHip
    widths = [784, 64, 64, 64, 64, 32, 10]
    acts = [1, 1, 1, 1, 1, 4]
    B = 32
    nbuf = TNNHip.mlpBufferFloats(widths, True, B)
    buf = torch.zeros(nbuf, device="cuda")
    # W ~ U[-sqrt(2/in), sqrt(2/in)], scales 1 (TConnectedLayer.Create)
    off = 0
    for l in range(len(widths) - 1):
        I, O = widths[l], widths[l + 1]
        r = float(np.sqrt(2.0 / I))
        buf[off:off + I * O] = synthetic(torch, (I * O,), 5 * 100 + l, -r, r)
        off += 2 * I * O + 2 * O
        buf[off:off + O] = 1.0
        off += 4 * O + 4 * B * O + 4 * O
    X = synthetic(torch, (B, 784), 5 * 1000 + ctx.rank, 0.0, 1.0)
    lab = torch.randint(0, 10, (B,), device="cuda")
    T = torch.zeros(B, 10, device="cuda")
    T[torch.arange(B, device="cuda"), lab] = 1.0
    cost = torch.zeros(1, device="cuda")

    def step():
        hip.mlpTrainStep(widths, acts, True, B, X, T, 1e-3, 0.9, 1e-4, buf, cost)

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ctx.barrier()
    wall = ctx.max((time.perf_counter() - t0) / steps)
    return {"batch": B, "net": "784-64-64-64-64-32-10 relu/linear + BN + softmax",
            "us_per_step": round(wall * 1e6, 2), "steps_per_s_total": round(ctx.world / wall, 1),
            "kernels_per_step": 3, "cost_after": round(float(cost.item()), 4)}


def cpu_baseline(n, target_s):
    """Oracle sgemm_nn (port of the reference CPU path) on a row sample."""
    from oracle import oracle as ora
    cpus = host_cpus()
    threads = int(os.environ.get("TNS_ORACLE_THREADS") or cpus["threads_used"])
    ora.set_threads(threads)
    A = ora.uniform(n * n, 2, 0).reshape(n, n)
    B = ora.uniform(n * n, 2, 1).reshape(n, n)
    C = np.zeros((n, n), np.float32)
    rows = max(threads, 16)
    t0 = time.perf_counter()
    ora.sgemm_rows(False, False, 0, rows, n, n, n, 1.0, A, n, B, n, 0.0, C, n)
    dt = time.perf_counter() - t0
    more = int(rows * max(target_s - dt, 0.0) / max(dt, 1e-9))
    more = min(more, n - rows)
    more -= more % threads if more > threads else 0
    if more > 0:
        t1 = time.perf_counter()
        ora.sgemm_rows(False, False, rows, rows + more, n, n, n, 1.0, A, n, B, n, 0.0, C, n)
        dt2 = time.perf_counter() - t1
        rows_t, secs = more, dt2
    else:
        rows_t, secs = rows, dt
    gflops = 2.0 * rows_t * n * n / secs / 1e9
    out = {"value": round(gflops, 3), "unit": "GFLOP/s", "cores": threads, "kind": "port",
           "sample": f"{rows_t} of {n} rows of the {n}^3 NN product "
                     f"(restated sgemm_nn/saxpy_avx2 FMA chain, {secs:.1f} s)",
           "host": cpus}
    out.update(cpu_yolo_mnist())
    return out


def cpu_yolo_mnist():
    """The oracle's restated conv-layer forward (im2col + sgemm_nn + bias +
    activation, same thread count) over all 75 YOLOv3 conv layers for one
    image, and the restated MNIST train step."""
    from oracle import oracle as ora
    from tensorium_amd.yolo import yolov3_conv_table
    table = yolov3_conv_table()
    flop_img = sum(s.flops for s in table)
    t_flop, t_sec = 0.0, 0.0
    for idx, s in enumerate(table):
        x = ora.uniform(s.c * s.h * s.h, 3, idx, 0.0, 1.0).reshape(1, s.c, s.h, s.h)
        sc = float(np.sqrt(2.0 / (s.size * s.size * s.c)))
        w = ora.uniform(s.filters * s.K, 4, idx, -sc, sc)
        b = ora.uniform(s.filters, 5, idx, -0.1, 0.1)
        t0 = time.perf_counter()
        ora.conv_forward(x, w, b, s.filters, s.size, s.stride, s.pad, s.activation)
        t_sec += time.perf_counter() - t0
        t_flop += s.flops
    widths, acts, B = [784, 64, 64, 64, 64, 32, 10], [1, 1, 1, 1, 1, 4], 32
    buf = ora.mlp_init(widths, 1, B)
    X, T = ora.mnist_batch(B)
    ora.mlp_train_step(widths, acts, 1, B, X, T, 1e-3, 0.9, 1e-4, buf)
    steps, t0 = 0, time.perf_counter()
    while steps < 50 and time.perf_counter() - t0 < 2.0:
        ora.mlp_train_step(widths, acts, 1, B, X, T, 1e-3, 0.9, 1e-4, buf)
        steps += 1
    mnist_s = (time.perf_counter() - t0) / steps
    return {"yolo_images_per_s": round(t_flop / t_sec / flop_img, 4),
            "yolo_sample": f"one image through all 75 conv layers ({t_flop / 1e9:.2f} GFLOP "
                           f"in {t_sec:.2f} s)",
            "mnist_steps_per_s": round(1.0 / mnist_s, 2),
            "mnist_sample": f"{steps} restated train steps (batch 32, BN)"}


def traffic_from_profiles(n):
    """HBM bytes per sgemm launch from the committed rocprofv3 PMC pass."""
    cands = sorted(ROOT.glob("profiles/*sgemm_traffic*.json"))
    if not cands:
        return None, None
    try:
        d = json.loads(cands[-1].read_text())
        if int(d.get("size", 0)) == n and d.get("bytes_per_launch"):
            return float(d["bytes_per_launch"]), str(cands[-1].relative_to(ROOT))
    except Exception:
        pass
    return None, None


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    if args.dry_run:
        dry_run(args)
        return
    import torch
    from tensorium_amd import dist as tdist
    ctx = tdist.init("nccl")
    if ctx.world != args.gpus:
        raise SystemExit(f"bench.py: {ctx.world} ranks but --gpus {args.gpus}")
    rank, world, local = ctx.rank, ctx.world, ctx.local
    from tensorium_amd.nnhip import TNNHip
    hip = TNNHip(ctx.gpu)
    n = args.size

    # The secondary workloads run first and the headline SGEMM last, so that
    # its K timed steps run at the clock the chip holds under sustained load:
    # a cold GPU ramps over its first ~20 launches (4096^3: 1.88 ms, then
    # 1.21 -> 1.0 ms; profiles/r01_clock_ramp.json), which a short warm-up
    # alone would leave inside the timed region.
    yolo = None
    if not args.no_yolo and args.yolo_steps > 0:
        y = bench_yolo(torch, hip, ctx, rank, args.yolo_steps)
        ms = ctx.max(y["ms_per_batch"])
        y["ms_per_batch"] = ms
        y["images_per_s"] = world * y["batch_per_gpu"] / (ms / 1e3)
        yolo = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in y.items()}

    yolo_net = None
    if not args.no_yolo and args.yolo_steps > 0:
        yolo_net = bench_yolo_network(torch, hip, ctx, args.yolo_steps)
    conv_bwd = None
    if not args.no_yolo and args.yolo_steps > 0:
        conv_bwd = bench_conv_backward(torch, hip, ctx, rank)
    train_bwd = None
    if not args.no_yolo and args.yolo_steps > 0:
        train_bwd = bench_train_backward(torch, hip, ctx)
    ew = None if args.no_yolo else bench_elementwise_roofline(torch, hip)
    yolo_dp = None
    if not args.no_yolo and args.yolo_steps > 0:
        yolo_dp = bench_yolo_dp(torch, hip, ctx, args.yolo_steps)
    mnist = None if args.no_mnist else bench_mnist(torch, hip, ctx)
    # (the MFMA-bound config 4 right before the headline: the clock settles
    # under MFMA load, not under the latency-bound train step)
    batched = None if args.no_batched else bench_batched(torch, hip, ctx)

    wall, kern_ms, kern_min = bench_sgemm(torch, hip, ctx, rank, n, args.steps, args.warmup)
    wall = ctx.max(wall)
    flop = 2.0 * n * n * n
    ms_per_step = wall / args.steps * 1e3
    value = world * flop / (ms_per_step / 1e3) / 1e9   # GFLOP/s, whole job
    achieved = flop / (kern_ms * 1e-3) / 1e12            # TFLOP/s, per launch
    traffic, traffic_src = traffic_from_profiles(n)
    host_api = bench_host_api(n) if rank == 0 and world == 1 and not args.no_cpu else None
    config1 = None
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            config1 = bench_config1()
        except Exception as e:  # reported, never required
            config1 = {"error": str(e)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            cpu = cpu_baseline(n, args.cpu_seconds)
        except Exception as e:  # the baseline is reported, never required
            cpu = {"value": None, "error": str(e)}

    if rank == 0:
        line = {
            "metric": "fp32 SGEMM GFLOP/s (M=N=K=4096) + YOLOv3 conv-fwd images/s",
            "value": round(value, 2),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic U[-1,1) operands generated on device (torch RNG), resident in HBM",
            "config": {"workload": f"sgemm_nn_{n}x{n}x{n}", "M": n, "N": n, "K": n,
                       "alpha": 1.0, "beta": 0.0, "gemms_per_gpu_per_step": 1,
                       "parallelism": f"{world} independent replicas, one process per GPU, "
                                      "no data-path collective"},
            "roofline": {"bound": "mfma", "kernel": "sgemm_nn_w4_kernel (256x256x32, 4 waves of 128x128 at one wave per SIMD, LDS-DMA operands; form 256x256x32_w2x2_dma_nn_big)",
                         "achieved": round(achieved, 3), "peak": PEAK_F32_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_F32_TFLOPS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel_ms_mean": round(kern_ms, 4), "kernel_ms_min": round(kern_min, 4),
                         "algorithmic_flop_per_launch": flop},
            "elementwise_roofline": ew,
            "cpu_baseline": cpu,
            "yolo": yolo,
            "yolo_network": yolo_net,
            "yolo_conv_backward": conv_bwd,
            "yolo_train_backward": train_bwd,
            "yolo_dp": yolo_dp,
            "config1_matmul": config1,
            "batched_gemm": batched,
            "mnist_train": mnist,
            "host_api": host_api,
        }
        print(json.dumps(line), flush=True)
    hip.finish()
    hip.close()
    ctx.close()


if __name__ == "__main__":
    main()
