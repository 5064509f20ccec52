"""Multi-rank path of config 4 (independent GEMMs sharded over ranks) on CPU
with the gloo backend, world size 2 and 3: shards cover the batch exactly
once, the per-GEMM checksums gathered over ranks equal a single-process run,
and the timing reduction takes the max over ranks.  The GEMMs themselves are
computed by the oracle here (no GPU in this container)."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_gemm, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, str(ROOT))
    try:
        from oracle import oracle as ora
        from tensorium_amd import dist as tdist
        from tensorium_amd.shard import shard_range
        ctx = tdist.init("gloo")
        ora.set_threads(1)
        lo, hi = shard_range(n_gemm, ctx.rank, ctx.world)
        sums = []
        for g in range(lo, hi):
            A = ora.uniform(n * n, 4, 2 * g)
            B = ora.uniform(n * n, 4, 2 * g + 1)
            C = np.zeros(n * n, np.float32)
            ora.sgemm(False, False, n, n, n, 1.0, A, n, B, n, 0.0, C, n)
            sums.append(float(C.astype(np.float64).sum()))
        # pad to equal length for all_gather
        per = -(-n_gemm // ctx.world)
        padded = sums + [float("nan")] * (per - len(sums))
        gathered = ctx.gather_floats(padded)
        t_max = ctx.max(float(rank + 1))
        total = ctx.sum(float(hi - lo))
        ctx.barrier()
        ctx.close()
        q.put((rank, gathered, t_max, total))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None, None))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_batched_gemm_gloo(ora, world):
    import torch.multiprocessing as mp
    n_gemm, n = 7, 24
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_gemm, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort()
    for r in res:
        assert not isinstance(r[1], str), r[1]
    gathered = res[0][1]
    flat = [v for rank_vals in gathered for v in rank_vals if not np.isnan(v)]
    assert len(flat) == n_gemm
    # single-process reference, same (seed, gemm index) operands
    ref = []
    for g in range(n_gemm):
        A = ora.uniform(n * n, 4, 2 * g)
        B = ora.uniform(n * n, 4, 2 * g + 1)
        C = np.zeros(n * n, np.float32)
        ora.sgemm(False, False, n, n, n, 1.0, A, n, B, n, 0.0, C, n)
        ref.append(float(C.astype(np.float64).sum()))
    assert flat == ref
    assert all(r[2] == float(world) for r in res)      # max over ranks
    assert all(r[3] == float(n_gemm) for r in res)     # every unit exactly once


def test_shard_range_partitions():
    from tensorium_amd.shard import all_shards
    for n in (0, 1, 7, 1024, 1023):
        for w in (1, 2, 3, 8):
            sh = all_shards(n, w)
            covered = [i for a, b in sh for i in range(a, b)]
            assert covered == list(range(n))
            sizes = [b - a for a, b in sh]
            assert max(sizes) - min(sizes) <= 1


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, str(ROOT))
    try:
        import torch
        from oracle import oracle as ora
        from tensorium_amd import dist as tdist
        from tensorium_amd.shard import shard_range
        ctx = tdist.init("gloo")
        ora.set_threads(1)
        batch, C, H, F, k = 8, 3, 9, 4, 3
        # weights exist on rank 0 only; one broadcast of the packed buffer
        if ctx.rank == 0:
            w = torch.from_numpy(ora.uniform(F * C * k * k, 7, 0, -0.3, 0.3))
            b = torch.from_numpy(ora.uniform(F, 7, 1, -0.1, 0.1))
        else:
            w, b = torch.zeros(F * C * k * k), torch.zeros(F)
        flat, meta = tdist.pack_flat(torch, [w, b], "cpu")
        ctx.broadcast(flat, src=0)
        w, b = (t.numpy().copy() for t in tdist.unpack_flat(flat, meta))
        lo, hi = shard_range(batch, ctx.rank, ctx.world)
        sums = []
        for g in range(lo, hi):
            x = ora.uniform(C * H * H, 8, g, 0.0, 1.0).reshape(1, C, H, H)
            y = ora.conv_forward(x, w, b, F, k, 1, 1, 9)
            sums.append(float(y.astype(np.float64).sum()))
        per = -(-batch // ctx.world)
        gathered = ctx.gather_floats(sums + [float("nan")] * (per - len(sums)))
        ctx.barrier()
        ctx.close()
        q.put((rank, gathered))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_yolo_image_sharded_with_weight_broadcast_gloo(ora, world):
    """Config 3's data-parallel path (bench.py bench_yolo_dp): weights on rank
    0 only reach every rank by one broadcast of the packed buffer; images
    split by shard_range; the per-image results equal one process."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert not isinstance(r[1], str), r[1]
    flat = [v for per_rank in res[0][1] for v in per_rank if not np.isnan(v)]
    w = ora.uniform(4 * 27, 7, 0, -0.3, 0.3)
    b = ora.uniform(4, 7, 1, -0.1, 0.1)
    ref = []
    for g in range(8):
        x = ora.uniform(3 * 81, 8, g, 0.0, 1.0).reshape(1, 3, 9, 9)
        ref.append(float(ora.conv_forward(x, w, b, 4, 3, 1, 1, 9).astype(np.float64).sum()))
    assert flat == ref
