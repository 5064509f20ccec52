"""Sharding of independent GEMMs across ranks (BASELINE config 4).

The reference has no multi-device code at all ("todo ... implement multi
GPU", nConvolutionLayer.pas:472, 498).  Config 4's units — 1024 independent
1024^3 GEMMs — need no data exchange: each rank (one process per GPU) takes a
contiguous block of GEMM indices, generates its operands on its own device
from (seed, gemm index) and runs them as one strided-batched launch.  The
only collectives are the timing barrier / max-reduction of the benchmark and
an optional checksum all-reduce used to verify that the shards cover the
whole batch exactly once.
"""
from __future__ import annotations


def shard_range(n_units: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [start, stop) of n_units for `rank` of `world`; the
    first n_units % world ranks get one extra unit (same rule as the
    reference's TOPool.&For contiguous groups, steroids.pas:606-641)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_units, world)
    start = rank * base + min(rank, extra)
    stop = start + base + (1 if rank < extra else 0)
    return start, stop


def all_shards(n_units: int, world: int) -> list[tuple[int, int]]:
    return [shard_range(n_units, r, world) for r in range(world)]
