"""One-process-per-GPU plumbing for the benchmark and multi-GPU runs.

torch.distributed carries rendezvous, barriers and scalar reductions
(timing max, checksums) everywhere; the only data-path collective is the
one-time broadcast of the YOLOv3 weights before the image-sharded forward
 — the independent GEMMs of config 4 exchange nothing.
Backend "nccl" is RCCL on ROCm (over xGMI between the GPUs of a node);
"gloo" is used by the CPU tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class DistCtx:
    dist: object | None
    rank: int
    world: int
    local: int
    device: str
    gpu: int = 0  # HIP device of this rank

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def _reduce(self, x: float, op_name: str) -> float:
        if self.dist is None:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op_name))
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, "MAX")

    def sum(self, x: float) -> float:
        return self._reduce(x, "SUM")

    def gather_floats(self, xs: list[float]) -> list[list[float]]:
        """All-gather a short list of floats from every rank (equal lengths)."""
        if self.dist is None:
            return [list(xs)]
        import torch
        t = torch.tensor(xs, dtype=torch.float64, device=self.device)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.tolist() for o in out]

    def broadcast(self, t, src: int = 0):
        """Broadcast one tensor (on this rank's device for RCCL) from src, in
        place.  One call per packed buffer: pack small tensors first
        (pack_flat) so the exchange is one large collective."""
        if self.dist is not None:
            self.dist.broadcast(t, src=src)
        return t

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


def init(backend: str | None = None, use_gpu: bool = True) -> DistCtx:
    """Initialise from RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* (torchrun or
    bench.py's own launcher).  Single process when WORLD_SIZE is unset or 1.
    use_gpu=False (launcher rehearsal) never touches the GPU: gloo only."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    # TNS_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share
    # devices round-robin; RCCL needs one device per rank)
    if use_gpu:
        backend = os.environ.get("TNS_DIST_BACKEND") or backend
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
    else:
        backend = "gloo"
    device = "cpu"
    gpu = 0
    if use_gpu and torch.cuda.is_available():
        ndev = max(torch.cuda.device_count(), 1)
        if backend == "nccl" and world > ndev:
            raise RuntimeError(f"{world} ranks over RCCL need {world} GPUs, {ndev} visible "
                               f"(TNS_DIST_BACKEND=gloo rehearses more ranks than GPUs)")
        gpu = local % ndev
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            device = f"cuda:{gpu}"
    if world <= 1:
        return DistCtx(None, 0, 1, local, device, gpu)
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = {}
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", gpu)
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return DistCtx(dist, rank, world, local, device, gpu)


def pack_flat(torch, tensors, device, align: int = 4):
    """One contiguous fp32 buffer holding `tensors` back to back, each
    starting on a multiple of `align` floats (16 bytes: the kernels' float4 /
    aligned-weight paths apply to the views as to separately allocated
    tensors), and the (offset, shape) list to view them out of it again
    (unpack_flat)."""
    meta, off = [], 0
    for t in tensors:
        meta.append((off, tuple(t.shape)))
        off += -(-int(t.numel()) // align) * align
    flat = torch.zeros(max(off, 1), dtype=torch.float32, device=device)
    for t, (o, _) in zip(tensors, meta):
        flat[o:o + int(t.numel())].copy_(t.reshape(-1))
    return flat, meta


def unpack_flat(flat, meta):
    return [flat[o:o + _numel(shape)].view(*shape) for o, shape in meta]


def _numel(shape) -> int:
    n = 1
    for d in shape:
        n *= int(d)
    return n
