"""One process per GPU over torch.distributed (RCCL on ROCm; gloo for CPU tests).

Stripes are independent objects: a batch is split into contiguous
near-equal stripe ranges, one per rank, with NO data-path collective.  The only
collectives are control: a barrier around timed regions, the max of per-rank
elapsed times, and the AND of per-rank parity checks.
"""
from __future__ import annotations

import os
from typing import List, Tuple


def world() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend: str = "nccl") -> None:
    import torch
    import torch.distributed as dist

    rank, local, ws = world()
    if ws <= 1 or dist.is_initialized():
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = {}
    rdzv = os.environ.get("RSGPU_RDZV_FILE")
    if rdzv:
        # bench.py's own launcher: a file store in a fresh directory, so no TCP port is
        # picked by one process and bound by another later (a port
        # freed by the launcher could be taken before rank 0 bound it)
        kw = {"init_method": "file://" + rdzv, "rank": rank, "world_size": ws}
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"), **kw)
    else:
        dist.init_process_group(backend, **kw)


def stripe_range(n_stripes: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous [begin, end) share of a batch for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n_stripes, world_size)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def _device():
    import torch
    import torch.distributed as dist

    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")


def barrier() -> None:
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier()


def max_over_ranks(x: float) -> float:
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_true(flag: bool) -> bool:
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return flag
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=_device())
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def gather_floats(x: float) -> List[float]:
    """Every rank's value of x, in rank order (on every rank)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return [x]
    ws = dist.get_world_size()
    t = torch.tensor([x], dtype=torch.float64, device=_device())
    out = [torch.zeros_like(t) for _ in range(ws)]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def distinct_count(key: int) -> int:
    """How many distinct values of `key` the ranks hold (e.g. how many physical GPUs
    a run used: ranks may share one when rehearsing the N > 1 path)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return 1
    ws = dist.get_world_size()
    t = torch.tensor([key], dtype=torch.int64, device=_device())
    out = [torch.zeros_like(t) for _ in range(ws)]
    dist.all_gather(out, t)
    return len({int(x.item()) for x in out})


def shutdown() -> None:
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
