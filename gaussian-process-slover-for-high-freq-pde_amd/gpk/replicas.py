"""Multi-GPU execution of the hot path: replicas.

One process per GPU (launched by `python -m torch.distributed.run`, env RANK / WORLD_SIZE /
LOCAL_RANK).  Each rank owns independent solver problems — the reference's `num_fold` loop
(code/model_GP_solver_2d.py:423-443, code/model_GP_solver_1d.py:366-377) or a bench replica —
so the data path has no collective.  The only cross-rank traffic is control: a barrier around
timed regions, a MAX of the per-rank elapsed time, and a gather of per-fold results.  Backend
"nccl" is RCCL on ROCm (GPU ranks); "gloo" runs the same code on CPU (tests).
"""
import os
from dataclasses import dataclass


@dataclass
class Ctx:
    world: int = 1
    rank: int = 0
    local: int = 0
    backend: str = ""

    @property
    def device(self):
        return self.local


def init(backend=None):
    """Join the process group if launched with WORLD_SIZE > 1; returns the rank context."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world <= 1:
        return Ctx(1, 0, local, "")
    import torch.distributed as dist
    backend = backend or "nccl"
    if not dist.is_initialized():
        if backend == "nccl":
            import torch
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    return Ctx(world, rank, local, backend)


def shutdown(ctx):
    if ctx.world > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def owned(n_items, ctx):
    """Items this rank owns: round-robin i = rank, rank + world, ... (disjoint, covering)."""
    return list(range(ctx.rank, n_items, ctx.world))


def _tensor(x, ctx):
    import torch
    dev = f"cuda:{ctx.local}" if ctx.backend == "nccl" else "cpu"
    return torch.tensor([float(x)], dtype=torch.float64, device=dev)


def barrier(ctx):
    if ctx.world > 1:
        import torch.distributed as dist
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.local])
        else:
            dist.barrier()


def max_over_ranks(x, ctx):
    if ctx.world == 1:
        return float(x)
    import torch.distributed as dist
    t = _tensor(x, ctx)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, ctx):
    if ctx.world == 1:
        return float(x)
    import torch.distributed as dist
    t = _tensor(x, ctx)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_by_index(local_items, n_items, ctx):
    """Reassemble {index: value} dicts produced under `owned()` into a list ordered by index
    (every rank gets the full list)."""
    if ctx.world == 1:
        return [local_items[i] for i in range(n_items)]
    import torch.distributed as dist
    parts = [None] * ctx.world
    dist.all_gather_object(parts, dict(local_items))
    merged = {}
    for p in parts:
        merged.update(p)
    return [merged[i] for i in range(n_items)]
