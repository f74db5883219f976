"""Row-sharded multi-GPU step of the 2D solvers.

One process per GPU (torch.distributed.run).  Rank 0 creates a 128-byte RCCL communicator id,
torch.distributed hands the same bytes to every rank, and each rank opens its libgpk handle
with gpk_create_sharded: the step then runs its rows of every product and exchanges row blocks
/ partial sums over RCCL (xGMI) inside the step's hipGraph.  torch.distributed is used only for
the id exchange and the timing barrier -- the data path is libgpk's own RCCL calls.
"""
from . import replicas
from .core import DeviceSolver, comm_unique_id


def broadcast_comm_id(ctx, make_id=None):
    """The RCCL id of rank 0 on every rank (gloo or nccl process group; world 1: local)."""
    make_id = make_id or comm_unique_id
    if ctx.world == 1:
        return make_id()
    import torch.distributed as dist
    obj = [make_id() if ctx.rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    cid = obj[0]
    if not isinstance(cid, (bytes, bytearray)) or len(cid) != 128:
        raise RuntimeError("bad RCCL communicator id")
    return bytes(cid)


def make_sharded_solver(config, ctx, seed=0, Q=30, lr=0.01, flags=0):
    """A row-sharded DeviceSolver for a 2D BASELINE config (same synthetic data on every rank)."""
    import numpy as np
    from .problems import CONFIGS, problem_arrays
    cfg = CONFIGS[config] if isinstance(config, str) else config
    if cfg["dim"] != 2:
        raise ValueError("row sharding is for the 2D (Kronecker) solvers")
    arr = problem_arrays(cfg)
    eq = {"poisson_2d": "poisson", "allencahn_2d": "allencahn", "advection": "advection"}[
        cfg["equation"].split("-")[0]]
    cid = broadcast_comm_id(ctx)
    s = DeviceSolver(2, eq, cfg["kernel"], arr["x1"], arr["src"], arr["bvals"], x2=arr["x2"], Q=Q,
                     llk_weight=cfg["llk_weight"], beta=cfg.get("beta", 1.0), lr=lr,
                     freq_scale=cfg["freq_scale"], device=ctx.local, flags=flags,
                     shard=(ctx.rank, ctx.world, cid))
    flat = s.get_flat()
    nu = cfg["n"] * cfg["n"]
    flat[:nu] = 0.1 * np.random.default_rng(seed).normal(size=nu)  # same U on every rank
    s.set_flat(flat)
    replicas.barrier(ctx)
    return s
