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


# ------------------------------------------------------------------------------------------
# The sharded step's plan (csrc/gpk_api.cpp build_shard; gpk_shard_plan returns the library's)
# ------------------------------------------------------------------------------------------
PADM = 32  # padding multiple of a matrix dimension (gpk_api.cpp make_layout), x nranks when sharded


def shard_rows(n, nranks, rank):
    """Rows [r0, r1) of a P-row output that `rank` computes: P = n padded to 32 * nranks, block
    height P / nranks (the last ranks' blocks may lie in the padding: r0 >= r1)."""
    m = PADM * nranks
    p = (n + m - 1) // m * m
    h = p // nranks
    r0 = rank * h
    return min(r0, n), min(n, r0 + h), h


def shard_plan(aug, refine_fwd=True, refine_rev=True, refine_fwd2=True):
    """The plan the library builds for a row-sharded 2D handle (gpk_api.cpp build_shard):
    "s<k>:<modes>" per GEMM stage with products -- r = this rank's output rows, k = its share of
    the contraction index, f = whole (replicated) -- and " g<buf>" per all-gather after the
    stage; then "ar" (the step's one all-reduce) and "gU" (U rows after Adam).

    aug: the augmented chain inverse (small factors: A, Bt and K^{-1} D^T whole on every rank);
    refine_fwd / refine_rev: the gated refinement stages of the forward solves (A, Bt) and of
    the reverse-pass solves (S, X) are in the graph (build_descs); refine_fwd2: Bt's forward
    refinement too (large factors at beta >= 16 -- advection, C5 -- refine A alone)."""
    out = []

    def stage(k, modes, gathers=()):
        if modes:
            out.append(f"s{k}:{modes}")
        out.extend(f"g{g}" for g in gathers)

    if not aug:
        stage(0, "rr", ("A",) if refine_fwd else ())
    if refine_fwd:
        m = ("f" if aug else "r") * (2 if refine_fwd2 else 1)
        stage(1, m, () if aug else ("W1",))
        stage(2, m, () if aug else ("A",))
    elif not aug:
        out.append("gA")
    stage(3, "rr", ("R",))
    if refine_rev:
        stage(4, "r")
        stage(5, "r")
    stage(6, "frrk" if aug else "rrrk", () if aug else ("T1",))
    if not aug:
        stage(7, "rr", ("X1",) if refine_rev else ())
    if refine_rev:
        stage(8, "fr" if aug else "rr", () if aug else ("W1",))
        stage(9, "fr" if aug else "rr")
    stage(10, "rk")
    out += ["ar", "gU"]
    return " ".join(out)


def parse_plan(plan):
    """[(stage, modes, [gathers after it])] + the tail ops, in order: the form a host stand-in
    executes (tests/shard_standin.py)."""
    steps = []
    for tok in plan.split():
        if tok.startswith("s"):
            k, modes = tok[1:].split(":")
            steps.append(("stage", int(k), modes))
        elif tok.startswith("g"):
            steps.append(("gather", tok[1:]))
        elif tok == "ar":
            steps.append(("allreduce",))
        else:
            raise ValueError(f"bad plan token {tok!r}")
    return steps


def plan_collectives(plan):
    """Collectives per step of a plan (all-gathers + all-reduces)."""
    return sum(1 for s in parse_plan(plan) if s[0] in ("gather", "allreduce"))
