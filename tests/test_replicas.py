"""Multi-process (world_size 2, gloo on CPU) coverage of the replica path (gpk/replicas.py):
fold ownership, the MAX-over-ranks timing reduction used by bench.py, and the ordered gather of
per-fold results used by model_GP_solver_{1d,2d}.test()."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from gpk import replicas
    ctx = replicas.init("gloo")
    try:
        folds = replicas.owned(5, ctx)
        res = {i: (0.1 * i, 100 + i) for i in folds}
        allres = replicas.gather_by_index(res, 5, ctx)
        replicas.barrier(ctx)
        mx = replicas.max_over_ranks(1.5 + rank, ctx)
        sm = replicas.sum_over_ranks(rank + 1, ctx)
        out.put((rank, folds, allres, mx, sm))
    finally:
        replicas.shutdown(ctx)


def test_replicas_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got.sort()
    owned = [g[1] for g in got]
    assert owned == [[0, 2, 4], [1, 3]]                     # disjoint, covering, round-robin
    for _, _, allres, mx, sm in got:
        assert allres == [(0.1 * i, 100 + i) for i in range(5)]   # fold order restored
        assert mx == 2.5 and sm == 3.0


def test_single_process_context_needs_no_group(monkeypatch):
    from gpk import replicas
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    ctx = replicas.init()
    assert (ctx.world, ctx.rank) == (1, 0)
    assert replicas.owned(3, ctx) == [0, 1, 2]
    assert replicas.max_over_ranks(2.0, ctx) == 2.0
    assert replicas.gather_by_index({0: "a", 1: "b"}, 2, ctx) == ["a", "b"]
