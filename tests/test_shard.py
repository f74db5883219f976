"""Row-sharded 2D step (gpk_create_sharded / gpk_group_create).

GPU: an in-process group of nranks handles on one device runs the same sharded step as RCCL
ranks (only the collective transport differs); its loss / full gradient must match the CPU
oracle and the unsharded handle, and its Adam trajectory the unsharded one.  RCCL itself is
exercised with one rank (a one-GPU box cannot host two RCCL ranks).
CPU: the communicator-id exchange over a world-size-2 gloo group.
"""
import os
import socket

import numpy as np
import pytest

from oracle import gp_oracle as O
from tests.helpers import device_solver, problem_2d, rel

# A sharded handle whose inverse is the augmented chain (small factors whose grids fit the
# device) gets A, Bt and K^{-1} D^T from it like an unsharded handle; otherwise it solves them by
# GEMMs against K^{-1} -- an unsharded handle does that with GPK_FLAG_NO_CHAIN_AUG.  Compare
# like with like.
from gpk._lib import GPK_FLAG_NO_CHAIN_AUG as NO_AUG  # noqa: E402


def _alg(g):
    """The unsharded handle's flag that runs the sharded handle g's algorithm."""
    return 0 if g.inverse_path() == "chain_aug" else NO_AUG


def _group(prob, Q, fs, nranks, flags=0):
    from gpk.core import DeviceGroup
    return DeviceGroup(nranks, 2, prob["eq"], prob["kind"], prob["x1"], prob["src"], prob["bvals"],
                       x2=prob["x2"], Q=Q, jitter=prob["jitter"], llk_weight=prob["llk_weight"],
                       logdet=prob["logdet"], beta=prob.get("beta", 1.0), lr=0.01, freq_scale=fs,
                       flags=flags)


def _tol(prob, params):
    c = max(np.linalg.cond(O.kernel_matrix(prob["kind"], prob["x1"], params["kernel_paras_1"], prob["jitter"])),
            np.linalg.cond(O.kernel_matrix(prob["kind"], prob["x2"], params["kernel_paras_2"], prob["jitter"])))
    return max(1e-10, 50 * c * np.finfo(float).eps)


@pytest.mark.gpu
@pytest.mark.parametrize("nranks", [1, 2, 3, 4])
@pytest.mark.parametrize("eq,kind,n1,n2", [("poisson", "Matern52_Cos_1d", 72, 56),
                                          ("allencahn", "SE_Cos_1d", 40, 66),
                                          ("advection", "Matern52_1d", 50, 90)])
def test_group_loss_grad(eq, kind, n1, n2, nranks):
    """Loss and full gradient of the sharded step vs the oracle and vs one unsharded handle
    (unequal axes, ragged last row blocks, padding to 32 * nranks)."""
    prob, params, _, fs = problem_2d(eq=eq, kind=kind, n1=n1, n2=n2, Q=5, seed=21)
    g = _group(prob, 5, fs, nranks)
    s = device_solver(prob, 5, fs, flags=_alg(g))  # the sharded step's own algorithm
    try:
        g.set_params(params)
        s.set_params(params)
        lg, gg = g.loss_grad()
        ls, gs = s.loss_grad()
        lo, go = O.loss_grad_2d(prob, params)
        tol = _tol(prob, params)
        assert abs(lg - lo) / abs(lo) < tol, (lg, lo)
        assert rel(gg, O.flatten_params(go)) < tol
        assert abs(lg - ls) / abs(ls) < 1e-11
        assert rel(gg, gs) < 1e-9
    finally:
        g.close()
        s.close()


@pytest.mark.gpu
def test_group_eight_ranks_c4_size():
    """Eight ranks (the MI355X node's GPU count) on the headline 256^2 problem (C4: Matern52_Cos,
    Q = 30, seeded like the bench): loss and full gradient vs the oracle and vs one handle, then
    5 Adam steps vs one handle."""
    from tests.test_gpu_fullsize import _config_problem
    prob, params, _, cfg = _config_problem("C4")
    fs = cfg["freq_scale"]
    g = _group(prob, 30, fs, 8)
    s = device_solver(prob, 30, fs, flags=_alg(g))
    try:
        assert g.shard_info()[1] == 8
        g.set_params(params)
        s.set_params(params)
        lg, gg = g.loss_grad()
        ls, gs = s.loss_grad()
        lo, go = O.loss_grad_2d(prob, params)
        tol = _tol(prob, params)
        assert abs(lg - lo) / abs(lo) < tol, (lg, lo)
        gd = O.unflatten_params(params, gg)
        for k in go:
            assert rel(O.flatten_params(gd[k]), O.flatten_params(go[k])) < tol, k
        assert abs(lg - ls) / abs(ls) < 1e-11
        assert rel(gg, gs) < 1e-9
        assert rel(g.step(5), s.step(5)) < 1e-10
        assert rel(g.get_flat(), s.get_flat()) < 1e-9
    finally:
        g.close()
        s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cid", ["C3", "C4"])
def test_group_chain_path_two_ranks(cid):
    """The exact per-rank path of an 8-GPU RCCL run (one process per GPU: the persistent chain
    inverse + row-sharded GEMM descriptors + collectives), on one device: a 2-rank in-process
    group whose two chain grids are co-resident takes the chain (gpk_inverse_path), and its loss /
    full gradient match the oracle and its 10-step Adam trajectory the unsharded handle, at the
    BASELINE configs C3 (128^2 SE_Cos) and C4 (256^2, the headline)."""
    from tests.test_gpu_fullsize import _config_problem
    prob, params, _, cfg = _config_problem(cid)
    fs = cfg["freq_scale"]
    g = _group(prob, 30, fs, 2)
    s = device_solver(prob, 30, fs, flags=_alg(g))
    try:
        # (C3: both ranks' augmented chains fit the device together; C4: the plain chain)
        assert g.inverse_path() == ("chain_aug" if cid == "C3" else "chain"), g.inverse_path()
        assert g.shard_info()[1] == 2
        g.set_params(params)
        s.set_params(params)
        lg, gg = g.loss_grad()
        ls, gs = s.loss_grad()
        lo, go = O.loss_grad_2d(prob, params)
        tol = _tol(prob, params)
        assert abs(lg - lo) / abs(lo) < tol, (lg, lo)
        gd = O.unflatten_params(params, gg)
        for k in go:
            assert rel(O.flatten_params(gd[k]), O.flatten_params(go[k])) < tol, k
        assert abs(lg - ls) / abs(ls) < 1e-11
        assert rel(gg, gs) < 1e-9
        assert rel(g.step(10), s.step(10)) < 1e-10
        assert rel(g.get_flat(), s.get_flat()) < 1e-9
    finally:
        g.close()
        s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nranks,flags", [(2, 0), (4, 0), (2, 8)])
def test_group_trajectory_matches_unsharded(nranks, flags):
    """10 Adam steps of the sharded group == 10 steps of one handle (params, losses); flags 8
    forces the 128x128 GEMM where the row blocks allow it (downgraded per stage otherwise)."""
    prob, params, (Xte, _), fs = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=200, n2=136, Q=6, seed=3)
    g = _group(prob, 6, fs, nranks, flags=flags)
    s = device_solver(prob, 6, fs, flags=_alg(g))
    try:
        g.set_params(params)
        s.set_params(params)
        lg = g.step(10)
        ls = s.step(10)
        assert rel(lg, ls) < 1e-11
        assert rel(g.get_flat(), s.get_flat()) < 1e-9
        assert rel(g.predict(Xte[0], Xte[1]), s.predict(Xte[0], Xte[1])) < 1e-9
    finally:
        g.close()
        s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nranks,big", [(2, False), (3, False), (4, True), (5, True)])
def test_group_split_factors_matches_unsharded(nranks, big):
    """GPK_FLAG_SPLIT_FACTORS: ranks [0, n/2) invert K1 only, [n/2, n) K2 only, and the inverses,
    log-det blocks and refinement gates are broadcast from ranks 0 and n/2.  Loss, gradient and
    a 5-step Adam trajectory vs one unsharded handle, with the per-sweep and the large-factor
    (forced, 64- and 128-wide) inverses; odd rank counts give unequal groups."""
    from gpk._lib import (GPK_FLAG_SPLIT_FACTORS, GPK_FLAG_FORCE_BIG_SPD, GPK_FLAG_FORCE_WIDE_SPD,
                          GPK_FLAG_NO_CHAIN)
    prob, params, _, fs = problem_2d(eq="advection", kind="Matern52_Cos_1d", n1=150, n2=96, Q=5, seed=22)
    extra = (GPK_FLAG_FORCE_BIG_SPD | (GPK_FLAG_FORCE_WIDE_SPD if nranks == 5 else 0)) if big else 0
    g = _group(prob, 5, fs, nranks, flags=GPK_FLAG_SPLIT_FACTORS | extra)
    s = device_solver(prob, 5, fs, flags=NO_AUG | GPK_FLAG_NO_CHAIN | extra)
    try:
        g.set_params(params)
        s.set_params(params)
        lg, gg = g.loss_grad()
        ls, gs = s.loss_grad()
        assert abs(lg - ls) / abs(ls) < 1e-11, (lg, ls)
        assert rel(gg, gs) < 1e-9
        lo, go = O.loss_grad_2d(prob, params)
        assert rel(gg, O.flatten_params(go)) < _tol(prob, params)
        # the row-sliced and K-split products sum in another order than one handle's; cond(K)
        # lifts those rounding differences over the trajectory (1.6e-10 observed at 5 steps)
        assert rel(g.step(5), s.step(5)) < 1e-9
        assert rel(g.get_flat(), s.get_flat()) < 1e-8
    finally:
        g.close()
        s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nranks,axis", [(2, 2), (4, 1), (3, 2)])
def test_group_split_factors_non_pd_is_group_wide(nranks, axis):
    """A factor that is not positive definite is seen on device only by the ranks that invert it;
    the step sums the status bits over the group, so EVERY rank reports it (group_run checks each
    rank's status and calls a disagreement an internal error): under RCCL a rank that carried on
    would enter the next collectives alone and hang.  The handles stay usable afterwards."""
    from gpk._lib import GPK_FLAG_SPLIT_FACTORS, GPKError, GPK_ENOTPD
    prob, params, _, fs = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=72, n2=64, Q=4, seed=8)
    g = _group(prob, 4, fs, nranks, flags=GPK_FLAG_SPLIT_FACTORS)
    try:
        bad = {k: (dict(v) if isinstance(v, dict) else v) for k, v in params.items()}
        kp = dict(bad[f"kernel_paras_{axis}"])
        kp["log-w"] = np.array(kp["log-w"], dtype=float)
        kp["log-w"][0] = np.nan                      # K_axis all NaN: no positive pivot
        bad[f"kernel_paras_{axis}"] = kp
        g.set_params(bad)
        with pytest.raises(GPKError) as ei:
            g.loss_grad()
        assert ei.value.code == GPK_ENOTPD, str(ei.value)
        assert "differs across the ranks" not in str(ei.value)
        g.set_params(params)                          # recovered: the next call is clean
        lg, gg = g.loss_grad()
        lo, go = O.loss_grad_2d(prob, params)
        assert abs(lg - lo) / abs(lo) < _tol(prob, params)
    finally:
        g.close()


@pytest.mark.gpu
def test_group_eight_ranks_c5_split_factors():
    """Eight ranks on the full C5 problem (advection 4096^2, Matern52_Cos, Q = 30) with one
    Kronecker factor per rank half (GPK_FLAG_SPLIT_FACTORS, the 128-wide large-factor inverse):
    loss and full gradient vs one unsharded handle."""
    from gpk._lib import GPK_FLAG_SPLIT_FACTORS
    from gpk.problems import make_solver
    from tests.test_gpu_fullsize import _config_problem, _cond_bound
    prob, params, _, cfg = _config_problem("C5")
    s = make_solver("C5", seed=0)
    try:
        assert s.inverse_path() == "big_wide"
        s.set_params(params)
        ls, gs = s.loss_grad()
    finally:
        s.close()
    g = _group(prob, 30, cfg["freq_scale"], 8, flags=GPK_FLAG_SPLIT_FACTORS)
    try:
        g.set_params(params)
        lg, gg = g.loss_grad()
    finally:
        g.close()
    # row-sliced products (other tile variants, other summation order) against one handle,
    # both without refinement: the cond(K) budget of the full-size oracle test applies
    tol = max(1e-10, 50 * _cond_bound(prob, params) * np.finfo(float).eps)
    assert abs(lg - ls) / abs(ls) < tol, (lg, ls)
    assert rel(gg, gs) < tol, (rel(gg, gs), tol)


@pytest.mark.gpu
def test_rccl_single_rank_sharded_handle():
    """gpk_create_sharded with a one-rank RCCL communicator: the captured step with RCCL
    all-gathers / all-reduces in its graph equals the unsharded step."""
    from gpk.core import DeviceSolver, comm_unique_id
    prob, params, _, fs = problem_2d(eq="poisson", kind="SE_Cos_1d", n1=64, n2=48, Q=4, seed=5)
    kw = dict(x2=prob["x2"], Q=4, jitter=prob["jitter"], llk_weight=prob["llk_weight"],
              logdet=prob["logdet"], lr=0.01, freq_scale=fs)
    r = DeviceSolver(2, prob["eq"], prob["kind"], prob["x1"], prob["src"], prob["bvals"],
                     shard=(0, 1, comm_unique_id()), **kw)
    s = device_solver(prob, 4, fs, flags=0 if r.inverse_path() == "chain_aug" else NO_AUG)
    try:
        assert r.inverse_path() == "chain_aug"  # (a one-rank RCCL handle: the augmented chain)
        assert r.shard_info() == (0, 1, 0, 64)
        r.set_params(params)
        s.set_params(params)
        lr_, gr = r.loss_grad()
        ls, gs = s.loss_grad()
        assert abs(lr_ - ls) / abs(ls) < 1e-12
        assert rel(gr, gs) < 1e-10
        # the sharded step reduces the gradient partials in another order (reduce_parts +
        # all-reduce vs the fused two-level tail): rounding-level gradient differences, which
        # Adam's m/sqrt(v) can lift to ~1e-11 in the losses over 5 steps
        assert rel(r.step(5), s.step(5)) < 1e-10
        assert rel(r.get_flat(), s.get_flat()) < 1e-10
    finally:
        r.close()
        s.close()


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from gpk import replicas, shard
    ctx = replicas.init("gloo")
    cid = shard.broadcast_comm_id(ctx, make_id=lambda: bytes((7 * i + 3) % 256 for i in range(128)))
    q.put((rank, cid))
    replicas.shutdown(ctx)


def test_comm_id_broadcast_gloo_world2():
    """Every rank of a 2-process gloo group receives rank 0's 128-byte communicator id."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = bytes((7 * i + 3) % 256 for i in range(128))
    assert got[0] == expect and got[1] == expect


# ---- the sharded step's plan across processes (CPU, gloo world 2) --------------------------
def _sharded_section_worker(rank, world, port, q, eq, aug, fwd2=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import types
    import bench
    from gpk import replicas
    from tests.shard_standin import HostShardedSolver, HostSolver
    ctx = replicas.init("gloo")
    try:
        prob, params, _, _ = problem_2d(eq=eq, kind="Matern52_Cos_1d", n1=40, n2=36, Q=4, seed=11)
        made = {}

        def make_sharded(cid, flags):
            made["s"] = HostShardedSolver(prob, params, ctx.world, ctx.rank, aug=aug, refine_fwd2=fwd2)
            return made["s"]

        a = types.SimpleNamespace(sharded_steps=3)
        out = bench.sharded_section(a, ctx, configs=("C4",), make_sharded=make_sharded,
                                    make_single=lambda cid: HostSolver(prob, params, aug=aug, refine_fwd2=fwd2))
        s = made["s"]
        q.put((rank, s.params, s.losses, s.plan, s.collectives_per_step, out["C4"]))
    finally:
        replicas.shutdown(ctx)


@pytest.mark.parametrize("eq,aug,fwd2", [("poisson", True, True), ("allencahn", True, True),
                                         ("advection", True, True), ("poisson", False, True),
                                         ("advection", False, False)])
def test_sharded_section_gloo_world2_plan(eq, aug, fwd2):
    """bench.py's sharded_section over two gloo processes, driving the host stand-in of the
    sharded step (tests/shard_standin.py): each rank computes only its rows of every product the
    plan of gpk/shard.py marks 'r' (row partition shard_rows: 40 rows -> 32 + 8), receives the
    rest only through the plan's all-gathers (rows it neither computed nor received are NaN),
    and sums its contraction / loss partials in the plan's one all-reduce.  After the section's
    2 + 3 Adam steps both ranks hold the unsharded oracle trajectory's params; the augmented-chain
    plan (the small-factor / C4 form) issues 3 collectives per step, the large-factor form 9 (7
    with the large advection factors' forward refinement of A alone, the C5 form)."""
    import multiprocessing as mp
    from gpk.shard import plan_collectives, shard_plan
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sharded_section_worker, args=(r, 2, port, q, eq, aug, fwd2)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict((r[0], r[1:]) for r in (q.get(timeout=300) for _ in ps))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    prob, params, _, _ = problem_2d(eq=eq, kind="Matern52_Cos_1d", n1=40, n2=36, Q=4, seed=11)
    # (explicit inverses against the oracle's LU solves: the cond(K) budget of the parity tests)
    tol = max(1e-9, _tol(prob, params))
    opt = O.Adam(0.01)
    st = opt.init(params)
    ref_losses = []
    for _ in range(5):
        lo, go = O.loss_grad_2d(prob, params)
        ref_losses.append(lo)
        params, st = opt.update(go, st, params)
    plan = shard_plan(aug, refine_fwd2=fwd2)
    for r in (0, 1):
        p_r, losses, plan_r, ncoll, entry = got[r]
        assert plan_r == plan
        assert ncoll == plan_collectives(plan) == (3 if aug else 9)
        assert np.isfinite(losses).all()
        assert rel(np.asarray(losses), np.asarray(ref_losses)) < tol
        assert rel(O.flatten_params(p_r), O.flatten_params(params)) < tol
        assert entry["ranks"] == 2 and entry["steps"] == 3 and entry["speedup_vs_1gpu"] > 0
    assert np.array_equal(O.flatten_params(got[0][0]), O.flatten_params(got[1][0]))


def test_shard_plan_missing_gather_poisons():
    """The stand-in detects a plan that lacks an all-gather a later product needs: without the
    R gather the reverse pass reads rows this rank never computed (NaN) and the gradient is
    poisoned -- the check the gloo test relies on."""
    from tests.shard_standin import HostShardedSolver

    class Local:  # two ranks' exchange emulated in one process is not needed: rank 0 of 2, no peers
        count = 0

        def gather_rows(self, M, h):
            self.count += 1
            return M

        def allreduce(self, v):
            self.count += 1
            return v

    prob, params, _, _ = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=40, n2=36, Q=4, seed=11)
    s = HostShardedSolver(prob, params, 2, 0, aug=True, exchange=Local())
    s.steps = [op for op in s.steps if op != ("gather", "R")]
    _, grad = s._loss_grad()
    assert not np.isfinite(O.flatten_params(grad)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("eq,flags_name,aug", [("poisson", None, True), ("poisson", "GPK_FLAG_NO_CHAIN_AUG", False),
                                               ("poisson", "GPK_FLAG_FORCE_BIG_SPD", False),
                                               ("advection", "GPK_FLAG_FORCE_BIG_SPD", False)])
def test_library_shard_plan_matches_gpk_shard(eq, flags_name, aug):
    """The library's sharded step (gpk_shard_plan of every rank of an in-process group) is the
    plan gpk/shard.py restates and the gloo stand-in test executes."""
    from gpk import _lib
    from gpk.shard import shard_plan
    flags = getattr(_lib, flags_name) if flags_name else 0
    prob, params, _, fs = problem_2d(eq=eq, kind="Matern52_Cos_1d", n1=72, n2=64, Q=4, seed=8)
    g = _group(prob, 4, fs, 2, flags=flags)
    try:
        assert (g.inverse_path() == "chain_aug") == aug, g.inverse_path()
        big = flags_name == "GPK_FLAG_FORCE_BIG_SPD"
        # (large factors: no reverse refinement; advection's beta = 200 >= 16: A's forward
        # refinement alone)
        fwd2 = not (big and eq == "advection")
        for k in range(2):
            assert g.shard_plan(k) == shard_plan(aug, True, not big, fwd2), g.shard_plan(k)
    finally:
        g.close()
