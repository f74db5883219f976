"""GPU parity at the BASELINE.json sizes the bench and DESIGN.md quote, on the paths they time.

  * C5 (advection-multiscale, 4096 x 4096 space-time grid, Matern52_Cos_1d, Q = 30; the
    large-factor SPD path and the 128 x 128 MFMA GEMMs): loss and the FULL gradient (every
    element of dL/dU, every kernel-parameter gradient) at the seeded bench params vs the fp64
    LU oracle (code/model_GP_solver_advection.py:87-179);
  * C4 (2D Poisson 256^2, the headline): element-wise loss + gradient on the default
    (augmented-chain, fast-graph) path, and an 11-step Adam trajectory whose last 8 steps run
    the fast multi-step graph the bench times (code/model_GP_solver_2d.py:87-183);
  * the chain inverse's co-residency guard: a capped capacity falls back to the per-sweep
    launches, bitwise equal to GPK_FLAG_NO_CHAIN, and matches the oracle.

Tolerance at C5: max(1e-10, 50 cond(K) eps), cond(K) bounded by ||K||_inf / jitter (the
kernel part is PSD, so lambda_min >= jitter): an SVD of two 4096^2 factors would cost minutes.
The 80-bit yardstick is out of reach at 4096, so the LU oracle is the reference value.
"""
import os

import numpy as np
import pytest

from oracle import gp_oracle as O
from tests.helpers import device_solver, problem_2d, rel

pytestmark = pytest.mark.gpu
EPS = np.finfo(np.float64).eps


def _config_problem(cid, seed=0, m_test=8):
    """The oracle's problem + params for a BASELINE config, seeded exactly as
    gpk.problems.make_solver seeds U (the bench's inputs)."""
    from gpk.problems import CONFIGS
    cfg = CONFIGS[cid]
    n = cfg["n"]
    prob, Xte, ute = O.setup_2d(cfg["equation"], n, cfg["scale"], cfg["kernel"],
                                llk_weight=cfg["llk_weight"], beta=cfg.get("beta"), m_test=m_test)
    params = O.init_params_2d(n, n, 30, cfg["freq_scale"])
    params["U"] = 0.1 * np.random.default_rng(seed).normal(size=n * n).reshape(n, n)
    return prob, params, (Xte, ute), cfg


def _cond_bound(prob, params):
    c = 0.0
    for ax in (1, 2):
        K = O.kernel_matrix(prob["kind"], prob[f"x{ax}"], params[f"kernel_paras_{ax}"], prob["jitter"])
        c = max(c, float(np.max(np.sum(np.abs(K), axis=1))) / prob["jitter"])
    return c


def test_c5_full_size_loss_grad_vs_oracle():
    from gpk.problems import make_solver
    O.set_backend(True)  # OpenMP C fields: the 4096^2 x Q=30 field evaluations in seconds
    prob, params, _, _ = _config_problem("C5")
    s = make_solver("C5", seed=0)
    try:
        assert s.inverse_path() == "big_wide"
        assert np.array_equal(s.get_flat(), O.flatten_params(params))  # same inputs as the oracle
        loss, g = s.loss_grad()
    finally:
        s.close()
    lo, go = O.loss_grad_2d(prob, params)
    cond = _cond_bound(prob, params)
    tol = max(1e-10, 50 * cond * EPS)
    gd = O.unflatten_params(params, g)
    errs = {k: rel(O.flatten_params(gd[k]), O.flatten_params(go[k])) for k in go}
    print(f"C5 cond<= {cond:.3e} tol {tol:.2e} loss {abs(loss - lo) / abs(lo):.2e} "
          + " ".join(f"{k} {v:.2e}" for k, v in sorted(errs.items())))
    assert abs(loss - lo) / abs(lo) < tol, (loss, lo)
    for k, e in errs.items():
        assert e < tol, (k, e, tol)
    assert np.all(np.isfinite(g))


def test_c4_default_path_elementwise_and_fast_graph_trajectory():
    from gpk.problems import make_solver
    from tests.test_gpu_parity import cond_tol, oracle_err
    prob, params, _, _ = _config_problem("C4")
    s = make_solver("C4", seed=0)
    try:
        assert s.inverse_path() == "chain_aug"
        loss, g = s.loss_grad()
        lo, go, errs = oracle_err(prob, params)  # + its own distance from 80-bit solves
        tol = cond_tol(prob, params)
        assert abs(loss - lo) / abs(lo) < max(tol, 4 * errs["loss"])
        gd = O.unflatten_params(params, g)
        for k in go:
            e = rel(O.flatten_params(gd[k]), O.flatten_params(go[k]))
            assert e < max(tol, 4 * errs[k]), (k, e, errs[k])
        # 3 steps (full graph until the gate has been seen), then 8 on the fast 8-step graph
        la = s.step(3)
        fast, rb0 = s.graph_mode()
        assert fast, "C4's refinement gate is closed: the bench path runs the fast graph"
        lb = s.step(8)
        fast_end, rb1 = s.graph_mode()
        assert rb1 == rb0
        pf = s.get_flat()
    finally:
        s.close()
    opt = O.Adam(0.01)
    st = opt.init(params)
    p = params
    losses = []
    for _ in range(11):
        lo_i, g_i = O.loss_grad_2d(prob, p)
        losses.append(lo_i)
        p, st = opt.update(g_i, st, p)
    assert rel(np.concatenate([la, lb]), np.array(losses)) < 1e-9
    assert rel(pf, O.flatten_params(p)) < 1e-9


@pytest.fixture
def capped_chain():
    from gpk.core import set_chain_capacity
    set_chain_capacity(16)
    yield
    set_chain_capacity(0)


def test_default_capacity_keeps_the_chain():
    prob, params, _, fs = problem_2d(n1=256, n2=256, Q=30, seed=0)
    s = device_solver(prob, 30, fs)
    assert s.inverse_path() == "chain_aug"  # 386 workgroups fit 256 CUs x 2
    s.close()


@pytest.mark.parametrize("eq,n1,n2", [("poisson", 256, 256), ("advection", 72, 64)])
def test_capped_capacity_falls_back_to_sweeps(capped_chain, eq, n1, n2):
    """A co-resident budget below the chain's grid (a CU-partitioned device, or CUs held by other
    work) selects the per-sweep launches: bitwise the GPK_FLAG_NO_CHAIN handle, and the oracle's
    loss / gradient within the cond(K) budget."""
    from gpk._lib import GPK_FLAG_NO_CHAIN
    from tests.test_gpu_parity import _cmp_lossgrad
    prob, params, _, fs = problem_2d(eq=eq, n1=n1, n2=n2, Q=8, seed=2)
    a = device_solver(prob, 8, fs)
    b = device_solver(prob, 8, fs, flags=GPK_FLAG_NO_CHAIN)
    try:
        assert a.inverse_path() == "sweep" and b.inverse_path() == "sweep"
        for s in (a, b):
            s.set_params(params)
        la, ga = a.loss_grad()
        lb, gb = b.loss_grad()
        assert la == lb and np.array_equal(ga, gb)
        assert np.array_equal(a.step(9), b.step(9))
        assert np.array_equal(a.get_flat(), b.get_flat())
    finally:
        a.close()
        b.close()
    _cmp_lossgrad(prob, params, 8, fs, extended=(n1 < 200))


def test_rank_group_chain_only_when_co_resident():
    """In-process rank groups launch concurrently on one device from several host threads: their
    handles use the persistent chain only when every rank's chain grid fits the device together
    (nranks x grid <= the co-resident capacity), else the per-sweep inverse.  A one-process-per-GPU
    RCCL rank only needs its own grid to fit."""
    from gpk.core import set_chain_capacity
    from tests.test_shard import _group
    prob, params, _, fs = problem_2d(n1=64, n2=64, Q=4, seed=1)   # P = 96 at 3 ranks: 20 workgroups
    g = _group(prob, 4, fs, 3)
    try:
        assert g.inverse_path() in ("chain", "chain_aug")  # (round 6: sharded handles take the
    finally:                                               # augmented chain when it fits too)
        g.close()
    set_chain_capacity(50)                 # one grid fits, three do not
    try:
        g = _group(prob, 4, fs, 3)
        s = device_solver(prob, 4, fs)
        try:
            assert g.inverse_path() == "sweep"
            assert s.inverse_path() in ("chain", "chain_aug")
        finally:
            g.close()
            s.close()
    finally:
        set_chain_capacity(0)


@pytest.mark.parametrize("n1,n2", [(3072, 3072), (4096, 4096)])
def test_wide_inverse_quarter_tiles_bitwise_whole_tiles(n1, n2):
    """The 128-wide update works its last round of tiles as quarter tiles when that round would
    leave most workgroups idle (C5 size: 64 of 1056 tiles; 3072^2: 24 of 600); each output
    block sees the same MFMA sequence, so the loss, gradient and a 2-step trajectory are bitwise
    those of whole tiles (GPK_FLAG_NO_QUARTER_TILES)."""
    from gpk._lib import GPK_FLAG_NO_QUARTER_TILES
    from gpk.problems import make_solver
    out = []
    for flags in (0, GPK_FLAG_NO_QUARTER_TILES):
        if n1 == 4096:
            s = make_solver("C5", seed=0, flags=flags)
        else:
            prob, params, _, fs = problem_2d(eq="advection", n1=n1, n2=n2, Q=6, seed=3)
            s = device_solver(prob, 6, fs, flags=flags)
            s.set_params(params)
        try:
            assert s.inverse_path() == "big_wide"
            loss, g = s.loss_grad()
            losses = s.step(2)
            s.sync()
            out.append((loss, g, losses, s.get_flat()))
        finally:
            s.close()
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(np.asarray(a), np.asarray(b))


def test_tile128_and_64x64_stages_vs_yardstick():
    """The C5-class GEMM stages run on the pipelined 128x128 tile (gemm_tile_dev.h; dual
    products as two passes, gemm.hip launch_huge); GPK_FLAG_FORCE_BIG_GEMM runs every stage on
    the 64x64 kernel instead -- the same algorithm in another summation order.  Each order is
    checked on its own against the long-double, exact-field yardstick of this 3072^2 advection
    problem (tests/golden/ext_T3072.npz, tools/solve_accuracy.py T3072 --fixture): loss and
    every gradient key within 4x the fp64 LU oracle's own distance from it (floor 1e-10) -- the
    bar of the random-parameter size tests (tests/test_gpu_parity.py: 4x the oracle's own
    distance); the seeded BASELINE configs use 2x / 1.5x (tests/test_gpu_accuracy.py).  Round 5
    compared the two orders with each other, at a bar (5e-8) above the LU oracle's whole error.
    Measured (round 6, tools/t3072_diag.py; device / LU distance): U 0.49x, kernel_paras_2
    0.34-0.75x, loss 0.68x for both orders; kernel_paras_1 0.69x (tile64) to 1.50x (tile128),
    2.1x with the round-6 default refinement of the large advection factors (A's forward solve
    alone).  This problem's kernel_paras_1 gradient scatters with last-bit changes of G
    (GPK_FLAG_REFINE_ALL, i.e. MORE accurate S and X solves: 3.1x; the fp64 contraction 3.5x):
    the fp64 representation of K and D times cond(K) (~1e-16 x 1e8), amplified by the
    contraction's cancellation, which every fp64 evaluation -- the LU oracle's included --
    carries at its own rounding.  At the seeded C5 config the same keys are 0.14-0.32x
    (tests/test_gpu_accuracy.py)."""
    from gpk._lib import GPK_FLAG_FORCE_BIG_GEMM
    from tests.helpers import record_parity
    from tests.test_gpu_accuracy import fixture_errors
    O.set_backend(True)
    fx = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ext_T3072.npz"))
    prob, params, _, fs = problem_2d(eq="advection", n1=3072, n2=3072, Q=6, seed=3)
    tol = {"loss": max(1e-10, 4.0 * float(fx["loss_lu_err"]))}
    for f in fx.files:
        if f.startswith("lu_err/"):
            tol[f[7:]] = max(1e-10, 4.0 * float(fx[f]))
    for tag, flags in (("tile128", 0), ("tile64", GPK_FLAG_FORCE_BIG_GEMM)):
        s = device_solver(prob, 6, fs, flags=flags)
        s.set_params(params)
        try:
            assert s.inverse_path() == "big_wide"
            loss, g = s.loss_grad()
        finally:
            s.close()
        gd = O.unflatten_params(params, g)
        errs = fixture_errors(fx, loss, {k: O.flatten_params(gd[k]) for k in gd})
        record_parity("test_tile128_and_64x64_stages_vs_yardstick", f"T3072/{tag}", errs, tol, {})
        for k, e in errs.items():
            assert e < tol[k], (tag, k, e, tol[k])
