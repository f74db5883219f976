"""The macro-tile persistent chain inverse (chain_multi_kernel, spdinv.hip): the default inverse of
large 1D factors (C2: 1D Poisson, N = 2048), replacing jnp.linalg.solve / slogdet of
code/model_GP_solver_1d.py:92,135-137.

  * forced at small sizes (GPK_FLAG_FORCE_CHAIN_MULTI): one macro row (T = 2), odd tile counts
    (the last macro row holds one tile row), plain + merged workgroups over many sweeps -- loss and
    full gradient vs the oracle, and BITWISE equal to the one-tile-per-workgroup chain (same
    operations per tile; the upper triangle written as the transpose of the lower);
  * C2 at full size on the default path: loss and every gradient element vs the fp64 LU oracle
    within the cond(K) budget, a 5-step Adam trajectory vs the oracle's optax restatement, and
    agreement with the 64-wide launch-per-sweep inverse (GPK_FLAG_FORCE_BIG_SPD);
  * a capped co-residency budget falls back to the launch-per-sweep path.
"""
import numpy as np
import pytest

from oracle import gp_oracle as O
from tests.helpers import device_solver, problem_1d, record_parity, rel
from tests.test_gpu_parity import _cmp_lossgrad, cond_tol

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("eq,kind,n", [("poisson", "Matern52_Cos_1d", 40),
                                       ("poisson", "Matern52_Cos_1d", 200),
                                       ("allencahn", "SE_1d", 97),
                                       ("poisson", "SE_Cos_1d", 330),
                                       ("poisson", "Matern52_1d", 520)])
def test_forced_multi_chain_vs_oracle(eq, kind, n):
    from gpk._lib import GPK_FLAG_FORCE_CHAIN_MULTI
    prob, params, _ = problem_1d(eq=eq, kind=kind, n=n, Q=6, seed=4)
    _cmp_lossgrad(prob, params, 6, 20.0, flags=GPK_FLAG_FORCE_CHAIN_MULTI, path="chain_multi",
                  extended=n <= 200)


@pytest.mark.parametrize("n", [40, 200, 330])
def test_forced_multi_chain_bitwise_equals_chain(n):
    """Same loss, gradient, 3-step trajectory and predictions as the one-tile-per-workgroup chain
    (the class sums read K^{-1} from both triangles, the log-det every pivot)."""
    from gpk._lib import GPK_FLAG_FORCE_CHAIN_MULTI
    prob, params, (Xte, _) = problem_1d(eq="poisson", kind="Matern52_Cos_1d", n=n, Q=6, seed=5)
    out = []
    for flags, path in ((0, "chain"), (GPK_FLAG_FORCE_CHAIN_MULTI, "chain_multi")):
        s = device_solver(prob, 6, 20.0, flags=flags)
        assert s.inverse_path() == path
        s.set_params(params)
        loss, g = s.loss_grad()
        losses = s.step(3)
        out.append((loss, g, losses, s.get_flat(), s.predict(Xte)))
        s.close()
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(np.asarray(a), np.asarray(b))


def _c2_problem(seed=0):
    """The oracle problem + params of C2, seeded as gpk.problems.make_solver seeds u."""
    from gpk.problems import CONFIGS
    cfg = CONFIGS["C2"]
    n = cfg["n"]
    prob, _, _ = O.setup_1d(cfg["equation"], n, cfg["scale"], cfg["kernel"], llk_weight=cfg["llk_weight"])
    params = O.init_params_1d(n, 30, cfg["freq_scale"])
    params["u"] = 0.1 * np.random.default_rng(seed).normal(size=n).reshape(n, 1)
    return prob, params


def test_c2_full_size_default_path_vs_oracle():
    from gpk.problems import make_solver
    O.set_backend(True)
    prob, params = _c2_problem()
    s = make_solver("C2", seed=0)
    try:
        assert s.inverse_path() == "chain_multi"
        assert np.array_equal(s.get_flat(), O.flatten_params(params))
        loss, g = s.loss_grad()
        losses = s.step(5)
        flat5 = s.get_flat()
    finally:
        s.close()
    lo, go = O.loss_grad_1d(prob, params)
    tol = cond_tol(prob, params)
    assert abs(loss - lo) / abs(lo) < tol, (loss, lo, tol)
    gd = O.unflatten_params(params, g)
    for key in sorted(go):
        r = rel(O.flatten_params(gd[key]), O.flatten_params(go[key]))
        assert r < tol, (key, r, tol)
    # 5 Adam steps (model_GP_solver_1d.py:151-158) vs the oracle's optax restatement, fp64 (the
    # reference's arithmetic) and on the exact-field long-double yardstick: Adam's m / sqrt(v)
    # carries a gradient component's RELATIVE error into the step, so at cond(K) ~ 1e8 the small
    # components' rounding reaches the params; the device's params after 5 steps stay within
    # max(tol, 4 x the fp64 trajectory's distance) of the yardstick's
    traj = []
    for ext in (False, True):
        opt = O.Adam(0.01)
        st = opt.init(params)
        p = params
        O.set_extended(ext)
        try:
            for i in range(5):
                li, gi = O.loss_grad_1d(prob, p)
                assert abs(losses[i] - li) / abs(li) < tol, (i, losses[i], li, ext)
                p, st = opt.update(gi, st, p)
        finally:
            O.set_extended(False)
        traj.append(O.flatten_params(p))
    lu_dist = rel(traj[0], traj[1])
    dev_dist = rel(flat5, traj[1])
    record_parity("test_c2_full_size_default_path_vs_oracle", "C2@5", {"params": dev_dist},
                  {"params": max(1e-9, tol, 4 * lu_dist)}, {"lu_oracle_err": {"params": lu_dist}})
    assert dev_dist < max(1e-9, tol, 4 * lu_dist), (dev_dist, lu_dist, tol)


def test_c2_multi_chain_matches_launch_per_sweep_path():
    from gpk._lib import GPK_FLAG_FORCE_BIG_SPD
    from gpk.problems import make_solver
    prob, params = _c2_problem()
    res = []
    for flags, path in ((0, "chain_multi"), (GPK_FLAG_FORCE_BIG_SPD, "big")):
        s = make_solver("C2", seed=0, flags=flags)
        assert s.inverse_path() == path
        res.append(s.loss_grad())
        s.close()
    tol = cond_tol(prob, params)
    assert abs(res[0][0] - res[1][0]) / abs(res[1][0]) < tol
    assert rel(res[0][1], res[1][1]) < tol


def test_c2_class_gemv_bitwise_equals_matrix_gemv():
    """The GEMVs read Kc and D as class ids + class values (the inverse launch writes neither
    matrix); GPK_FLAG_MATRIX_GEMV keeps the round-2 form.  Bitwise the same loss, gradient,
    3-step trajectory, predictions and u_xx field."""
    from gpk._lib import GPK_FLAG_MATRIX_GEMV
    from gpk.problems import make_solver
    xte = np.linspace(0.0, 1.0, 300)
    out = []
    for flags in (0, GPK_FLAG_MATRIX_GEMV):
        s = make_solver("C2", seed=0, flags=flags)
        try:
            assert s.inverse_path() == "chain_multi"
            loss, g = s.loss_grad()
            losses = s.step(3)
            out.append((loss, g, losses, s.get_flat(), s.predict(xte), s.forward_field("u_xx"), s.forward_field("K")))
        finally:
            s.close()
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(np.asarray(a), np.asarray(b))


def test_capped_capacity_falls_back_to_launch_per_sweep():
    from gpk.core import set_chain_capacity
    from gpk.problems import make_solver
    set_chain_capacity(400)  # < the 498 workgroups C2's macro-tile grid needs
    try:
        s = make_solver("C2", seed=0)
        assert s.inverse_path() == "big"
        s.close()
    finally:
        set_chain_capacity(0)
