"""The CPU oracle against the reference's own artefacts and an independent transcription.

Pinning:
  * end to end: replaying the reference's committed 100-epoch runs from their logged
    configuration reproduces the logged min rel-L2 error (tests/golden/ref_runs.json, read from
    code/result_log/*/log.txt:3) — 1D to the 8 printed digits, 2D (chaotic) to 1e-4;
  * per step: the closed-form adjoints equal torch autograd through a transcription of
    code/kernel_matrix.py + the reference loss (tests/autograd_ref.py);
  * the committed fixtures (tests/golden/*.npz) guard the oracle against regressions.
"""
import json
import os

import numpy as np
import pytest

from oracle import gp_oracle as O
from tests import autograd_ref as AR
from tests.helpers import problem_1d, problem_2d, rel

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KINDS = ["SE_Cos_1d", "Matern52_Cos_1d", "SE_1d", "Matern52_1d"]


@pytest.fixture(params=[False, True], ids=["numpy", "c"])
def backend(request):
    O.set_backend(request.param)
    yield request.param
    O.set_backend(True)


def test_kernel_blocks_vs_fixture(backend):
    z = np.load(os.path.join(GOLD, "kd.npz"))
    kp = {"log-w": z["logw"], "log-ls": z["logls"], "freq": z["freq"]}
    for kind in KINDS:
        assert rel(O.kernel_block(kind, z["x1"], z["x2"], kp, 0), z[f"K_{kind}"]) < 1e-14
        for deriv in (1, 2):
            assert rel(O.kernel_block(kind, z["x1"], z["x2"], kp, deriv), z[f"D{deriv}_{kind}"]) < 1e-13
    Q = 30
    kp0 = {"log-w": np.log(1 / Q) * np.ones(Q), "log-ls": np.zeros(Q), "freq": np.linspace(0, 1, Q) * 20}
    K, D = O.kernel_kd("Matern52_Cos_1d", z["xsq"], kp0, 1e-6, 2)
    assert rel(K, z["Ksq"]) < 1e-14 and rel(D, z["Dsq"]) < 1e-13
    if backend:  # the C helper evaluates one triangle and mirrors it
        assert np.array_equal(K, K.T) and np.array_equal(D, D.T)


@pytest.mark.parametrize("kind", KINDS)
def test_kernel_blocks_vs_autograd(kind):
    """Closed-form K, dK/dx1, d2K/dx1^2 vs nested autograd of kappa (code/kernel_matrix.py:49-57),
    including the JAX abs'(0)=+1 convention on the diagonal."""
    import torch
    x = np.linspace(0, 1, 17) * 2 * np.pi
    rng = np.random.default_rng(0)
    kp = {"log-w": rng.normal(size=4) - 1, "log-ls": rng.normal(size=4) * 0.3, "freq": rng.uniform(0, 3, 4)}
    for deriv in (1, 2):
        Ka, Da = AR.mats(kind, torch.tensor(x), {k: torch.tensor(v) for k, v in kp.items()}, 0.0, deriv)
        assert rel(O.kernel_block(kind, x, x, kp, 0), Ka.detach().numpy()) < 1e-14
        assert rel(O.kernel_block(kind, x, x, kp, deriv), Da.detach().numpy()) < 1e-12


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("eq", ["poisson", "allencahn"])
def test_loss_grad_1d_vs_autograd(kind, eq):
    prob, params, _ = problem_1d(eq=eq, kind=kind, n=30, Q=4, seed=2)
    lo, go = O.loss_grad_1d(prob, params)
    la, ga = AR.loss_grad_1d(prob, params)
    cond = np.linalg.cond(O.kernel_matrix(kind, prob["x"], params["kernel_paras"], prob["jitter"]))
    tol = max(1e-11, 100 * cond * np.finfo(float).eps)
    assert abs(lo - la) / abs(la) < tol
    assert rel(O.flatten_params(go), O.flatten_params(ga)) < tol


@pytest.mark.parametrize("kind_extra", ["Matern52_1d", "SE_1d"])
@pytest.mark.parametrize("eq", ["poisson", "allencahn"])
def test_loss_grad_1d_extra_vs_autograd(kind_extra, eq):
    """The extra GP's loss (model_GP_solver_1d_extra.py:101-137): closed-form oracle vs the
    literal torch transcription, first GP frozen at random params."""
    from tests.helpers import extra_params
    prob, params, _ = problem_1d(eq=eq, kind="Matern52_Cos_1d", n=30, Q=4, seed=3)
    pe = extra_params(np.random.default_rng(5), 30)
    lo, go = O.loss_grad_1d_extra(prob, params, pe, kind_extra)
    la, ga = AR.loss_grad_1d_extra(prob, params, pe, kind_extra)
    cond = max(np.linalg.cond(O.kernel_matrix("Matern52_Cos_1d", prob["x"], params["kernel_paras"], prob["jitter"])),
               np.linalg.cond(O.kernel_matrix(kind_extra, prob["x"], O._extra_kp(pe["kernel_paras"]), prob["jitter"])))
    tol = max(1e-11, 100 * cond * np.finfo(float).eps)
    assert abs(lo - la) / abs(la) < tol
    assert rel(O.flatten_params(go), O.flatten_params(ga)) < tol


def test_extra_loss_is_shifted_1d_loss():
    """The identity the device path relies on: loss_extra == the single-GP 1D loss of the extra
    GP on (y - u[Xind], f - u_xx) for Poisson (gpk/model_GP_solver_1d_extra.py docstring)."""
    from tests.helpers import extra_params
    prob, params, _ = problem_1d(eq="poisson", kind="SE_Cos_1d", n=26, Q=3, seed=4)
    pe = extra_params(np.random.default_rng(6), 26)
    lo, go = O.loss_grad_1d_extra(prob, params, pe, "Matern52_1d")
    u, uxx = O.frozen_fields_1d(prob, params)
    shifted = dict(prob, kind="Matern52_1d", y=prob["y"] - u[prob["xind"]], src=prob["src"] - uxx)
    ps = dict(pe, kernel_paras=O._extra_kp(pe["kernel_paras"]))
    ls, gs = O.loss_grad_1d(shifted, ps)
    assert abs(lo - ls) / abs(lo) < 1e-12
    for k in ("log_tau", "log_v"):
        assert abs(go[k] - gs[k]) <= 1e-9 * max(1.0, abs(go[k]))
    assert rel(go["u"], gs["u"]) < 1e-10
    assert rel(go["kernel_paras"]["log-w"], gs["kernel_paras"]["log-w"]) < 1e-10


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("eq", ["poisson", "allencahn", "advection"])
def test_loss_grad_2d_vs_autograd(kind, eq):
    prob, params, _, _ = problem_2d(eq=eq, kind=kind, n1=14, n2=11, Q=3, seed=5)
    lo, go = O.loss_grad_2d(prob, params)
    la, ga = AR.loss_grad_2d(prob, params)
    conds = [np.linalg.cond(O.kernel_matrix(kind, prob[x], params[k], prob["jitter"]))
             for x, k in (("x1", "kernel_paras_1"), ("x2", "kernel_paras_2"))]
    tol = max(1e-11, 100 * max(conds) * np.finfo(float).eps)
    assert abs(lo - la) / abs(la) < tol
    for key in go:
        assert rel(O.flatten_params(go[key]), O.flatten_params(ga[key])) < tol, key


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("eq", ["poisson", "allencahn"])
def test_loss_grad_3d_vs_dense_kronecker_autograd(kind, eq):
    """The 3-axis oracle (mode products, unfoldings, log-det weights, six boundary faces) vs
    torch autograd of the same log joint written with dense Kronecker matrices."""
    from tests.helpers import problem_3d
    prob, params, _ = problem_3d(eq=eq, kind=kind, ns=(6, 5, 4), Q=3, seed=11)
    lo, go = O.loss_grad_3d(prob, params)
    la, ga = AR.loss_grad_3d(prob, params)
    conds = [np.linalg.cond(O.kernel_matrix(kind, prob[f"x{a}"], params[f"kernel_paras_{a}"], prob["jitter"]))
             for a in (1, 2, 3)]
    tol = max(1e-11, 100 * float(np.prod(conds)) * np.finfo(float).eps)
    assert abs(lo - la) / abs(la) < tol, (lo, la)
    for key in go:
        assert rel(O.flatten_params(go[key]), O.flatten_params(ga[key])) < tol, key


def test_loss_grad_3d_two_axis_reduction():
    """With a single point on axis 3 the 3-axis prior is the 2-axis one times the scalar factor
    k3 = K3[0,0]: logdet(K1 (x) K2 (x) k3) = logdet(K1 (x) K2) + N1 N2 log k3 and
    <U, S> = <U, S_2d> / k3 -- so the 3-axis loss equals the 2-axis loss of U / sqrt(k3)-free
    form below (the residual of a 1-point axis has D3 = k''(0) / k3 times U)."""
    from tests.helpers import problem_2d
    prob2, params2, _, _ = problem_2d(eq="poisson", kind="SE_Cos_1d", n1=9, n2=7, Q=3, seed=4)
    x3 = np.array([0.0])
    kp3 = {"freq": np.array([0.0, 1.0, 2.0]), "log-ls": np.zeros(3), "log-w": np.log(np.ones(3) / 3)}
    K3, D3 = O.kernel_kd(prob2["kind"], x3, kp3, prob2["jitter"], 2)
    k3, d3 = float(K3[0, 0]), float(D3[0, 0])
    U = params2["U"]
    prob3 = dict(prob2, x3=x3, src=prob2["src"][:, :, None] + d3 / k3 * U[:, :, None],
                 bvals=O.boundary_3d(np.repeat(U[:, :, None], 1, axis=2)))
    params3 = dict(params2, U=U[:, :, None], kernel_paras_3=kp3)
    l3, g3 = O.loss_grad_3d(prob3, params3, want_grad=True)
    # the 2-axis log joint with the same R (the d3/k3 U term cancels against the shifted source),
    # prior weights N3 = 1, an extra N1 N2 log k3 / 2 and <U,S> scaled by 1/k3; boundary faces:
    # U[0], U[-1], U[:,0], U[:,-1] as in 2D plus U[:,:,0] and U[:,:,-1] = U (zero gap here)
    prob2b = dict(prob2, bvals=O.boundary_2d(U))
    N1, N2 = U.shape
    l2, _ = O.loss_grad_2d(prob2b, params2, want_grad=False)
    lds, quad = _parts_2d(prob2b, params2)
    c = prob2["logdet"]
    expect = l2 + 0.5 * c * N1 * N2 * np.log(k3) + 0.5 * quad * (1.0 / k3 - 1.0)
    # boundary: 2D counts N_b = 2N1 + 2N2 faces entries, 3D adds 2 N1 N2 (all zero gap)
    expect -= prob2["llk_weight"] * 0.5 * (2 * N1 * N2) * params2["log_tau"]
    assert abs(l3 - expect) / abs(expect) < 1e-10, (l3, expect)


def _parts_2d(prob, params):
    K1 = O.kernel_matrix(prob["kind"], prob["x1"], params["kernel_paras_1"], prob["jitter"])
    K2 = O.kernel_matrix(prob["kind"], prob["x2"], params["kernel_paras_2"], prob["jitter"])
    U = params["U"]
    S = np.linalg.solve(K1, U) @ np.linalg.inv(K2)
    return (np.linalg.slogdet(K1)[1], np.linalg.slogdet(K2)[1]), float(np.sum(U * S))


def test_loss_grad_vs_fixture():
    z = np.load(os.path.join(GOLD, "lossgrad.npz"))
    cases = {
        "1d_poisson": lambda: problem_1d(eq="poisson", kind="Matern52_Cos_1d", n=40, Q=5, seed=1),
        "1d_allencahn": lambda: problem_1d(eq="allencahn", kind="SE_Cos_1d", n=40, Q=5, seed=1),
        "1d_matern52": lambda: problem_1d(eq="poisson", kind="Matern52_1d", n=40, Q=5, seed=1),
        "2d_poisson": lambda: problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=24, n2=20, Q=5, seed=0),
        "2d_allencahn": lambda: problem_2d(eq="allencahn", kind="SE_Cos_1d", n1=24, n2=20, Q=5, seed=0),
        "2d_advection": lambda: problem_2d(eq="advection", kind="Matern52_Cos_1d", n1=24, n2=20, Q=5, seed=0),
    }
    O.set_backend(False)
    try:
        for name, mk in cases.items():
            prob, params = mk()[:2]
            assert np.array_equal(O.flatten_params(params), z[f"{name}/params"])
            fn = O.loss_grad_1d if "x" in prob else O.loss_grad_2d
            lo, go = fn(prob, params)
            assert abs(lo - z[f"{name}/loss_lu"]) <= 1e-13 * abs(lo), name
            assert rel(O.flatten_params(go), z[f"{name}/grad_lu"]) < 1e-12, name
            # the fp64 LU statement stays within its rounding budget of the extended value
            assert rel(O.flatten_params(go), z[f"{name}/grad_ext"]) < 1e-8, name
    finally:
        O.set_backend(True)


def test_extended_mode_agrees_when_well_conditioned():
    prob, params, _, _ = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=12, n2=10, Q=3, seed=1)
    lo, go = O.loss_grad_2d(prob, params)
    O.set_extended(True)
    try:
        lt, gt = O.loss_grad_2d(prob, params)
    finally:
        O.set_extended(False)
    assert abs(lo - lt) / abs(lt) < 1e-13
    assert rel(O.flatten_params(go), O.flatten_params(gt)) < 1e-12


def test_extended_c_kernel_equals_numpy_loops():
    """oracle/ext_solve.c (blocked, OpenMP) is the same long-double LU as the NumPy loops: same
    pivots and factors, solves within long-double rounding (blocking reorders the sums)."""
    if O._extlib() is None:
        pytest.skip("oracle/_build/libgpk_ext.so not built")
    rng = np.random.default_rng(3)
    n = 150                                     # > 2 blocks of 64, ragged last block
    M = rng.normal(size=(n, n))
    K = M @ M.T / n + 1e-3 * np.eye(n)
    B = rng.normal(size=(n, 5))
    fp, fc = O._ext_lu_py(K), O._ext_lu(K)
    assert np.array_equal(np.asarray(fp[1]), np.asarray(fc[1]))
    assert float(np.max(np.abs(fp[0] - fc[0]))) <= 1e-17 * float(np.max(np.abs(fp[0])))
    xp, xc = O._ext_solve_py(fp, B), O._ext_solve(fc, B)
    assert rel(xc, xp) < 1e-15
    assert O._slogdet_from_lu(("ext", fc)) == pytest.approx(O._slogdet_from_lu(("ext", fp)), rel=1e-15)


@pytest.mark.parametrize("cid", ["C1", "C3"])
def test_extended_fixture_reproduces(cid):
    """tests/golden/ext_<cfg>.npz (tools/solve_accuracy.py --fixture) is what the yardstick
    gives here: recompute it for the small configs (C1 200-point 1D, C3 128^2)."""
    import tools.solve_accuracy as SA
    from tests.helpers import config_problem
    fx = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"ext_{cid}.npz"))
    prob, params, _, _ = config_problem(cid)
    le, ge = SA.run_mode(prob, params, "ext")
    ll, gl = SA.run_mode(prob, params, "lu")
    assert abs(le - float(fx["loss_ext"])) <= 1e-14 * abs(le)
    for k, v in ge.items():
        assert rel(v, fx[f"ext/{k}"]) < 1e-13, k
        assert rel(gl[k], v) == pytest.approx(float(fx[f"lu_err/{k}"]), rel=0.5, abs=1e-15), k


def test_adam_matches_optax_formula():
    """optax 0.1.4 scale_by_adam + scale(-lr), eps_root=0, bias correction by count."""
    opt = O.Adam(0.01)
    p = {"a": np.array([1.0, -2.0]), "b": 0.5}
    st = opt.init(p)
    g = {"a": np.array([0.3, -0.1]), "b": 2.0}
    p1, st1 = opt.update(g, st, p)
    for k in ("a", "b"):
        gk = np.asarray(g[k])
        m = 0.1 * gk
        v = 0.001 * gk ** 2
        exp = np.asarray(p[k]) - 0.01 * (m / 0.1) / (np.sqrt(v / 0.001) + 1e-8)
        assert np.allclose(p1[k], exp, rtol=0, atol=1e-15)
    assert st1["count"] == 1


def test_flatten_order_is_jax_sorted_keys():
    from gpk.core import tree_flatten, params_template
    t = params_template(2, 3, 2, 2)
    t["U"] = np.arange(6.0).reshape(3, 2)
    t["kernel_paras_1"] = {"freq": np.array([10, 11.]), "log-ls": np.array([12, 13.]), "log-w": np.array([14, 15.])}
    t["kernel_paras_2"] = {"freq": np.array([20, 21.]), "log-ls": np.array([22, 23.]), "log-w": np.array([24, 25.])}
    t["log_tau"], t["log_v"] = 30.0, 31.0
    f = tree_flatten(t)
    assert np.array_equal(f, np.r_[np.arange(6.0), 10, 11, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 30, 31])
    assert np.array_equal(f, O.flatten_params(t))


def _ref_run(key):
    with open(os.path.join(GOLD, "ref_runs.json")) as f:
        return json.load(f)[key]


def test_replay_1d_reference_run():
    """code/result_log/poisson_1d-single_sin/kernel_Matern52_Cos_1d/epoch_100/Q30/log.txt:3."""
    r = _ref_run("poisson_1d-single_sin/Matern52_Cos_1d")
    c = r["config"]
    prob, Xte, Yte = O.setup_1d(c["equation"], c["N_col"], 2 * np.pi, c["kernel"], llk_weight=c["llk_weight"])
    params = O.init_params_1d(c["N_col"], c["Q"], c["freq_scale"])
    _, _, rec = O.train_replay(1, prob, params, c["lr"], c["nepoch"], (Xte, Yte))
    # the log prints 8 decimals
    assert abs(rec["min_err"] - r["min_err"][0]) < 1e-8, rec["min_err"]


@pytest.mark.slow
def test_replay_2d_reference_run():
    """code/result_log/poisson_2d-sin_sin/kernel_Matern52_Cos_1d/epoch_100/Q30/log.txt:3.
    400^2, 100 Adam steps: rounding differences grow chaotically, so 1e-4 rel."""
    r = _ref_run("poisson_2d-sin_sin/Matern52_Cos_1d")
    c = r["config"]
    prob, Xte, ute = O.setup_2d(c["equation"], c["N_col"], 2 * np.pi, c["kernel"], llk_weight=c["llk_weight"])
    params = O.init_params_2d(c["N_col"], c["N_col"], c["Q"], c["freq_scale"])
    _, _, rec = O.train_replay(2, prob, params, c["lr"], c["nepoch"], (Xte, ute))
    assert abs(rec["min_err"] - r["min_err"][0]) / r["min_err"][0] < 1e-4, rec["min_err"]
