"""GPU parity: libgpk (HIP, gfx950) vs the CPU oracle on identical seeded inputs.

Tolerances (SURVEY.md §8(c) parity contract):
  K, D blocks             <= 1e-13 relative (max-abs / max)
  loss, full gradient     <= max(1e-10, 50 cond(K) eps, 4 x oracle-vs-extended-precision error)
  predictions             <= 1e-10 relative
  short Adam trajectories <= 1e-9 relative
"""
import numpy as np
import pytest

from oracle import gp_oracle as O
from tests.helpers import device_solver, problem_1d, problem_2d, rel

pytestmark = pytest.mark.gpu

KINDS = ["SE_Cos_1d", "Matern52_Cos_1d", "SE_1d", "Matern52_1d"]


@pytest.fixture(autouse=True)
def _numpy_oracle():
    O.set_backend(False)  # pin against the pure-NumPy statement
    yield
    O.set_backend(True)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("deriv", [0, 1, 2])
def test_kernel_matrices(kind, deriv):
    from gpk.core import kernel_matrices
    rng = np.random.default_rng(3)
    x1 = np.sort(rng.uniform(0, 3, 37))
    x2 = np.sort(rng.uniform(0, 3, 29))
    x2[4] = x1[7]  # a zero distance off the diagonal exercises abs'(0) = +1
    kp = {"log-w": rng.normal(size=5) - 1, "log-ls": rng.normal(size=5), "freq": rng.uniform(0, 5, 5)}
    K, D = kernel_matrices(kind, x1, x2, kp, 0.0, deriv)
    assert rel(K, O.kernel_block(kind, x1, x2, kp, 0)) < 1e-13
    if deriv:
        assert rel(D, O.kernel_block(kind, x1, x2, kp, deriv)) < 1e-13


def test_kernel_matrix_square_jitter():
    from gpk.core import kernel_matrices
    x = np.linspace(0, 1, 50) * 2 * np.pi
    Q = 30
    kp = {"log-w": np.log(1 / Q) * np.ones(Q), "log-ls": np.zeros(Q), "freq": np.linspace(0, 1, Q) * 20}
    K, D = kernel_matrices("Matern52_Cos_1d", x, x, kp, 1e-6, 2)
    assert rel(K, O.kernel_matrix("Matern52_Cos_1d", x, kp, 1e-6)) < 1e-13
    assert rel(D, O.kernel_block("Matern52_Cos_1d", x, x, kp, 2)) < 1e-13
    # jax abs'(0)=+1 convention: diagonal of DD is k''(0) = sum w(-5a^2/3 - omega^2)
    w, om = np.exp(kp["log-w"]), 2 * np.pi * kp["freq"]
    assert np.allclose(np.diag(D), np.sum(w * (-5.0 / 3.0 - om ** 2)), rtol=1e-13)


def cond_tol(prob, params, floor=1e-10, factor=50.0):
    """max(floor, factor * cond(K) * eps): GPU and LU/autograd references agree to this order;
    the explicit-inverse path and LU differ by O(cond * eps) (tools/diag_parity.py)."""
    if "x" in prob:
        c = np.linalg.cond(O.kernel_matrix(prob["kind"], prob["x"], params["kernel_paras"], prob["jitter"]))
    else:
        c = max(np.linalg.cond(O.kernel_matrix(prob["kind"], prob["x1"], params["kernel_paras_1"], prob["jitter"])),
                np.linalg.cond(O.kernel_matrix(prob["kind"], prob["x2"], params["kernel_paras_2"], prob["jitter"])))
    return max(floor, factor * c * np.finfo(np.float64).eps)


def oracle_err(prob, params):
    """Distance of the fp64 LU oracle (the reference's algorithm) from the same formulas
    evaluated with extended-precision (80-bit) solves: its own rounding error, per key."""
    fn = O.loss_grad_1d if "x" in prob else O.loss_grad_2d
    lo, go = fn(prob, params)
    O.set_extended(True)
    try:
        lt, gt = fn(prob, params)
    finally:
        O.set_extended(False)
    errs = {k: rel(O.flatten_params(go[k]), O.flatten_params(gt[k])) for k in go}
    errs["loss"] = abs(lo - lt) / abs(lt)
    return lo, go, errs


def _cmp_lossgrad(prob, params, Q, fs, tol=None, flags=0, extended=True, path=None):
    """GPU vs oracle within max(cond_tol, 4 x the oracle's own distance from exact arithmetic):
    at cond(K) ~ 1e5..1e7 the reference algorithm itself is only good to ~1e-9 (kernel-parameter
    gradients through the explicit K^{-1} of slogdet's backward rule)."""
    tol = cond_tol(prob, params) if tol is None else tol
    s = device_solver(prob, Q, fs, flags=flags)
    if path is not None:
        assert s.inverse_path() == path
    s.set_params(params)
    loss, g = s.loss_grad()
    if extended:
        lo, go, errs = oracle_err(prob, params)
    else:  # large N: the 80-bit yardstick takes minutes; the cond(K) budget alone
        fn = O.loss_grad_1d if "x" in prob else O.loss_grad_2d
        lo, go = fn(prob, params)
        errs = {k: 0.0 for k in list(go) + ["loss"]}
    gflat = O.flatten_params(go)
    assert abs(loss - lo) / abs(lo) < max(tol, 4 * errs["loss"]), (loss, lo)
    gd = O.unflatten_params(params, g)
    for key in sorted(go):
        a, b = O.flatten_params(gd[key]), O.flatten_params(go[key])
        assert rel(a, b) < max(tol, 4 * errs[key]), (key, rel(a, b), errs[key])
    assert rel(g, gflat) < max(tol, 4 * max(errs.values()))
    s.close()


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("eq", ["poisson", "allencahn"])
def test_loss_grad_1d(kind, eq):
    prob, params, _ = problem_1d(eq=eq, kind=kind, n=40, Q=5, seed=1)
    _cmp_lossgrad(prob, params, 5, 20.0)


def test_loss_grad_1d_large():
    prob, params, _ = problem_1d(n=200, Q=30, seed=2)  # C1 size, pads 200 -> 224
    _cmp_lossgrad(prob, params, 30, 20.0)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("eq", ["poisson", "allencahn", "advection"])
def test_loss_grad_2d(kind, eq):
    prob, params, _, fs = problem_2d(eq=eq, kind=kind, n1=40, n2=36, Q=5, seed=4)
    _cmp_lossgrad(prob, params, 5, fs)


def test_loss_grad_2d_c3_shape():
    prob, params, _, fs = problem_2d(eq="poisson", kind="SE_Cos_1d", n1=128, n2=128, Q=30, seed=5)
    _cmp_lossgrad(prob, params, 30, fs)


@pytest.mark.parametrize("dim", [1, 2])
def test_adam_trajectory(dim):
    if dim == 1:
        prob, params, _ = problem_1d(n=64, Q=8, seed=6)
        fs = 20.0
    else:
        prob, params, _, fs = problem_2d(n1=48, n2=40, Q=8, seed=6)
    s = device_solver(prob, params_q(params), fs)
    s.set_params(params)
    losses = s.step(5)
    opt = O.Adam(0.01)
    st = opt.init(params)
    p = params
    ref_losses = []
    for _ in range(5):
        lo, g = (O.loss_grad_1d if dim == 1 else O.loss_grad_2d)(prob, p)
        ref_losses.append(lo)
        p, st = opt.update(g, st, p)
    assert rel(losses, ref_losses) < 1e-9
    assert rel(s.get_flat(), O.flatten_params(p)) < 1e-9
    cnt, mu, nu = s.get_opt_state()
    assert cnt == 5
    assert rel(mu, O.flatten_params(st["mu"])) < 1e-8
    s.close()


def params_q(params):
    kp = params.get("kernel_paras", params.get("kernel_paras_1"))
    return len(kp["freq"])


@pytest.mark.parametrize("dim", [1, 2])
def test_predict_and_criterion(dim):
    if dim == 1:
        prob, params, (Xte, Yte) = problem_1d(n=64, Q=8, seed=7)
        s = device_solver(prob, 8)
        s.set_params(params)
        pred = s.predict(Xte)
        ref = O.preds_1d(prob, params, Xte)
        crit_ref = O.criterion_1d(prob, params)
    else:
        prob, params, (Xte, ute), fs = problem_2d(n1=48, n2=40, Q=8, seed=7)
        s = device_solver(prob, 8, fs)
        s.set_params(params)
        pred = s.predict(Xte[0], Xte[1])
        ref = O.preds_2d(prob, params, Xte[0], Xte[1])
        crit_ref = O.criterion_2d(prob, params)
    assert rel(pred, ref) < 1e-10
    assert abs(s.criterion() - crit_ref) / abs(crit_ref) < 1e-10
    s.close()


def test_step_deterministic():
    prob, params, _, fs = problem_2d(n1=64, n2=64, Q=10, seed=8)
    out = []
    for _ in range(2):
        s = device_solver(prob, 10, fs)
        s.set_params(params)
        s.step(3)
        out.append(s.get_flat())
        s.close()
    assert np.array_equal(out[0], out[1])


@pytest.mark.parametrize("variant", ["big", "huge"])
@pytest.mark.parametrize("eq,kind,n1,n2", [("poisson", "Matern52_Cos_1d", 96, 80),
                                          ("advection", "SE_Cos_1d", 72, 150),
                                          ("allencahn", "Matern52_1d", 40, 36),
                                          ("advection", "Matern52_Cos_1d", 136, 200)])
def test_loss_grad_2d_big_gemm_path(eq, kind, n1, n2, variant):
    """The 64x64 (big) and 128x128 (huge) throughput GEMMs (used from ~1500^2 / ~2048^2 up,
    e.g. C5's 4096^2), forced at small sizes: every stage, all transpose signatures (one
    launch per signature for huge), dual products (folded by alpha2/alpha for huge), fused
    epilogues, and tiles partly outside the 32-padded matrices (clamped loads)."""
    from gpk._lib import GPK_FLAG_FORCE_BIG_GEMM, GPK_FLAG_FORCE_HUGE_GEMM
    flags = GPK_FLAG_FORCE_BIG_GEMM if variant == "big" else GPK_FLAG_FORCE_HUGE_GEMM
    prob, params, _, fs = problem_2d(eq=eq, kind=kind, n1=n1, n2=n2, Q=5, seed=7)
    _cmp_lossgrad(prob, params, 5, fs, flags=flags)


def test_big_gemm_adam_and_predict_match_small():
    """Same trajectory and predictions with the big and the small GEMM kernels."""
    from gpk._lib import GPK_FLAG_FORCE_BIG_GEMM, GPK_FLAG_FORCE_HUGE_GEMM
    prob, params, (Xte, _), fs = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=72, n2=56, Q=6, seed=2)
    out = []
    for flags in (0, GPK_FLAG_FORCE_BIG_GEMM, GPK_FLAG_FORCE_HUGE_GEMM):
        s = device_solver(prob, 6, fs, flags=flags)
        s.set_params(params)
        losses = s.step(10)
        out.append((losses, s.get_flat(), s.predict(Xte[0], Xte[1])))
        s.close()
    for o in out[1:]:
        assert rel(out[0][0], o[0]) < 1e-11
        assert rel(out[0][1], o[1]) < 1e-9
        assert rel(out[0][2], o[2]) < 1e-10


@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("dim,eq,kind,n1,n2", [(1, "poisson", "Matern52_Cos_1d", 200, 0),
                                               (1, "allencahn", "SE_1d", 40, 0),
                                               (1, "poisson", "SE_Cos_1d", 330, 0),
                                               (2, "poisson", "Matern52_Cos_1d", 96, 80),
                                               (2, "advection", "SE_Cos_1d", 72, 150),
                                               (2, "allencahn", "Matern52_1d", 130, 64),
                                               (2, "poisson", "Matern52_Cos_1d", 300, 600)])
def test_loss_grad_big_spd_path(dim, eq, kind, n1, n2, wide):
    """The panel/update SPD inverse (spdinv_big.hip, used from p >= 1600: C2, C5), 64-wide and
    128-wide sweeps, forced at small sizes: one-sweep factors (p=64, 96), ragged last pivots
    of 32/64/96 (p=96, 160, 224, 352), the 128-pivot with a 32- or 64-wide second half, a last
    sweep narrower than 64, in-launch pivot hand-off (1 or 3 tiles) over several sweeps, the
    final mirror and the refinement gate.  300 x 600 (128-wide: T2 = 3 and 5) gives the two
    factors schedules of different lengths in one update launch: each factor keeps its own
    two-sweep table and the launch's item slots cover the longer list (the shorter
    stride used to null the second factor's schedule and starve its one-sweep tile list)."""
    from gpk._lib import GPK_FLAG_FORCE_BIG_SPD, GPK_FLAG_FORCE_WIDE_SPD, GPK_FLAG_FORCE_NARROW_SPD
    flags = GPK_FLAG_FORCE_BIG_SPD | (GPK_FLAG_FORCE_WIDE_SPD if wide else GPK_FLAG_FORCE_NARROW_SPD)
    if dim == 1:
        prob, params, _ = problem_1d(eq=eq, kind=kind, n=n1, Q=6, seed=3)
        _cmp_lossgrad(prob, params, 6, 20.0, flags=flags, path="big_wide" if wide else "big")
    else:
        prob, params, _, fs = problem_2d(eq=eq, kind=kind, n1=n1, n2=n2, Q=5, seed=8)
        _cmp_lossgrad(prob, params, 5, fs, flags=flags, path="big_wide" if wide else "big")


@pytest.mark.parametrize("wide", [False, True])
def test_big_spd_long_tile_runs(wide):
    """The update launch with 3 tile workgroups per factor: every workgroup walks a run of
    tiles across block rows (panel blocks staged per unit and reused along a row at 64-wide,
    the next unit prefetched under the current one's MFMAs, hand-off tiles at the start of
    three runs, the last sweep's mirror stage reusing the panel LDS)."""
    from gpk._lib import GPK_FLAG_FORCE_BIG_SPD, GPK_FLAG_FORCE_WIDE_SPD, GPK_FLAG_FORCE_NARROW_SPD
    from gpk.core import set_spd_big_workgroups
    flags = GPK_FLAG_FORCE_BIG_SPD | (GPK_FLAG_FORCE_WIDE_SPD if wide else GPK_FLAG_FORCE_NARROW_SPD)
    set_spd_big_workgroups(3)
    try:
        prob, params, _ = problem_1d(eq="poisson", kind="Matern52_Cos_1d", n=330, Q=6, seed=4)
        _cmp_lossgrad(prob, params, 6, 20.0, flags=flags)
        prob, params, _, fs = problem_2d(eq="advection", kind="SE_Cos_1d", n1=200, n2=150, Q=5, seed=9)
        _cmp_lossgrad(prob, params, 5, fs, flags=flags)
    finally:
        set_spd_big_workgroups(0)


def test_big_spd_adam_and_predict_match_small():
    """Same Adam trajectory and predictions with the large- (64- and 128-wide sweeps) and the
    small-factor SPD inverses."""
    from gpk._lib import (GPK_FLAG_FORCE_BIG_SPD, GPK_FLAG_FORCE_SMALL_SPD, GPK_FLAG_FORCE_WIDE_SPD,
                          GPK_FLAG_FORCE_NARROW_SPD)
    prob, params, (Xte, _), fs = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=200, n2=136, Q=6, seed=2)
    out = []
    for flags in (GPK_FLAG_FORCE_SMALL_SPD, GPK_FLAG_FORCE_BIG_SPD | GPK_FLAG_FORCE_NARROW_SPD,
                  GPK_FLAG_FORCE_BIG_SPD | GPK_FLAG_FORCE_WIDE_SPD):
        s = device_solver(prob, 6, fs, flags=flags)
        s.set_params(params)
        losses = s.step(10)
        out.append((losses, s.get_flat(), s.predict(Xte[0], Xte[1])))
        s.close()
    for o in out[1:]:
        assert rel(out[0][0], o[0]) < 1e-10
        assert rel(out[0][1], o[1]) < 1e-8
        assert rel(out[0][2], o[2]) < 1e-9


def test_loss_grad_1d_c2_size():
    """C2's shape (1D, N = 2048, Matern52_Cos_1d, Q = 30): the large-factor inverse at its
    natural size, against the LU oracle within the cond(K)-scaled budget."""
    prob, params, _ = problem_1d(n=2048, Q=30, seed=6)
    _cmp_lossgrad(prob, params, 30, 20.0, extended=False)


def _extra_model(eq, kind, n, Q, nepoch=40, change_point=0.5, n_test=50):
    from gpk.kernel_matrix import kernel_class
    from gpk.model_GP_solver_1d_extra import GP_solver_1d_extra
    name = {"poisson": "poisson_1d-mix_sin", "allencahn": "allencahn_1d-single_sin"}[eq]
    prob, Xte, Yte = O.setup_1d(name, n, 1.0 if eq == "poisson" else 2 * np.pi, kind, m_test=n_test)
    tp = {"equation": name, "kernel": kernel_class(kind), "kernel_extra": kernel_class("Matern52_1d"),
          "Q": Q, "lr": 0.01, "llk_weight": 200.0, "freq_scale": 30.0, "logdet": True, "nepoch": nepoch,
          "change_point": change_point, "tol": -1.0, "num_u_trick": 1, "other_paras": ""}
    m = GP_solver_1d_extra(prob["xind"], prob["y"], prob["x"].reshape(-1, 1), prob["src"], 1e-6, Xte, Yte, tp)
    return m, prob, (Xte, Yte)


@pytest.mark.parametrize("eq", ["poisson", "allencahn"])
def test_extra_gp_loss_grad(eq):
    """Extra-GP second phase on the device (shifted data + Allen-Cahn offset) vs the oracle's
    literal loss_extra (model_GP_solver_1d_extra.py:101-137), first GP frozen at random params."""
    from tests.helpers import extra_params
    m, prob, _ = _extra_model(eq, "Matern52_Cos_1d", 48, 5)
    _, params, _ = problem_1d(eq=eq, kind="Matern52_Cos_1d", n=48, Q=5, seed=11)
    prob_t = dict(prob, eq=eq)
    try:
        m._make_extra(params)
        pe = extra_params(np.random.default_rng(12), 48)
        loss, g = m.value_and_grad_extra(pe)
        lo, go = O.loss_grad_1d_extra(prob_t, params, pe, "Matern52_1d")
        c = max(np.linalg.cond(O.kernel_matrix("Matern52_Cos_1d", prob["x"], params["kernel_paras"], prob["jitter"])),
                np.linalg.cond(O.kernel_matrix("Matern52_1d", prob["x"], O._extra_kp(pe["kernel_paras"]), prob["jitter"])))
        tol = max(1e-9, 100 * c * np.finfo(float).eps)
        assert abs(loss - lo) / abs(lo) < tol, (loss, lo)
        for k in ("log_tau", "log_v"):
            assert abs(g[k] - go[k]) <= tol * max(1.0, abs(go[k])), k
        assert rel(g["u"], go["u"]) < tol
        assert rel(g["kernel_paras"]["log-w"], go["kernel_paras"]["log-w"]) < tol
        assert rel(g["kernel_paras"]["log-ls"], go["kernel_paras"]["log-ls"]) < tol
        # criterion of both GPs together (compute_early_stopping_extra, :180-193)
        assert abs(m.compute_early_stopping_extra(pe) - O.criterion_1d_extra(prob_t, params, pe, "Matern52_1d")) \
            < tol * O.criterion_1d_extra(prob_t, params, pe, "Matern52_1d")
    finally:
        m.close()


def test_extra_gp_two_phase_train_matches_replay():
    """GP_solver_1d_extra.train (two phases, records incl. the change-point preds_extra quirk)
    vs the oracle's replay of model_GP_solver_1d_extra.py:195-339, 40 epochs, N=64."""
    m, prob, test = _extra_model("poisson", "Matern52_Cos_1d", 64, 6, nepoch=40)
    try:
        log, es, min_err = m.train(40, verbose=False)
        _, pe, rec = O.train_replay_extra(prob, "Matern52_1d", 6, 30.0, 0.01, 40, 0.5, test)
        assert log["epoch_list"] == rec["epoch_list"]
        assert rel(log["loss_list"], rec["loss_list"]) < 1e-8
        assert rel(log["err_list"], rec["err_list"]) < 1e-6
        assert abs(min_err - rec["min_err"]) < 1e-6 * rec["min_err"]
        assert rel(O.flatten_params(m.params_extra), O.flatten_params(pe)) < 1e-6
    finally:
        m.close()
