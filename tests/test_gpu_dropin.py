"""GPU: the drop-in kernel layer and the forward fields, called the way the reference calls them.

  * Kernel_1d.kappa / D_x1_kappa / DD_x1_kappa (code/kernel_matrix.py:45-57) -- vmapped over
    pairs in the reference (gpk_kernel_pairs here) -- and scalar calls;
  * Kernel_matrix.get_kernel_matrix (code/kernel_matrix.py:21-30) on flattened meshgrid pairs;
  * value_and_grad_kernel (code/model_GP_solver_2d.py:87-121, code/model_GP_solver_advection.py
    :87-121, code/model_GP_solver_1d.py:80-99) through the solver classes, i.e. every
    gpk_forward_field output: K1, K2, K1inv_U, K2inv_Ut, U_xx (U_x), U_yy (U_y) / K, Kinv_u, u_xx.

Tolerances: kernel values <= 1e-13 relative; solved fields within
50 cond(K) eps of the LU oracle (the K^{-1} application; tests/test_gpu_parity.py cond_tol).
"""
import numpy as np
import pytest

from oracle import gp_oracle as O
from tests.helpers import device_solver, problem_1d, problem_2d, rand_kp, rel
from tests.test_gpu_parity import cond_tol

pytestmark = pytest.mark.gpu

KINDS = ["SE_Cos_1d", "Matern52_Cos_1d", "SE_1d", "Matern52_1d"]


@pytest.mark.parametrize("kind", KINDS)
def test_kernel_class_methods_vs_oracle(kind):
    from gpk.kernel_matrix import kernel_class
    rng = np.random.default_rng(7)
    Q = 6
    kp = rand_kp(rng, Q, 5.0)
    k = kernel_class(kind)()
    x = rng.uniform(0, 2, 300)
    y = rng.uniform(0, 2, 300)
    y[:20] = x[:20]  # zero distances: JAX's abs'(0) = +1 in D_x1_kappa / DD_x1_kappa
    for deriv, fn in ((0, k.kappa), (1, k.D_x1_kappa), (2, k.DD_x1_kappa)):
        got = fn(x, y, kp)
        ref = np.diag(O.kernel_block(kind, x, y, kp, deriv))
        assert got.shape == x.shape
        assert rel(got, ref) < 1e-13, (deriv, rel(got, ref))
        # scalar call (the reference's kappa(x1, y1, paras) on two floats)
        s = fn(float(x[3]), float(y[3]), kp)
        assert isinstance(s, float) and abs(s - ref[3]) <= 1e-13 * max(1.0, np.max(np.abs(ref)))
    # 2D arrays of pairs keep their shape (vmap over a meshgrid)
    xm, ym = np.meshgrid(x[:7], y[:5], indexing="ij")
    got = k.DD_x1_kappa(xm, ym, kp)
    assert got.shape == (7, 5)
    assert rel(got, O.kernel_block(kind, x[:7], y[:5], kp, 2)) < 1e-13


def test_invalid_kernel_name():
    from gpk.kernel_matrix import kernel_class
    with pytest.raises(Exception, match="Invalid Kernel"):
        kernel_class("Matern32_1d")


@pytest.mark.parametrize("kind", KINDS)
def test_get_kernel_matrix_vs_oracle(kind):
    """Kernel_matrix(jitter, K_u).get_kernel_matrix(X1, X2, paras): vmap(kappa) over the N^2
    flattened meshgrid pairs + jitter I (code/kernel_matrix.py:21-30, called at
    code/model_GP_solver_2d.py:97-102 with meshgrid(x, x, indexing='ij'))."""
    from gpk.kernel_matrix import Kernel_matrix, kernel_class
    Q = 30
    n = 64
    x = np.linspace(0, 1, n) * 2 * np.pi
    kp = O.init_params_2d(n, n, Q, 20.0)["kernel_paras_1"]
    X1, X2 = np.meshgrid(x, x, indexing="ij")
    km = Kernel_matrix(1e-6, kernel_class(kind)())
    K = km.get_kernel_matrix(X1.reshape(-1), X2.reshape(-1), kp)
    assert K.shape == (n, n)
    assert rel(K, O.kernel_matrix(kind, x, kp, 1e-6)) < 1e-13


def _solver_class(eq):
    """A reference-shaped solver object (GP_solver_2d_single / _advection) on a small grid."""
    from gpk import model_GP_solver_2d as m2d
    from gpk import model_GP_solver_advection as madv
    from gpk.kernel_matrix import kernel_class
    prob, params, (Xte, ute), fs = problem_2d(eq=eq, kind="Matern52_Cos_1d", n1=48, n2=40, Q=6, seed=4)
    tp = {"kernel": kernel_class("Matern52_Cos_1d"), "llk_weight": prob["llk_weight"], "Q": 6,
          "lr": 0.01, "freq_scale": fs, "logdet": True,
          "equation": {"poisson": "poisson_2d-sin_sin", "advection": "advection-multiscale"}[eq]}
    cls = m2d.GP_solver_2d_single
    if eq == "advection":
        tp["beta"] = prob["beta"]
        cls = madv.GP_solver_2d_single_advection
    s = cls(prob["bvals"], (prob["x1"], prob["x2"]), prob["src"], prob["jitter"], Xte, ute, tp)
    return s, prob, params


@pytest.mark.parametrize("eq", ["poisson", "advection"])
def test_value_and_grad_kernel_2d_fields(eq):
    """All six outputs of value_and_grad_kernel (every gpk_forward_field field) vs the oracle's
    LU-based restatement of code/model_GP_solver_2d.py:97-121 at seeded params."""
    s, prob, params = _solver_class(eq)
    K1, K2, A, Bt_t, Uxx, Uyy = s.value_and_grad_kernel(params)
    deriv = 1 if eq == "advection" else 2
    kind, j = prob["kind"], prob["jitter"]
    K1o, D1 = O.kernel_kd(kind, prob["x1"], params["kernel_paras_1"], j, deriv)
    K2o, D2 = O.kernel_kd(kind, prob["x2"], params["kernel_paras_2"], j, deriv)
    U = params["U"]
    Ao = np.linalg.solve(K1o, U)          # K1inv_U   (:104)
    Bo = np.linalg.solve(K2o, U.T)        # K2inv_Ut  (:105)
    tol = cond_tol(prob, params)
    assert rel(K1, K1o) < 1e-13 and rel(K2, K2o) < 1e-13
    assert A.shape == U.shape and Bt_t.shape == U.T.shape
    assert rel(A, Ao) < tol, rel(A, Ao)
    assert rel(Bt_t, Bo) < tol, rel(Bt_t, Bo)
    assert rel(Uxx, D1 @ Ao) < tol          # U_xx / U_x   (:112)
    assert rel(Uyy, (D2 @ Bo).T) < tol      # U_yy / U_y   (:119)
    # boundary_and_eq_gap on those fields equals the device's criterion terms
    bg, eg = s.boundary_and_eq_gap(U, Uxx, Uyy)
    crit = s.compute_early_stopping(params)
    assert abs((bg / s.Nb + eg / s.Nc) - crit) / abs(crit) < 1e-8
    s.dev.close()


@pytest.mark.parametrize("eq", ["poisson", "allencahn"])
def test_forward_fields_1d(eq):
    """1D: K, K^{-1} u and u_xx = D K^{-1} u (code/model_GP_solver_1d.py:86-99)."""
    prob, params, _ = problem_1d(eq=eq, kind="SE_Cos_1d", n=90, Q=6, seed=5)
    s = device_solver(prob, 6, 20.0)
    s.set_params(params)
    K, D = O.kernel_kd(prob["kind"], prob["x"], params["kernel_paras"], prob["jitter"], 2)
    u = params["u"].reshape(-1)
    alpha = np.linalg.solve(K, u)
    tol = cond_tol(prob, params)
    assert rel(s.forward_field("K"), K) < 1e-13
    assert rel(s.forward_field("Kinv_u").reshape(-1), alpha) < tol
    assert rel(s.forward_field("u_xx").reshape(-1), D @ alpha) < tol
    s.close()


def test_forward_fields_c4_size():
    """The same six fields at the headline size (256^2, Q=30, the augmented-chain inverse that
    produces A and Bt inside its launch)."""
    prob, params, _, fs = problem_2d(n1=256, n2=256, Q=30, seed=0)
    s = device_solver(prob, 30, fs)
    s.set_params(params)
    assert s.inverse_path() == "chain_aug"
    K1o, D1 = O.kernel_kd(prob["kind"], prob["x1"], params["kernel_paras_1"], prob["jitter"], 2)
    K2o, D2 = O.kernel_kd(prob["kind"], prob["x2"], params["kernel_paras_2"], prob["jitter"], 2)
    U = params["U"]
    Ao, Bo = np.linalg.solve(K1o, U), np.linalg.solve(K2o, U.T)
    tol = cond_tol(prob, params)
    assert rel(s.forward_field("K1"), K1o) < 1e-13
    assert rel(s.forward_field("K2"), K2o) < 1e-13
    assert rel(s.forward_field("K1inv_U"), Ao) < tol
    assert rel(s.forward_field("K2inv_Ut"), Bo) < tol
    assert rel(s.forward_field("U_xx"), D1 @ Ao) < tol
    assert rel(s.forward_field("U_yy"), (D2 @ Bo).T) < tol
    s.close()
