"""3-axis Kronecker solver (gpk_create3 / gpk_step3) vs the 3-axis oracle.

The reference has no d > 2 solver: parity is against oracle/gp_oracle.py loss_grad_3d, which is
pinned by torch autograd of the dense-Kronecker log joint and by its 2-axis reduction
(tests/test_oracle.py) -- "parity unpinned" against the reference itself.
"""
import numpy as np
import pytest

from oracle import gp_oracle as O
from tests.helpers import problem_3d, rel

pytestmark = pytest.mark.gpu

KINDS = ["SE_Cos_1d", "Matern52_Cos_1d", "SE_1d", "Matern52_1d"]


def _solver(prob, Q, fs, lr=0.01):
    from gpk.model_GP_solver_3d import DeviceSolver3
    return DeviceSolver3(prob["eq"], prob["kind"], (prob["x1"], prob["x2"], prob["x3"]), prob["src"],
                         prob["bvals"], Q=Q, jitter=prob["jitter"], llk_weight=prob["llk_weight"],
                         logdet=prob["logdet"], lr=lr, freq_scale=fs)


def _tol(prob, params):
    c = max(np.linalg.cond(O.kernel_matrix(prob["kind"], prob[f"x{a}"], params[f"kernel_paras_{a}"],
                                           prob["jitter"])) for a in (1, 2, 3))
    return max(1e-10, 50 * c * np.finfo(float).eps)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("eq", ["poisson", "allencahn"])
def test_loss_grad_3d_vs_oracle(eq, kind):
    """Loss and every gradient block at seeded params, unequal axes (padding per axis)."""
    prob, params, fs = problem_3d(eq=eq, kind=kind, ns=(20, 14, 9), Q=4, seed=3)
    s = _solver(prob, 4, fs)
    try:
        s.set_params(params)
        assert np.array_equal(s.get_flat(), O.flatten_params(params))
        loss, g = s.loss_grad()
    finally:
        s.close()
    lo, go = O.loss_grad_3d(prob, params)
    tol = _tol(prob, params)
    assert abs(loss - lo) / abs(lo) < tol, (loss, lo)
    gd = O.unflatten_params(params, g)
    for k in go:
        assert rel(O.flatten_params(gd[k]), O.flatten_params(go[k])) < tol, (k, tol)


def test_adam_trajectory_3d_vs_oracle():
    """10 device Adam steps vs 10 oracle steps (optax.adam, lr 0.01) from the reference init
    with seeded U: losses and params."""
    prob, params, fs = problem_3d(eq="poisson", kind="Matern52_Cos_1d", ns=(24, 18, 12), Q=5, seed=8)
    s = _solver(prob, 5, fs)
    try:
        s.set_params(params)
        losses = s.step(10)
        flat = s.get_flat()
    finally:
        s.close()
    opt = O.Adam(0.01)
    st = opt.init(params)
    p = params
    ref = []
    for _ in range(10):
        lo, go = O.loss_grad_3d(prob, p)
        ref.append(lo)
        p, st = opt.update(go, st, p)
    tol = _tol(prob, params)
    assert rel(losses, ref) < max(1e-9, tol)
    assert rel(flat, O.flatten_params(p)) < max(1e-8, 10 * tol)


def test_init_params_3d_and_errors():
    """The handle starts at the 2-axis train() init extended to three axes; bad inputs raise."""
    from gpk._lib import GPKError
    prob, _, fs = problem_3d(eq="poisson", kind="SE_Cos_1d", ns=(8, 7, 6), Q=3, seed=1)
    s = _solver(prob, 3, fs)
    try:
        ref = O.init_params_3d(8, 7, 6, 3, fs)
        assert rel(s.get_flat(), O.flatten_params(ref)) < 1e-15
    finally:
        s.close()
    bad = dict(prob, kind="Nope")
    with pytest.raises(KeyError):
        _solver(bad, 3, fs)
    with pytest.raises((GPKError, ValueError)):
        _solver(dict(prob, bvals=prob["bvals"][:-1]), 3, fs)
