"""GPU: the persistent small-factor SPD inverse (one launch, sweeps ordered by flags;
include/gpk.h GPK_FLAG_NO_CHAIN) against the one-launch-per-sweep inverse.  It performs the
same operations in the same order, so loss, gradient and Adam trajectories are bitwise equal --
with the distance-class gather (K, Kc, D built inside the inverse launch) and with the per-pair
assembly alike.  The augmented form (GPK_FLAG_NO_CHAIN_AUG; A = K1^{-1} U, Bt, K^{-1} D^T out
of the same sweeps) solves by the sweep operator instead of explicit-inverse GEMMs: it agrees
with the oracle and the GEMM form to the solves' rounding budget."""
import numpy as np
import pytest

from tests.helpers import device_solver, problem_1d, problem_2d

pytestmark = pytest.mark.gpu


def _case(name):
    if name == "1d":
        prob, params, _ = problem_1d(n=200, Q=8, seed=2)  # C1 size: 224 padded, T = 7
        return prob, params, 8, 20.0
    if name == "1d_ac":
        prob, params, _ = problem_1d(eq="allencahn", kind="SE_Cos_1d", n=72, Q=6, seed=3)
        return prob, params, 6, 20.0
    if name == "2d":
        prob, params, _, fs = problem_2d(n1=96, n2=72, Q=8, seed=1)
        return prob, params, 8, fs
    if name == "adv":
        prob, params, _, fs = problem_2d(eq="advection", kind="Matern52_Cos_1d", n1=72, n2=64, Q=6, seed=2)
        return prob, params, 6, fs
    prob, params, _, fs = problem_2d(n1=256, n2=256, Q=30, seed=0)  # C4
    return prob, params, 30, fs


@pytest.mark.parametrize("name", ["1d", "1d_ac", "2d", "adv", "c4"])
@pytest.mark.parametrize("dclass", [True, False])
def test_chain_bitwise_sweeps(name, dclass):
    from gpk._lib import GPK_FLAG_NO_CHAIN, GPK_FLAG_NO_CHAIN_AUG, GPK_FLAG_NO_DCLASS
    prob, params, Q, fs = _case(name)
    base = (0 if dclass else GPK_FLAG_NO_DCLASS) | GPK_FLAG_NO_CHAIN_AUG
    a = device_solver(prob, Q, fs, flags=base)
    b = device_solver(prob, Q, fs, flags=base | GPK_FLAG_NO_CHAIN)
    for s in (a, b):
        s.set_params(params)
    la, ga = a.loss_grad()
    lb, gb = b.loss_grad()
    assert la == lb and np.array_equal(ga, gb)
    assert np.array_equal(a.step(6), b.step(6))
    assert np.array_equal(a.get_flat(), b.get_flat())
    a.close()
    b.close()


def test_chain_repeated_launches_rearm():
    """Many back-to-back inverses (captured multi-step graphs + predict) keep re-arming the
    hand-off flags: the trajectory of 40 steps in one call equals 40 single-step calls."""
    prob, params, Q, fs = _case("2d")
    a = device_solver(prob, Q, fs)
    b = device_solver(prob, Q, fs)
    for s in (a, b):
        s.set_params(params)
    la = a.step(40)
    lb = np.concatenate([b.step(1) for _ in range(40)])
    assert np.array_equal(la, lb)
    a.close()
    b.close()


@pytest.mark.parametrize("name", ["2d", "adv", "c4"])
@pytest.mark.parametrize("dclass", [True, False])
def test_chain_aug_matches_gemm_form_and_oracle(name, dclass):
    from gpk._lib import GPK_FLAG_NO_CHAIN_AUG, GPK_FLAG_NO_DCLASS
    from tests.helpers import rel
    from tests.test_gpu_parity import _cmp_lossgrad, cond_tol
    prob, params, Q, fs = _case(name)
    base = 0 if dclass else GPK_FLAG_NO_DCLASS
    a = device_solver(prob, Q, fs, flags=base)
    b = device_solver(prob, Q, fs, flags=base | GPK_FLAG_NO_CHAIN_AUG)
    for s in (a, b):
        s.set_params(params)
    la, ga = a.loss_grad()
    lb, gb = b.loss_grad()
    tol = cond_tol(prob, params)
    assert abs(la - lb) / abs(lb) < tol
    assert rel(ga, gb) < tol, rel(ga, gb)
    sa, sb = a.step(10), b.step(10)
    assert np.max(np.abs(sa - sb) / np.abs(sb)) < 1e-8
    a.close()
    b.close()
    _cmp_lossgrad(prob, params, Q, fs, flags=base)
