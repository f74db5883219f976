"""Pipelined class values (gpk.h GPK_FLAG_NO_CLASS_PIPE): in a multi-step batch, step s + 1's class
values are evaluated at the end of step s's parameter-gradient launch, right after the kernel-
parameter Adam, and step s + 1 skips its class-value launch.  The values come from the same
parameters through the same code (prep_dev.h class_value_store), so every trajectory must be
BITWISE the one of a handle that launches the class values in every step -- across batch
boundaries, set_params between calls, the fast graph's rollback, 1D and 2D, padded axes and the
advection sign.  (The default path is also the one every other GPU parity test runs.)"""
import numpy as np
import pytest

from tests.helpers import config_problem, device_solver, problem_1d, problem_2d

pytestmark = pytest.mark.gpu


def _pair(prob, Q, fs, flags=0):
    from gpk._lib import GPK_FLAG_NO_CLASS_PIPE
    a = device_solver(prob, Q, fs, flags=flags)
    b = device_solver(prob, Q, fs, flags=flags | GPK_FLAG_NO_CLASS_PIPE)
    return a, b


def _same_trajectory(a, b, params, calls):
    for s in (a, b):
        s.set_params(params)
    for n in calls:
        la, lb = a.step(n), b.step(n)
        assert np.array_equal(la, lb), (n, np.max(np.abs(la - lb)))
        assert np.array_equal(a.get_flat(), b.get_flat()), n


@pytest.mark.parametrize("eq,kind,n1,n2,Q", [("poisson", "Matern52_Cos_1d", 40, 36, 8),
                                             ("advection", "Matern52_Cos_1d", 72, 40, 6),
                                             ("allencahn", "SE_Cos_1d", 72, 40, 6),
                                             ("poisson", "Matern52_Cos_1d", 256, 256, 30)])
def test_pipelined_class_values_bitwise_2d(eq, kind, n1, n2, Q):
    prob, params, _, fs = problem_2d(eq=eq, kind=kind, n1=n1, n2=n2, Q=Q, seed=11)
    a, b = _pair(prob, Q, fs)
    try:
        assert a.class_pipe() and not b.class_pipe()
        _same_trajectory(a, b, params, (1, 2, 9, 20, 3))
        # new parameters between calls: the next call's first step evaluates its own class values
        rng = np.random.default_rng(5)
        p2 = dict(params)
        p2["kernel_paras_1"] = {k: v + 0.05 * rng.normal(size=len(v)) for k, v in params["kernel_paras_1"].items()}
        _same_trajectory(a, b, p2, (7, 1, 20))
    finally:
        a.close()
        b.close()


def test_pipelined_class_values_bitwise_fast_rollback():
    """The fast graph's rollback (FAST_FIRST: a step that needed refinement undoes its batch and
    reruns it on the full graph) with pipelined class values in both graphs."""
    from gpk._lib import GPK_FLAG_FAST_FIRST
    prob, params, _, fs = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=40, n2=36, Q=8, seed=2)
    a, b = _pair(prob, 8, fs, flags=GPK_FLAG_FAST_FIRST)
    try:
        _same_trajectory(a, b, params, (12, 12))
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("n,Q", [(40, 5), (200, 30)])
def test_pipelined_class_values_bitwise_1d(n, Q):
    prob, params, _ = problem_1d(eq="poisson", kind="Matern52_Cos_1d", n=n, Q=Q, seed=4)
    a, b = _pair(prob, Q, 20.0)
    try:
        assert a.class_pipe() and not b.class_pipe()
        _same_trajectory(a, b, params, (1, 9, 20))
    finally:
        a.close()
        b.close()


def test_pipelined_class_values_bitwise_c2():
    """C2 (1D, p = 2048: the macro-tile chain, class-operand GEMVs)."""
    prob, params, _, cfg = config_problem("C2")
    a, b = _pair(prob, 30, cfg["freq_scale"])
    try:
        assert a.inverse_path() == "chain_multi" and a.class_pipe()
        _same_trajectory(a, b, params, (5, 1))
    finally:
        a.close()
        b.close()
