"""Edge cases of the step path on the device vs the oracle (the reference's own tests
exercise only its configs; these pin the padding and size boundaries of the HIP path): the
smallest grids (2 collocation points per axis: boundary rows only), sizes around the 32-row
padding (31/32/33, 63/64/65), one mixture component and the maximum (Q = 64), zero-step calls,
and the argument checks of gpk_create (the reference raises on an unknown kernel name; the ABI
returns GPK_EINVAL with a message)."""
import numpy as np
import pytest

from tests.helpers import device_solver, problem_1d, problem_2d, rel
from tests.test_gpu_parity import _cmp_lossgrad

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2, 3, 31, 32, 33, 63, 64, 65])
@pytest.mark.parametrize("eq", ["poisson", "allencahn"])
def test_1d_sizes_around_padding(n, eq):
    prob, params, _ = problem_1d(eq=eq, kind="Matern52_Cos_1d", n=n, Q=4, seed=n)
    _cmp_lossgrad(prob, params, 4, 20.0)


@pytest.mark.parametrize("n1,n2", [(2, 2), (3, 3), (2, 33), (33, 31), (32, 64), (65, 3)])
@pytest.mark.parametrize("eq", ["poisson", "advection"])
def test_2d_sizes_around_padding(n1, n2, eq):
    prob, params, _, fs = problem_2d(eq=eq, kind="SE_Cos_1d", n1=n1, n2=n2, Q=3, seed=n1 + n2)
    _cmp_lossgrad(prob, params, 3, fs)


@pytest.mark.parametrize("Q", [1, 64])
@pytest.mark.parametrize("dim", [1, 2])
def test_mixture_size_limits(Q, dim):
    if dim == 1:
        prob, params, _ = problem_1d(eq="poisson", kind="SE_Cos_1d", n=40, Q=Q, seed=Q)
        _cmp_lossgrad(prob, params, Q, 20.0)
    else:
        prob, params, _, fs = problem_2d(eq="allencahn", kind="Matern52_Cos_1d", n1=24, n2=20, Q=Q, seed=Q)
        _cmp_lossgrad(prob, params, Q, fs)


def test_zero_step_call_changes_nothing():
    prob, params, _, fs = problem_2d(n1=24, n2=20, Q=3, seed=3)
    s = device_solver(prob, 3, fs)
    try:
        s.set_params(params)
        before = s.get_flat()
        out = s.step(0)
        assert len(out) == 0
        assert np.array_equal(before, s.get_flat())
        l0, g0 = s.loss_grad()
        s.step(1)
        assert not np.array_equal(before, s.get_flat())
    finally:
        s.close()


def test_create_rejects_bad_sizes():
    from gpk import _lib
    prob, params, _ = problem_1d(n=8, Q=3)
    with pytest.raises(_lib.GPKError, match="Q must be in"):
        device_solver(prob, 65)
    with pytest.raises(_lib.GPKError, match="Q must be in"):
        device_solver(prob, 0)
