"""GPU: the distance-class step (include/gpk.h GPK_FLAG_NO_DCLASS; fields evaluated once per
distinct |x_i - x_j|, hyper-parameter gradient contracted per class) against the per-pair
kernels and the oracle.  The two paths evaluate the same closed forms at the same fp64
distances; they differ only in the order in which mixture components and gradient terms are
summed, so they agree to the rounding budget of the solves (cond(K) * eps)."""
import numpy as np
import pytest

from oracle import gp_oracle as O
from tests.helpers import device_solver, problem_1d, problem_2d, rel
from tests.test_gpu_parity import _cmp_lossgrad, cond_tol

pytestmark = pytest.mark.gpu


def _pair(prob, Q, fs, params):
    from gpk._lib import GPK_FLAG_NO_DCLASS
    cls = device_solver(prob, Q, fs)
    pair = device_solver(prob, Q, fs, flags=GPK_FLAG_NO_DCLASS)
    for s in (cls, pair):
        s.set_params(params)
    assert all(c > 0 for c in cls.class_counts())
    assert all(c == 0 for c in pair.class_counts())
    return cls, pair


def _u_mask(prob, params):
    flat = O.flatten_params(params)
    names = O.unflatten_params(params, np.arange(len(flat), dtype=np.float64))
    key = "U" if "U" in names else "u"
    m = np.zeros(len(flat), bool)
    m[np.asarray(O.flatten_params(names[key]), dtype=int)] = True
    return m


CASES = [("1d", "poisson", "Matern52_Cos_1d"), ("1d", "allencahn", "SE_1d"),
         ("2d", "poisson", "Matern52_Cos_1d"), ("2d", "allencahn", "SE_Cos_1d"),
         ("2d", "advection", "Matern52_Cos_1d"), ("2d", "poisson", "Matern52_1d")]


def _problem(dim, eq, kind):
    if dim == "1d":
        prob, params, _ = problem_1d(eq=eq, kind=kind, n=72, Q=6, seed=3)
        return prob, params, 6, 20.0
    prob, params, _, fs = problem_2d(eq=eq, kind=kind, n1=72, n2=40, Q=6, seed=3)
    return prob, params, 6, fs


@pytest.mark.parametrize("dim,eq,kind", CASES)
def test_class_path_matches_pairs(dim, eq, kind):
    prob, params, Q, fs = _problem(dim, eq, kind)
    cls, pair = _pair(prob, Q, fs, params)
    lc, gc = cls.loss_grad()
    lp, gp = pair.loss_grad()
    tol = cond_tol(prob, params)
    assert abs(lc - lp) / abs(lp) < tol
    m = _u_mask(prob, params)
    assert rel(gc[m], gp[m]) < tol, rel(gc[m], gp[m])
    assert rel(gc[~m], gp[~m]) < tol, rel(gc[~m], gp[~m])
    cls.close()
    pair.close()
    _cmp_lossgrad(prob, params, Q, fs)  # and the oracle (class path: the default)


@pytest.mark.parametrize("dim", ["1d", "2d"])
def test_class_path_trajectory(dim):
    prob, params, Q, fs = _problem(dim, "poisson", "Matern52_Cos_1d")
    cls, pair = _pair(prob, Q, fs, params)
    a, b = cls.step(20), pair.step(20)
    assert np.max(np.abs(a - b) / np.abs(b)) < 1e-9
    assert rel(cls.get_flat(), pair.get_flat()) < 1e-8
    cls.close()
    pair.close()


def test_class_path_deterministic():
    prob, params, Q, fs = _problem("2d", "poisson", "Matern52_Cos_1d")
    out = []
    for _ in range(2):
        s = device_solver(prob, Q, fs)
        s.set_params(params)
        out.append((s.step(5), s.get_flat()))
        s.close()
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])


def test_random_grid_uses_pairs_and_matches_oracle():
    prob, params, Q, fs = _problem("2d", "poisson", "Matern52_Cos_1d")
    rng = np.random.default_rng(7)
    prob = dict(prob)
    prob["x1"] = np.sort(rng.uniform(0, 2 * np.pi, len(prob["x1"])))
    s = device_solver(prob, Q, fs)
    assert s.class_counts() == [0, 0]  # axis 1 is scattered: both axes stay per-pair
    s.close()
    _cmp_lossgrad(prob, params, Q, fs)


def test_c4_size_class_counts():
    prob, params, _, fs = problem_2d(n1=256, n2=256, Q=30, seed=0)
    s = device_solver(prob, 30, fs)
    assert s.class_counts() == [1297, 1297]
    assert s.class_sums_in_epilogue()  # 9 variants per diagonal at most: the GEMM epilogue path
    s.close()


# The class sums of G_K / G_D formed in the epilogues of the GEMMs that produce them (default,
# gpk.h GPK_FLAG_NO_CLASS_BINS) against the class-sum launch: the same pairs summed in another
# order, so the kernel-parameter gradients agree to rounding, everything else bitwise (the loss
# and dL/dU never read the class sums).  Padded axes (72 x 40 -> 96 x 64), the D_x1 sign
# (advection), Allen-Cahn, and C4's size (9 variants on some diagonals: the v + 8 slots).
@pytest.mark.parametrize("eq,kind,n1,n2", [("poisson", "Matern52_Cos_1d", 72, 40),
                                           ("advection", "Matern52_Cos_1d", 72, 40),
                                           ("allencahn", "SE_Cos_1d", 72, 40),
                                           ("poisson", "Matern52_Cos_1d", 256, 256)])
def test_epilogue_class_sums_match_class_sum_launch(eq, kind, n1, n2):
    from gpk._lib import GPK_FLAG_NO_CLASS_BINS
    Q = 30 if n1 == 256 else 6
    prob, params, _, fs = problem_2d(eq=eq, kind=kind, n1=n1, n2=n2, Q=Q, seed=3)
    a = device_solver(prob, Q, fs)
    b = device_solver(prob, Q, fs, flags=GPK_FLAG_NO_CLASS_BINS)
    try:
        assert a.class_sums_in_epilogue() and not b.class_sums_in_epilogue()
        for s in (a, b):
            s.set_params(params)
        la, ga = a.loss_grad()
        lb, gb = b.loss_grad()
        assert la == lb
        m = _u_mask(prob, params)
        assert np.array_equal(ga[m], gb[m])
        assert rel(ga[~m], gb[~m]) < 1e-10, rel(ga[~m], gb[~m])
        # and after steps (the step graph's own stages): trajectories within rounding (Adam's
        # normalised steps amplify last-bit differences of near-zero gradient components: the
        # class-path-vs-pairs budget above)
        ta, tb = a.step(10), b.step(10)
        assert np.max(np.abs(ta - tb) / np.abs(tb)) < 1e-9
        assert rel(a.get_flat(), b.get_flat()) < 1e-8
    finally:
        a.close()
        b.close()
    if n1 < 256:
        _cmp_lossgrad(prob, params, Q, fs)  # and the oracle (the default path)



@pytest.mark.parametrize("eq,n1,n2,big", [("advection", 1056, 64, True), ("poisson", 1024, 1056, False),
                                           ("poisson", 2048, 512, False), ("advection", 320, 1664, False)])
def test_wide_gather_bitwise_class_table(eq, n1, n2, big):
    """The large-factor gather (max p >= 1024: gather_wide_kernel, class = cbase[|i - j|] + the
    pair's variant byte) writes exactly the class table's values on EVERY axis, the one below
    1024 included: K (+ jitter), its kept copy and D (with the advection sign) bitwise equal to
    the host expansion of (class ids, class values).  (the variant bytes used to be
    built only for axes with p >= 1024, and the launch returned without assembling anything
    when one axis lacked them.)"""
    from gpk._lib import GPK_FLAG_FORCE_BIG_SPD
    prob, params, _, fs = problem_2d(eq=eq, kind="Matern52_Cos_1d", n1=n1, n2=n2, Q=4, seed=5)
    s = device_solver(prob, 4, fs, flags=GPK_FLAG_FORCE_BIG_SPD if big else 0)
    try:
        s.set_params(params)
        s.loss_grad()
        for a in (1, 2):
            kc, kcls = s.forward_field(f"Kc{a}"), s.forward_field(f"K{a}_classes")
            assert np.isfinite(kc).all() and np.any(kc != 0)
            assert np.array_equal(kc, kcls)
            assert np.array_equal(s.forward_field(f"D{a}"), s.forward_field(f"D{a}_classes"))
    finally:
        s.close()


def test_wide_gather_unequal_axes_loss_grad():
    """2048 x 512 (the large-factor path on axis 1; axis 2 below the wide gather's own size):
    loss and full gradient against the oracle."""
    prob, params, _, fs = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=2048, n2=512, Q=4, seed=7)
    _cmp_lossgrad(prob, params, 4, fs, extended=False)
