"""CPU: the distance classes of include/gpk.h (GPK_FLAG_NO_DCLASS, gpk_distance_classes) --
per diagonal k = |i - j| the distinct exact fp64 values of |x_i - x_j| -- against a numpy count,
on the reference's collocation grids (linspace(0,1,N)*scale, code/model_GP_solver_2d.py:369-374)
and on grids that must fall back to the per-pair kernels."""
import numpy as np
import pytest

from gpk.core import distance_classes


def np_classes(x):
    n = len(x)
    per = [len(np.unique(np.abs(x[k:] - x[:n - k]))) for k in range(n)]
    return sum(per), max(per)


@pytest.mark.parametrize("n,scale", [(200, 1.0), (256, 2 * np.pi), (128, 2 * np.pi), (40, 2 * np.pi),
                                     (2048, 2 * np.pi), (1, 1.0), (2, 1.0)])
def test_linspace_grid_classes(n, scale):
    x = np.linspace(0, 1, n) * scale
    ncls, vmax = distance_classes(x)
    want, wmax = np_classes(x)
    assert (ncls, vmax) == (want, wmax)
    assert ncls < 8 * n  # ~5n classes instead of n^2 pairs


def test_random_grid_falls_back():
    x = np.sort(np.random.default_rng(0).uniform(0, 1, 300))
    ncls, vmax = distance_classes(x)
    assert ncls == 0 and vmax > 32


def test_duplicate_coordinates():
    # repeated points: d = 0 also off the main diagonal (its own class on that diagonal)
    x = np.array([0.0, 0.5, 0.5, 1.0, 1.0, 1.0])
    ncls, vmax = distance_classes(x)
    assert (ncls, vmax) == np_classes(x)
