"""The 128-wide SPD inverse's two-sweep update schedule (csrc/spdinv_big.hip wide_schedule, via
the host-only ABI entry gpk_wide_schedule): replayed on the CPU with small blocks, the schedule's
tile lists and composed coefficients must turn K into K^{-1} exactly as the one-sweep form does
(block Gauss-Jordan with Cholesky pivots, the update of the reference's solves / slogdet,
code/model_GP_solver_advection.py:104-105, 153-158), every tile applying every sweep once, in
order, at most one sweep late, and the next panel's row / column and pivot up to date when read."""
import ctypes

import numpy as np
import pytest

from gpk import _lib


def schedule(T2, paired):
    S = 2 + T2 * (T2 + 1) // 2
    out = (ctypes.c_uint32 * (T2 * S))()
    _lib.check(_lib.load().gpk_wide_schedule(T2, 1 if paired else 0, out, T2 * S))
    return np.frombuffer(out, dtype=np.uint32).reshape(T2, S)


def decode(e):
    code = {0: 0.0, 1: 1.0, 3: -1.0}
    return (int(e >> 8) & 255, int(e) & 255, bool((e >> 16) & 1), code[int(e >> 18) & 3],
            code[int(e >> 20) & 3], code[int(e >> 22) & 3])


def replay(K, b, tab):
    """Blocked sweeps on the lower b x b tiles of X driven by the schedule; returns X."""
    T2 = K.shape[0] // b
    X = {(I, J): K[I * b:(I + 1) * b, J * b:(J + 1) * b].copy() for I in range(T2) for J in range(I + 1)}
    lag = {t: -1 for t in X}                     # last sweep each tile has applied
    Z = {}

    def xt(I, J):                                # full-matrix block from the lower tiles
        return X[(I, J)] if I >= J else X[(J, I)].T

    for k in range(T2):
        # panel k (the previous launch's fused panel): row k must be current through sweep k - 1
        for J in range(T2):
            assert lag[(max(k, J), min(k, J))] == k - 1, ("stale panel input", k, J)
        L = np.linalg.cholesky(xt(k, k))
        Li = np.linalg.inv(L)
        Z[k] = np.hstack([Li if J == k else Li @ xt(k, J) for J in range(T2)])
        row = tab[k]
        ents = [row[2 + i] for i in range(int(row[0]))] + ([row[1]] if k + 1 < T2 else [])
        seen = set()
        for e in ents:
            I, J, two, c0, c1, c2 = decode(e)
            assert (I, J) not in seen
            seen.add((I, J))
            assert lag[(I, J)] == (k - 2 if two or lag[(I, J)] == k - 2 else k - 1), (k, I, J, lag[(I, J)])
            v = c0 * X[(I, J)] + c2 * Z[k][:, I * b:(I + 1) * b].T @ Z[k][:, J * b:(J + 1) * b]
            if two:
                v = v + c1 * Z[k - 1][:, I * b:(I + 1) * b].T @ Z[k - 1][:, J * b:(J + 1) * b]
            X[(I, J)] = v
            lag[(I, J)] = k
        for t in X:                               # never more than one sweep behind
            assert lag[t] >= k - 1, ("lagging tile", k, t)
    assert all(v == T2 - 1 for v in lag.values())
    out = np.zeros_like(K)
    for (I, J), v in X.items():
        out[I * b:(I + 1) * b, J * b:(J + 1) * b] = v
    return out


@pytest.mark.parametrize("T2", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("paired", [False, True])
def test_schedule_inverts(T2, paired):
    rng = np.random.default_rng(T2)
    b = 3
    n = T2 * b
    M = rng.normal(size=(n, n))
    K = M @ M.T / n + 0.5 * np.eye(n)
    tab = schedule(T2, paired)
    X = replay(K, b, tab)
    Ki = np.linalg.inv(K)
    low = np.tril(np.ones((T2, T2)))
    mask = np.kron(low, np.ones((b, b))).astype(bool)
    assert np.max(np.abs(X[mask] - Ki[mask])) < 1e-10 * np.max(np.abs(Ki))


def test_schedule_halves_the_passes():
    """At C5's 32 tiles per dimension the paired schedule writes each tile ~once per two sweeps:
    0.545x the one-sweep form's tile passes, 83 % of them carrying two sweeps (K = 256)."""
    T2 = 32
    one, two = schedule(T2, False), schedule(T2, True)
    nt = T2 * (T2 + 1) // 2
    assert all(int(one[k][0]) + (1 if k + 1 < T2 else 0) == nt for k in range(T2))
    w1 = sum(int(one[k][0]) for k in range(T2))
    w2 = sum(int(two[k][0]) for k in range(T2))
    pairs = sum(int(decode(two[k][2 + i])[2]) for k in range(T2) for i in range(int(two[k][0])))
    assert w2 < 0.56 * w1
    assert pairs > 0.8 * w2


@pytest.mark.parametrize("T2", [3, 8, 32])
def test_pivot_tile_one_sweep(T2):
    """The pivot workgroup's tile (k + 1, k + 1), first on the launch's serial chain, carries one
    sweep (K = 128) in every launch of the paired schedule: it was brought up to date one
    launch earlier."""
    tab = schedule(T2, True)
    for k in range(T2 - 1):
        I, J, two = decode(tab[k][1])[:3]
        assert (I, J) == (k + 1, k + 1)
        assert not two, k
