"""Bounded waits: a hand-off that never arrives fails the call instead of hanging the device, and a
failed gpk_step batch is undone (gpu).

gpk_set_wait_limit(1) makes every inter-workgroup wait whose first poll fails give up (status bit
2); every other wait of the launch -- and of the batch's later steps -- then gives up within 64
polls, so the graph drains.  The call must return GPK_ENOTPD ("hand-off timed out"), the handle's
params / Adam state must be exactly those before the call (the batch's snapshot), and after the
limit is lifted the next call must be bitwise the call a fresh handle makes (the hand-off slots,
flags and counters were reset).  Covered for the persistent chain inverse (fast and full graph),
the large-factor 128-wide inverse, the 1D macro-tile chain and an in-process sharded group.
"""
import numpy as np
import pytest

from tests.helpers import device_solver, problem_1d, problem_2d

pytestmark = pytest.mark.gpu


@pytest.fixture
def wait_limit():
    from gpk.core import set_wait_limit
    yield set_wait_limit
    set_wait_limit(0)


def _state(s):
    c, mu, nu = s.get_opt_state()
    return s.get_flat(), c, mu, nu


def _same_state(a, b):
    return (np.array_equal(a[0], b[0]) and a[1] == b[1] and np.array_equal(a[2], b[2])
            and np.array_equal(a[3], b[3]))


def _timeout_then_clean(make, params, wait_limit, steps, path_ok):
    from gpk._lib import GPKError, GPK_ENOTPD
    s = make()
    f = make()
    try:
        assert path_ok(s.inverse_path()), s.inverse_path()
        s.set_params(params)
        f.set_params(params)
        s.step(2)                      # a few clean steps first: Adam state and count are nonzero
        f.step(2)
        before = _state(s)
        wait_limit(1)
        with pytest.raises(GPKError) as ei:
            s.step(steps)
        wait_limit(0)
        assert ei.value.code == GPK_ENOTPD and "timed out" in str(ei.value), str(ei.value)
        s.sync()
        assert _same_state(_state(s), before), "the failed batch was not undone"
        with pytest.raises(GPKError):  # the loss_grad path reports it too
            wait_limit(1)
            s.loss_grad()
        wait_limit(0)
        # the next calls are those of a handle that never timed out
        assert np.array_equal(s.step(steps), f.step(steps))
        s.sync()
        f.sync()
        assert _same_state(_state(s), _state(f))
        ls, gs = s.loss_grad()
        lf, gf = f.loss_grad()
        assert ls == lf and np.array_equal(gs, gf)
    finally:
        s.close()
        f.close()


@pytest.mark.parametrize("steps,flags", [(1, 0), (5, 0), (3, 16)])
def test_chain_timeout_undoes_batch(steps, flags, wait_limit):
    """Persistent chain inverse (C4's path): step(1) (one whole-call graph), a multi-step fast
    batch, and the full graph (GPK_FLAG_NO_FAST_GRAPH = 16)."""
    prob, params, _, fs = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=96, n2=80, Q=5, seed=4)
    _timeout_then_clean(lambda: device_solver(prob, 5, fs, flags=flags), params, wait_limit, steps,
                        lambda p: p in ("chain", "chain_aug"))


def test_big_wide_timeout_undoes_batch(wait_limit):
    """The large-factor 128-wide inverse (C5's path), forced at 520^2: the update launches' pivot
    and fused-panel hand-offs."""
    from gpk._lib import GPK_FLAG_FORCE_BIG_SPD, GPK_FLAG_FORCE_WIDE_SPD
    prob, params, _, fs = problem_2d(eq="advection", kind="Matern52_Cos_1d", n1=520, n2=300, Q=4, seed=6)
    _timeout_then_clean(lambda: device_solver(prob, 4, fs, flags=GPK_FLAG_FORCE_BIG_SPD | GPK_FLAG_FORCE_WIDE_SPD),
                        params, wait_limit, 2, lambda p: p == "big_wide")


def test_chain_multi_timeout_undoes_batch(wait_limit):
    """The 1D macro-tile chain (C2's path), forced at N = 700."""
    from gpk._lib import GPK_FLAG_FORCE_CHAIN_MULTI
    prob, params, _ = problem_1d(n=700, Q=5, seed=2)
    _timeout_then_clean(lambda: device_solver(prob, 5, 20.0, flags=GPK_FLAG_FORCE_CHAIN_MULTI), params,
                        wait_limit, 3, lambda p: p == "chain_multi")


def test_group_timeout_is_enotpd(wait_limit):
    """A timeout is rank-local; an in-process group reports it as GPK_ENOTPD on the whole group
    (not as an internal status disagreement), and recovers."""
    from gpk._lib import GPKError, GPK_ENOTPD
    from tests.test_shard import _group
    from oracle import gp_oracle as O
    prob, params, _, fs = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=72, n2=64, Q=4, seed=8)
    g = _group(prob, 4, fs, 2)
    try:
        g.set_params(params)
        wait_limit(1)
        with pytest.raises(GPKError) as ei:
            g.loss_grad()
        wait_limit(0)
        assert ei.value.code == GPK_ENOTPD and "timed out" in str(ei.value), str(ei.value)
        g.set_params(params)
        lg, _ = g.loss_grad()
        lo, _ = O.loss_grad_2d(prob, params)
        assert abs(lg - lo) / abs(lo) < 1e-9
    finally:
        g.close()


def test_group_step_timeout_undone_on_every_rank(wait_limit):
    """A hand-off timeout inside a group's step batch: the status bits are summed over the group
    every sharded step (gpk_api.cpp status_allreduce), so every rank fails the batch and restores
    its snapshot -- params and Adam state equal the pre-call state on every rank, the ranks agree,
    and the next batch equals a group that never timed out."""
    from gpk._lib import GPKError, GPK_ENOTPD
    from tests.test_shard import _group
    prob, params, _, fs = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=72, n2=64, Q=4, seed=8)
    g = _group(prob, 4, fs, 2)
    f = _group(prob, 4, fs, 2)
    try:
        g.set_params(params)
        f.set_params(params)
        g.step(2)
        f.step(2)
        before = [g.rank_state(k) for k in range(2)]
        wait_limit(1)
        with pytest.raises(GPKError) as ei:
            g.step(3)
        wait_limit(0)
        assert ei.value.code == GPK_ENOTPD and "timed out" in str(ei.value), str(ei.value)
        after = [g.rank_state(k) for k in range(2)]
        for k in range(2):
            assert _same_state(after[k], before[k]), f"rank {k}: the failed batch was not undone"
        # (Adam moments of U are kept per rank for its own rows only; params and count are shared)
        assert np.array_equal(after[0][0], after[1][0]) and after[0][1] == after[1][1], \
            "the ranks disagree after the failed batch"
        assert np.array_equal(g.step(3), f.step(3))
        assert _same_state(g.rank_state(1), f.rank_state(1))
    finally:
        g.close()
        f.close()


def test_failure_in_second_chunk_keeps_first_chunk():
    """A call is split into 64-step batches whenever the handle has a fast graph, on the full
    (refining) graph too (include/gpk.h gpk_step): a hand-off timeout in the call's SECOND chunk
    undoes that chunk only -- the handle ends exactly where a handle that ran the first 64 steps
    alone is (params, Adam state, count), and the first chunk's losses were written."""
    import ctypes
    from gpk import _lib
    from gpk._lib import GPK_ENOTPD
    from gpk.core import set_wait_limit_chunk
    prob, params, _, fs = problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=96, n2=80, Q=5, seed=4)
    s = device_solver(prob, 5, fs)
    f = device_solver(prob, 5, fs)
    try:
        s.set_params(params)
        f.set_params(params)
        lf = f.step(64)
        f.sync()
        assert not s.graph_mode()[0], "the call must start on the full (refining) graph"
        set_wait_limit_chunk(1, 1)
        out = np.full(130, np.nan)
        try:
            rc = _lib.load().gpk_step(s._h, 130, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        finally:
            set_wait_limit_chunk(0, -1)
        assert rc == GPK_ENOTPD and b"timed out" in _lib.load().gpk_last_error(), rc
        s.sync()
        assert _same_state(_state(s), _state(f)), "chunk 0 must stay applied, chunk 1 undone"
        assert np.array_equal(out[:64], lf)
        # and the handle goes on as one that never failed
        assert np.array_equal(s.step(3), f.step(3))
    finally:
        s.close()
        f.close()
