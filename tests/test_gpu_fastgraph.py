"""GPU: the fast step graph (refinement GEMM stages left out while the cond(K) gate is closed with
margin, include/gpk.h GPK_FLAG_NO_FAST_GRAPH) is bitwise the full graph, and a fast batch that
meets an open gate is rolled back and rerun with the full graph.

The reference has no such switch (its LU solves are unrefined); the oracle-parity tests in
test_gpu_parity.py pin the full graph, and these tests pin the fast graph to it bit for bit."""
import numpy as np
import pytest

from oracle import gp_oracle as O
from tests.helpers import device_solver, problem_1d, problem_2d

pytestmark = pytest.mark.gpu


def _gate_lb(prob, params):
    """max over axes of K00 * max diag K^{-1}: the device's cond(K) lower bound (gpk_internal.h)."""
    if "x" in prob:
        axes = [(prob["x"], params["kernel_paras"])]
    else:
        axes = [(prob["x1"], params["kernel_paras_1"]), (prob["x2"], params["kernel_paras_2"])]
    out = 0.0
    for x, kp in axes:
        K = O.kernel_matrix(prob["kind"], x, kp, prob["jitter"])
        out = max(out, K[0, 0] * float(np.max(np.diag(np.linalg.inv(K)))))
    return out


def _case(name):
    if name == "2d_closed":
        prob, params, _, fs = problem_2d(n1=48, n2=40, Q=8, seed=6)
    elif name == "2d_open":
        prob, params, _, fs = problem_2d(eq="allencahn", kind="Matern52_1d", n1=40, n2=36, Q=5, seed=4)
    elif name == "1d_closed":
        prob, params, _ = problem_1d(n=64, Q=8, seed=6)
        fs = 20.0
    else:
        prob, params, _ = problem_1d(kind="SE_1d", n=40, Q=5, seed=1)
        fs = 20.0
    kp = params.get("kernel_paras", params.get("kernel_paras_1"))
    return prob, params, len(kp["freq"]), fs


def _state(s):
    cnt, mu, nu = s.get_opt_state()
    return s.get_flat(), cnt, mu, nu


@pytest.mark.parametrize("name", ["2d_closed", "1d_closed"])
def test_fast_graph_bitwise_full(name):
    from gpk._lib import GPK_FLAG_NO_FAST_GRAPH
    prob, params, Q, fs = _case(name)
    assert _gate_lb(prob, params) * 8 < 100  # precondition: gate closed with margin
    full = device_solver(prob, Q, fs, flags=GPK_FLAG_NO_FAST_GRAPH)
    fast = device_solver(prob, Q, fs)
    for s in (full, fast):
        s.set_params(params)
    assert fast.graph_mode() == (False, 0)  # new params: full graph until the gate is seen
    for b in range(4):
        l_full, l_fast = full.step(3), fast.step(3)
        assert np.array_equal(l_full, l_fast), b
        assert fast.graph_mode() == (True, 0)
        assert full.graph_mode()[0] is False
    for a, b in zip(_state(full), _state(fast)):
        assert np.array_equal(a, b)
    lf, gf = full.loss_grad()
    lq, gq = fast.loss_grad()
    assert lf == lq and np.array_equal(gf, gq)
    full.close()
    fast.close()


@pytest.mark.parametrize("name", ["2d_open", "1d_open"])
def test_fast_graph_rollback(name):
    from gpk._lib import GPK_FLAG_FAST_FIRST, GPK_FLAG_NO_FAST_GRAPH
    prob, params, Q, fs = _case(name)
    assert _gate_lb(prob, params) > 100  # precondition: refinement needed
    full = device_solver(prob, Q, fs, flags=GPK_FLAG_NO_FAST_GRAPH)
    fast = device_solver(prob, Q, fs, flags=GPK_FLAG_FAST_FIRST)
    for s in (full, fast):
        s.set_params(params)
    assert fast.graph_mode() == (True, 0)
    # loss_grad in fast mode meets the open gate: rerun with the full graph, nothing to restore
    lf, gf = full.loss_grad()
    lq, gq = fast.loss_grad()
    assert lf == lq and np.array_equal(gf, gq)
    assert fast.graph_mode() == (False, 1)
    fast.set_params(params)  # FAST_FIRST: back to fast mode
    l_full, l_fast = full.step(4), fast.step(4)
    assert np.array_equal(l_full, l_fast)
    assert fast.graph_mode() == (False, 2)  # rolled back once more, then stays on the full graph
    for a, b in zip(_state(full), _state(fast)):
        assert np.array_equal(a, b)
    assert np.array_equal(full.step(2), fast.step(2))
    assert fast.graph_mode() == (False, 2)
    full.close()
    fast.close()


@pytest.mark.parametrize("name", ["2d_closed", "2d_open", "1d_closed"])
def test_multi_step_graph_bitwise_single(name):
    """Batches of >= 8 steps run graphs of 8 captured steps (+ single-step graphs for the
    remainder): bitwise the same trajectory as one graph launch per step."""
    prob, params, Q, fs = _case(name)
    a = device_solver(prob, Q, fs)
    b = device_solver(prob, Q, fs)
    for s in (a, b):
        s.set_params(params)
    la = np.concatenate([a.step(2), a.step(19), a.step(16)])
    lb = np.concatenate([b.step(1) for _ in range(37)])
    assert np.array_equal(la, lb)
    for x, y in zip(_state(a), _state(b)):
        assert np.array_equal(x, y)
    a.close()
    b.close()


@pytest.mark.parametrize("name", ["2d_closed", "2d_open", "1d_closed"])
def test_prepared_batch_graphs_bitwise_single(name):
    """gpk_prepare(n) captures one graph per chunk size of a step(n) call (64 steps and the
    remainder); prepared calls of 150 (64 + 64 + 22) and 22 steps, and an unprepared length
    (falls back to 8-step + single-step graphs), are bitwise one graph launch per step --
    fast batches (their chunk checks and rollbacks) included."""
    prob, params, Q, fs = _case(name)
    a = device_solver(prob, Q, fs)
    b = device_solver(prob, Q, fs)
    for s in (a, b):
        s.set_params(params)
    a.prepare(150)
    la = np.concatenate([a.step(150), a.step(22), a.step(13)])
    lb = np.concatenate([b.step(1) for _ in range(185)])
    assert np.array_equal(la, lb)
    for x, y in zip(_state(a), _state(b)):
        assert np.array_equal(x, y)
    a.close()
    b.close()


@pytest.mark.parametrize("name", ["2d_open", "1d_open"])
def test_single_step_call_graph_rollback(name):
    """step(1) runs one captured call graph (batch begin + step + pinned-memory report); a fast
    call that meets an open gate restores the snapshot that graph took and reruns on the full
    graph: bitwise the full-graph trajectory, call after call."""
    from gpk._lib import GPK_FLAG_FAST_FIRST, GPK_FLAG_NO_FAST_GRAPH
    prob, params, Q, fs = _case(name)
    full = device_solver(prob, Q, fs, flags=GPK_FLAG_NO_FAST_GRAPH)
    fast = device_solver(prob, Q, fs, flags=GPK_FLAG_FAST_FIRST)
    for s in (full, fast):
        s.set_params(params)
    lf = [full.step(1)[0] for _ in range(3)]
    lq = [fast.step(1)[0] for _ in range(3)]
    assert lf == lq
    assert fast.graph_mode() == (False, 1)
    for a, b in zip(_state(full), _state(fast)):
        assert np.array_equal(a, b)
    full.close()
    fast.close()


def test_step_returns_on_report_and_later_calls_are_ordered():
    """Whole-call graphs fold the batch begin into the chain launch and the report into the last
    step's loss workgroup, and gpk_step returns on the report's ready word -- before the last
    step's U update has finished.  Everything after it on the handle is stream-ordered: state read
    right after step(1) is the state after the update, and 20 x step(1) is bitwise step(20)."""
    from gpk.problems import make_solver
    a = make_solver("C4", seed=0)
    b = make_solver("C4", seed=0)
    try:
        a.prepare(20)
        la = np.concatenate([a.step(1) for _ in range(20)])
        early = _state(a)  # no sync: ordered after the last call's tail on the handle's stream
        a.sync()
        for x, y in zip(early, _state(a)):
            assert np.array_equal(x, y)
        b.prepare(20)
        lb = b.step(20)
        assert np.array_equal(la, lb)
        for x, y in zip(_state(a), _state(b)):
            assert np.array_equal(x, y)
        assert np.all(np.isfinite(la))
    finally:
        a.close()
        b.close()


def test_many_single_step_calls_bitwise_one_long_call():
    """500 step(1) calls (each returning on its report's ready word while the device still runs
    the previous call's tail) against one step(500) call (prepared 64-step chunks + remainder):
    bitwise the same losses and final state."""
    from gpk.problems import make_solver
    a = make_solver("C4", seed=1)
    b = make_solver("C4", seed=1)
    try:
        la = np.concatenate([a.step(1) for _ in range(500)])
        b.prepare(500)
        lb = b.step(500)
        assert np.array_equal(la, lb)
        for x, y in zip(_state(a), _state(b)):
            assert np.array_equal(x, y)
        assert a.graph_mode()[1] == b.graph_mode()[1]  # same rollbacks
    finally:
        a.close()
        b.close()


def test_long_first_call_then_fast_graph_c4():
    """A handle's first call of 200 steps (round 4's bench with --warmup 200) starts on the full
    graph, but both graphs now run in 64-step chunks while the fast one is available, so the mode
    is re-decided every chunk: the next call runs on the fast graph.  Bitwise the same trajectory
    as 200 steps in 5-step calls (the fast graph is bitwise the full one)."""
    from gpk.problems import make_solver
    a = make_solver("C4", seed=0)
    b = make_solver("C4", seed=0)
    try:
        la = a.step(200)
        fast_a, _ = a.graph_mode()
        lb = np.concatenate([b.step(5) for _ in range(40)])
        assert fast_a, "still on the full graph after a 200-step first call"
        assert np.array_equal(la, lb)
        assert np.array_equal(a.get_flat(), b.get_flat())
    finally:
        a.close()
        b.close()
