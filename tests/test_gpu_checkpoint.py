"""Checkpoint / resume of the drop-in train() loop (beyond the reference, whose
code/utils.py:580-597 pickles only the final params): a run stopped after a record epoch and
resumed from its .npz checkpoint in a fresh solver ends with the uninterrupted run's params,
optimizer state and record lists, bitwise; the JSONL perf log gets one line per record."""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _model(nepoch, N=40, tol=None):
    from gpk import model_GP_solver_2d as m2d
    from gpk.equations import EQUATIONS_2D
    from gpk.infras.exp_config import ExpConfig
    from gpk.model_GP_solver_2d import get_boundary_vals, get_mesh_data, get_source_val
    args = ExpConfig()
    args.parse({"equation": "poisson_2d-sin_sin", "kernel": "Matern52_Cos_1d", "nepoch": nepoch})
    tp = dict(m2d.build_config(args, EQUATIONS_2D), N_col=N, Q=8)
    if tol is not None:
        tp["tol"] = tol
    u, src = m2d.solution_2d(tp["equation"], None)
    xt, yt, ut = get_mesh_data(u, 30, 30, tp["scale"])
    x, y, umh = get_mesh_data(u, N, N, tp["scale"])
    src_vals = get_source_val(src, x, y).reshape((x.size, y.size))
    return m2d.SOLVER(get_boundary_vals(umh), (x, y), src_vals, 1e-6, (xt, yt), ut, tp)


def _state(model):
    count, mu, nu = model.dev.get_opt_state()
    return model.dev.get_flat(), count, mu, nu


def test_train_checkpoint_resume_matches_uninterrupted(tmp_path):
    nepoch = 60
    a = _model(nepoch)
    try:
        log_a, _, err_a = a.train(nepoch, verbose=False)
        st_a = _state(a)
    finally:
        a.dev.close()
    ck = str(tmp_path / "ck.npz")
    b = _model(nepoch)
    try:
        log_b, _, _ = b.train(nepoch, verbose=False, checkpoint=ck, stop_at=25)
        assert len(log_b["epoch_list"]) < len(log_a["epoch_list"])
    finally:
        b.dev.close()
    perf = tmp_path / "perf.jsonl"
    c = _model(nepoch)
    try:
        log_c, _, err_c = c.train(nepoch, verbose=False, resume=ck, perf_log=str(perf))
        st_c = _state(c)
    finally:
        c.dev.close()
    assert err_c == err_a
    for x, y in zip(st_a, st_c):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    assert log_a.keys() == log_c.keys()
    for k in log_a:
        assert len(log_a[k]) == len(log_c[k]), k
        for x, y in zip(log_a[k], log_c[k]):
            assert np.array_equal(np.asarray(x), np.asarray(y)), k
    lines = [json.loads(l) for l in perf.read_text().splitlines()]
    assert [l["epoch"] for l in lines] == log_c["epoch_list"][len(log_b["epoch_list"]):]
    assert all(l["steps"] > 0 and l["seconds"] > 0 for l in lines)


def test_resume_after_early_stop_record(tmp_path):
    """A record that meets both the early-stop rule and stop_at: the checkpoint (written at exactly
    the given path, no ".npz" appended) carries the early stop, so the resumed run stops where
    the uninterrupted one did -- same flag, epoch, params and records."""
    nepoch = 60
    a = _model(nepoch, tol=1e300)  # criterion < tol at the first record
    try:
        log_a, es_a, err_a = a.train(nepoch, verbose=False)
        st_a = _state(a)
    finally:
        a.dev.close()
    assert es_a["flag"] and es_a["epoch"] == log_a["epoch_list"][-1]
    ck = str(tmp_path / "ck")
    b = _model(nepoch, tol=1e300)
    try:
        b.train(nepoch, verbose=False, checkpoint=ck, stop_at=1)
    finally:
        b.dev.close()
    import os
    assert os.path.exists(ck) and not os.path.exists(ck + ".npz")
    c = _model(nepoch, tol=1e300)
    try:
        log_c, es_c, err_c = c.train(nepoch, verbose=False, resume=ck)
        st_c = _state(c)
    finally:
        c.dev.close()
    assert es_c == es_a and err_c == err_a
    for x, y in zip(st_a, st_c):
        assert np.array_equal(np.asarray(x), np.asarray(y))
    for k in log_a:
        assert len(log_a[k]) == len(log_c[k]), k
