"""Host-side drop-in surface (no GPU): names, flags, configs, record cadence, result-log format."""
import json
import os

import numpy as np
import pytest

from tests.conftest import PKG_DIR

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_kernel_classes_and_dispatch():
    from gpk import kernel_matrix as km
    for name in ["Matern52_Cos_1d", "SE_Cos_1d", "Matern52_1d", "SE_1d"]:
        cls = km.kernel_class(name)
        assert cls.__name__ == name and cls.KIND == name
        k = cls()
        for meth in ("kappa", "D_x1_kappa", "DD_x1_kappa"):
            assert callable(getattr(k, meth))
    with pytest.raises(Exception, match="Invalid Kernel"):
        km.kernel_class("Periodic_1d")
    assert km.Kernel_matrix(1e-6, km.SE_1d()).jitter == 1e-6


def test_record_cadence_matches_reference():
    """`if i % (nepoch / 20) == 0` with Python float division (code/model_GP_solver_2d.py:293)."""
    from gpk.solver_common import record_epochs
    assert record_epochs(100) == list(range(0, 100, 5))
    assert record_epochs(20) == list(range(20))
    assert record_epochs(30) == [0, 3, 6, 9, 12, 15, 18, 21, 24, 27]  # 1.5-step cadence
    assert record_epochs(7) == [0]  # i % 0.35 == 0 only at i = 0


def test_cli_flag_syntax():
    from gpk.cli import parse_flags
    f = parse_flags(["-equation='poisson_2d-sin_sin'", "-kernel=Matern52_Cos_1d", "-nepoch=100",
                     "--device", "3", "-flag"])
    assert f == {"equation": "poisson_2d-sin_sin", "kernel": "Matern52_Cos_1d", "nepoch": 100,
                 "device": 3, "flag": True}


def test_configs_present_and_parsed():
    import yaml
    cdir = os.path.join(PKG_DIR, "gpk", "config")
    names = sorted(os.listdir(cdir))
    assert "poisson_2d-sin_sin.yaml" in names and "advection-sin.yaml" in names and len(names) == 11
    for n in names:
        with open(os.path.join(cdir, n)) as f:
            c = yaml.safe_load(f)
        assert c["equation"] == n[:-5]
        for key in ("Q", "lr", "logdet", "llk_weight", "freq_scale", "N_col", "scale", "nepoch", "num_fold"):
            assert key in c, (n, key)


def test_build_config_like_reference():
    from gpk import model_GP_solver_2d as m2d
    from gpk.equations import EQUATIONS_2D
    from gpk.infras.exp_config import ExpConfig
    args = ExpConfig()
    args.parse({"equation": "poisson_2d-sin_sin", "kernel": "Matern52_Cos_1d", "nepoch": 100})
    cfg = m2d.build_config(args, EQUATIONS_2D)
    assert cfg["scale"] == 2 * np.pi and cfg["nepoch"] == 100 and cfg["kernel"].__name__ == "Matern52_Cos_1d"
    assert cfg["other_paras"].endswith("-Ncol-400")
    with pytest.raises(AssertionError):
        args.equation = "heat_2d"
        m2d.build_config(args, EQUATIONS_2D)


def test_result_log_format_matches_reference_log(tmp_path, monkeypatch):
    """utils.wrirte_log writes the header line of the reference's committed log byte-for-byte."""
    from gpk import model_GP_solver_2d as m2d
    from gpk import utils
    from gpk.equations import EQUATIONS_2D
    from gpk.infras.exp_config import ExpConfig
    with open(os.path.join(GOLD, "ref_runs.json")) as f:
        ref = json.load(f)["poisson_2d-sin_sin/Matern52_Cos_1d"]
    args = ExpConfig()
    args.parse({"equation": "poisson_2d-sin_sin", "kernel": "Matern52_Cos_1d", "nepoch": 100})
    cfg = m2d.build_config(args, EQUATIONS_2D)
    monkeypatch.chdir(tmp_path)

    class _M:
        cov_func = cfg["kernel"]()
    err = {"mean": 0.4676, "std": 0.0, "used_time": 1.0, "avg_time": 1.0, "stop_epoch_mean": 100,
           "err_list": [0.46758844]}
    utils.wrirte_log(_M(), err, cfg)
    path = tmp_path / "result_log/poisson_2d-sin_sin/kernel_Matern52_Cos_1d/epoch_100/Q30/log.txt"
    lines = path.read_text().splitlines()
    assert lines[0] == ref["log_header"]
    assert lines[1].startswith("err_mean: 0.4676, err_std: 0.0000")
    assert utils.get_save_name(cfg) == "llk_weight-200.0-nu-1-Q-30-epoch-100-lr-0.0100-freqscale=20-logdet-1-x-2pi-Ncol-400"


def test_tree_roundtrip_and_template():
    from gpk.core import params_template, tree_flatten, tree_unflatten
    t = params_template(1, 7, 1, 3)
    flat = np.arange(3 * 3 + 2 + 7, dtype=float)
    back = tree_unflatten(t, flat)
    assert np.array_equal(tree_flatten(back), flat)
    assert back["u"].shape == (7, 1) and isinstance(back["log_tau"], float)
    # 1D order: freq, log-ls, log-w, log_tau, log_v, u
    assert back["kernel_paras"]["freq"][0] == 0 and back["log_tau"] == 9 and back["u"][0, 0] == 11
    with pytest.raises(ValueError):
        tree_unflatten(t, np.zeros(3))


def test_problem_configs_match_baseline():
    from gpk.problems import CONFIGS, problem_arrays
    assert CONFIGS["C4"]["n"] == 256 and CONFIGS["C4"]["kernel"] == "Matern52_Cos_1d"
    assert CONFIGS["C3"]["kernel"] == "SE_Cos_1d" and CONFIGS["C2"]["n"] == 2048
    a = problem_arrays(CONFIGS["C3"])
    assert a["src"].shape == (128, 128) and a["bvals"].shape == (4 * 128,)
    b = problem_arrays(CONFIGS["C1"])
    assert list(b["bidx"]) == [0, 199]
