"""Shared problem builders for the parity tests (test infrastructure)."""
import numpy as np

from oracle import gp_oracle as O


def rand_kp(rng, Q, fs):
    return {"freq": np.linspace(0, 1, Q) * fs + 0.3 * rng.normal(size=Q),
            "log-ls": 0.3 * rng.normal(size=Q),
            "log-w": np.log(1.0 / Q) + 0.3 * rng.normal(size=Q)}


def problem_1d(eq="poisson", kind="Matern52_Cos_1d", n=40, Q=5, seed=0, scale=2 * np.pi, fs=20.0):
    name = {"poisson": "poisson_1d-single_sin", "allencahn": "allencahn_1d-single_sin"}[eq]
    prob, Xte, Yte = O.setup_1d(name, n, scale, kind)
    rng = np.random.default_rng(seed)
    params = {"kernel_paras": rand_kp(rng, Q, fs), "log_tau": 0.2, "log_v": -0.1,
              "u": 0.1 * rng.normal(size=(n, 1))}
    return prob, params, (Xte, Yte)


def problem_2d(eq="poisson", kind="Matern52_Cos_1d", n1=24, n2=20, Q=5, seed=0, fs=20.0):
    if eq == "advection":
        prob, Xte, ute = O.setup_2d("advection-multiscale", n1, 1.0, kind, llk_weight=500.0,
                                    beta=200.0, n_col2=n2, m_test=30)
        fs = 40.0
    elif eq == "allencahn":
        prob, Xte, ute = O.setup_2d("allencahn_2d-mix-sincos", n1, 1.0, kind, n_col2=n2, m_test=30)
        fs = 30.0
    else:
        prob, Xte, ute = O.setup_2d("poisson_2d-sin_sin", n1, 2 * np.pi, kind, n_col2=n2, m_test=30)
    rng = np.random.default_rng(seed)
    params = {"U": 0.1 * rng.normal(size=(n1, n2)), "kernel_paras_1": rand_kp(rng, Q, fs),
              "kernel_paras_2": rand_kp(rng, Q, fs), "log_tau": 0.2, "log_v": -0.1}
    return prob, params, (Xte, ute), fs


def problem_3d(eq="poisson", kind="Matern52_Cos_1d", ns=(10, 8, 6), Q=4, seed=0, fs=5.0):
    """A 3-axis Kronecker problem (oracle setup_3d) with seeded random params."""
    name = {"poisson": "poisson_3d-mix_sin", "allencahn": "allencahn_3d-sin"}[eq]
    prob = O.setup_3d(name, ns, 2 * np.pi if eq == "poisson" else 1.0, kind)
    rng = np.random.default_rng(seed)
    params = {"U": 0.1 * rng.normal(size=ns), "kernel_paras_1": rand_kp(rng, Q, fs),
              "kernel_paras_2": rand_kp(rng, Q, fs), "kernel_paras_3": rand_kp(rng, Q, fs),
              "log_tau": 0.2, "log_v": -0.1}
    return prob, params, fs


def config_problem(cid, seed=0, m_test=8):
    """The oracle problem + params of a BASELINE config (gpk.problems.CONFIGS), the random field
    seeded exactly as gpk.problems.make_solver seeds it (the bench's inputs); returns
    (prob, params, (test inputs, test solution), cfg).  m_test=300 is the reference's test grid
    (code/model_GP_solver_2d.py:369-374, code/model_GP_solver_1d.py:307-312)."""
    from gpk.problems import CONFIGS
    cfg = CONFIGS[cid]
    n = cfg["n"]
    rng = np.random.default_rng(seed)
    if cfg["dim"] == 1:
        prob, Xte, ute = O.setup_1d(cfg["equation"], n, cfg["scale"], cfg["kernel"],
                                    llk_weight=cfg["llk_weight"], m_test=m_test)
        params = O.init_params_1d(n, 30, cfg["freq_scale"])
        params["u"] = 0.1 * rng.normal(size=n).reshape(n, 1)
    else:
        prob, Xte, ute = O.setup_2d(cfg["equation"], n, cfg["scale"], cfg["kernel"],
                                    llk_weight=cfg["llk_weight"], beta=cfg.get("beta"), m_test=m_test)
        params = O.init_params_2d(n, n, 30, cfg["freq_scale"])
        params["U"] = 0.1 * rng.normal(size=n * n).reshape(n, n)
    return prob, params, (Xte, ute), cfg


def device_solver(prob, Q, fs=20.0, lr=0.01, flags=0):
    from gpk.core import DeviceSolver
    if "x" in prob:
        return DeviceSolver(1, prob["eq"], prob["kind"], prob["x"], prob["src"], prob["y"],
                            bidx=prob["xind"], Q=Q, jitter=prob["jitter"],
                            llk_weight=prob["llk_weight"], logdet=prob["logdet"], lr=lr,
                            freq_scale=fs, flags=flags)
    return DeviceSolver(2, prob["eq"], prob["kind"], prob["x1"], prob["src"], prob["bvals"],
                        x2=prob["x2"], Q=Q, jitter=prob["jitter"], llk_weight=prob["llk_weight"],
                        logdet=prob["logdet"], beta=prob.get("beta", 1.0), lr=lr, freq_scale=fs,
                        flags=flags)


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def extra_params(rng, n):
    """Seeded extra-GP params (model_GP_solver_1d_extra.py:317-328 shapes, perturbed)."""
    return {"log_tau": 0.1, "log_v": -0.2,
            "kernel_paras": {"log-w": 0.2 * rng.normal(size=1), "log-ls": 0.2 * rng.normal(size=1)},
            "u": 0.05 * rng.normal(size=(n, 1))}


def record_parity(test, config, errors, tol=None, extra=None):
    """Append one line of observed parity errors (per key) to $GPK_PARITY_LOG (default
    gpurun_out/parity.jsonl): the GPU parity tests' margins, summarised into profiles/r*_parity.json
    (tools/parity_summary.py).  Never fails a test."""
    import json
    import os
    import time
    path = os.environ.get("GPK_PARITY_LOG", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "parity.jsonl"))
    rec = {"test": test, "config": config, "errors": {k: float(v) for k, v in errors.items()},
           "time": time.strftime("%Y-%m-%dT%H:%M:%S")}
    if tol is not None:
        rec["tol"] = {k: float(v) for k, v in tol.items()} if isinstance(tol, dict) else float(tol)
    if extra:
        rec.update(extra)
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")
    except OSError:
        pass
