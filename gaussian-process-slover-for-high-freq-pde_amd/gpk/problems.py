"""BASELINE.json configurations as concrete synthetic problems.

Grids follow test() of the reference (linspace(0,1,N)*scale, model_GP_solver_2d.py:369-374);
sources are the analytic Laplacian / advection operator of the configured exact solution
(the reference differentiates it with jax.grad, model_GP_solver_2d.py:355-366).
"""
import numpy as np

from .core import DeviceSolver
from .equations import boundary_2d, solution_1d, solution_2d

CONFIGS = {
    # id: dim, equation, kernel, N (per axis), scale, freq_scale, llk_weight, beta
    "C1": dict(dim=1, equation="poisson_1d-single_sin", kernel="Matern52_1d", n=200,
               scale=2 * np.pi, freq_scale=20.0, llk_weight=200.0),
    "C2": dict(dim=1, equation="poisson_1d-single_sin", kernel="Matern52_Cos_1d", n=2048,
               scale=2 * np.pi, freq_scale=20.0, llk_weight=200.0),
    "C3": dict(dim=2, equation="poisson_2d-sin_sin", kernel="SE_Cos_1d", n=128,
               scale=2 * np.pi, freq_scale=20.0, llk_weight=200.0),
    "C4": dict(dim=2, equation="poisson_2d-sin_sin", kernel="Matern52_Cos_1d", n=256,
               scale=2 * np.pi, freq_scale=20.0, llk_weight=200.0),
    "C5": dict(dim=2, equation="advection-multiscale", kernel="Matern52_Cos_1d", n=4096,
               scale=1.0, freq_scale=40.0, llk_weight=500.0, beta=200.0),
}

# The reference's own committed runs (code/result_log/*/kernel_Matern52_Cos_1d/epoch_100/Q30/
# log.txt:2: N_col 400, Q 30, lr 0.01, freq_scale 20): the configs its run times -- the CPU
# baseline's calibration points -- not BASELINE.json configs.
REFERENCE_RUNS = {
    "R1": dict(dim=1, equation="poisson_1d-single_sin", kernel="Matern52_Cos_1d", n=400,
               scale=2 * np.pi, freq_scale=20.0, llk_weight=200.0),
    "R2": dict(dim=2, equation="poisson_2d-sin_sin", kernel="Matern52_Cos_1d", n=400,
               scale=2 * np.pi, freq_scale=20.0, llk_weight=200.0),
}


def get_config(name):
    """A BASELINE config (C1..C5) or a reference run (R1, R2) by name."""
    return CONFIGS[name] if name in CONFIGS else REFERENCE_RUNS[name]


def problem_arrays(cfg):
    """Host arrays (x1, x2, src, bvals, bidx) for a config dict."""
    n, scale = cfg["n"], cfg["scale"]
    if cfg["dim"] == 1:
        u, src = solution_1d(cfg["equation"])
        x = np.linspace(0, 1, num=n) * scale
        xind = np.array([0, n - 1], dtype=np.int32)
        return dict(x1=x, src=src(x), bvals=u(x[xind]), bidx=xind)
    u, src = solution_2d(cfg["equation"], cfg.get("beta"))
    x = np.linspace(0, 1, num=n) * scale
    xm, ym = np.meshgrid(x, x, indexing="ij")
    return dict(x1=x, x2=x.copy(), src=src(xm, ym) * np.ones_like(xm), bvals=boundary_2d(u(xm, ym)))


def make_solver(config, seed=0, device=0, Q=30, lr=0.01, random_u=True, flags=0):
    """A DeviceSolver for a BASELINE config with U ~ 0.1 N(0,1) (seeded), other params at the
    reference init."""
    cfg = get_config(config) if isinstance(config, str) else config
    arr = problem_arrays(cfg)
    eq = cfg["equation"].split("-")[0]
    eq = {"poisson_1d": "poisson", "allencahn_1d": "allencahn", "poisson_2d": "poisson",
          "allencahn_2d": "allencahn", "advection": "advection"}[eq]
    s = DeviceSolver(cfg["dim"], eq, cfg["kernel"], arr["x1"], arr["src"], arr["bvals"],
                     x2=arr.get("x2"), bidx=arr.get("bidx"), Q=Q, llk_weight=cfg["llk_weight"],
                     beta=cfg.get("beta", 1.0), lr=lr, freq_scale=cfg["freq_scale"], device=device,
                     flags=flags)
    if random_u:
        flat = s.get_flat()
        rng = np.random.default_rng(seed)
        if cfg["dim"] == 2:
            nu = cfg["n"] * cfg["n"]
            flat[:nu] = 0.1 * rng.normal(size=nu)
        else:
            flat[3 * Q + 2:] = 0.1 * rng.normal(size=cfg["n"])
        s.set_flat(flat)
    return s
