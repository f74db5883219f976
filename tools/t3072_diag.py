"""T3072 (tests/test_gpu_fullsize.py's 3072^2 advection problem): device loss / gradient against
the exact-field yardstick fixture (tests/golden/ext_T3072.npz) under several path flags, next to
the fp64 LU oracle's own distance.   usage: python tools/t3072_diag.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np

from gpk import _lib
from oracle import gp_oracle as O
from tests.helpers import device_solver, problem_2d
from tests.test_gpu_accuracy import fixture_errors

fx = np.load(os.path.join(ROOT, "tests", "golden", "ext_T3072.npz"))
lu = {f[7:]: float(fx[f]) for f in fx.files if f.startswith("lu_err/")}
lu["loss"] = float(fx["loss_lu_err"])
print("lu_oracle " + " ".join(f"{k} {v:.3e}" for k, v in sorted(lu.items())), flush=True)
prob, params, _, fs = problem_2d(eq="advection", n1=3072, n2=3072, Q=6, seed=3)
for name in ("0", "GPK_FLAG_FORCE_BIG_GEMM", "GPK_FLAG_REFINE_ALL", "GPK_FLAG_NO_DD_CONTRACTION"):
    flags = 0 if name == "0" else getattr(_lib, name)
    s = device_solver(prob, 6, fs, flags=flags)
    s.set_params(params)
    try:
        loss, g = s.loss_grad()
    finally:
        s.close()
    gd = O.unflatten_params(params, g)
    e = fixture_errors(fx, loss, {k: O.flatten_params(gd[k]) for k in gd})
    print(f"{name:28s} " + " ".join(f"{k} {v:.3e} ({v / max(lu[k], 1e-300):.2f}x)" for k, v in sorted(e.items())), flush=True)
