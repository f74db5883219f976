"""C5 (advection 4096^2) loss / gradient against the exact-field yardstick (tests/golden/ext_C5.npz)
with the forward solves refined (default), not refined (GPK_FLAG_NO_REFINE) and all solves refined
(GPK_FLAG_REFINE_ALL), next to the fp64 LU oracle's own distance, and each variant's ms/step.
    python tools/c5_refine_diag.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np

from gpk import _lib
from gpk.problems import make_solver
from oracle import gp_oracle as O
from tests.helpers import config_problem
from tests.test_gpu_accuracy import fixture_errors, fixture_tol

fx = np.load(os.path.join(ROOT, "tests", "golden", "ext_C5.npz"))
prob, params, _, cfg = config_problem("C5")
tol = fixture_tol(fx, "C5")
lu = {f[7:]: float(fx[f]) for f in fx.files if f.startswith("lu_err/")}
lu["loss"] = float(fx["loss_lu_err"])
print("lu  " + " ".join(f"{k} {v:.2e}" for k, v in sorted(lu.items())), flush=True)
print("bar " + " ".join(f"{k} {v:.2e}" for k, v in sorted(tol.items())), flush=True)
for name in (sys.argv[1:] or ["0", "GPK_FLAG_NO_REFINE", "GPK_FLAG_REFINE_ALL"]):
    flags = 0 if name == "0" else getattr(_lib, name)
    s = make_solver("C5", seed=0, flags=flags)
    try:
        loss, g = s.loss_grad()
        s.prepare(3)
        s.step(1)
        s.sync()
        t0 = time.perf_counter()
        s.step(3)
        s.sync()
        ms = (time.perf_counter() - t0) / 3 * 1e3
    finally:
        s.close()
    gd = O.unflatten_params(params, g)
    e = fixture_errors(fx, loss, {k: O.flatten_params(gd[k]) for k in gd})
    worst = max(e[k] / tol[k] for k in e)
    print(f"{name:22s} {ms:6.2f} ms/step  worst/bar {worst:.2f}  " +
          " ".join(f"{k} {v:.2e} ({v / max(lu[k], 1e-300):.2f}x)" for k, v in sorted(e.items())), flush=True)
