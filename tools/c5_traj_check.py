"""C5: 20 Adam steps with the default refinement (large advection factors: A's forward solve
refined alone) against every solve refined (GPK_FLAG_REFINE_ALL): loss trajectory and final
params, relative (max-abs / max-abs), and each one's ms/step.     python tools/c5_traj_check.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np

from gpk._lib import GPK_FLAG_REFINE_ALL
from gpk.problems import make_solver

out = {}
for tag, flags in (("default", 0), ("refine_all", GPK_FLAG_REFINE_ALL)):
    s = make_solver("C5", seed=0, flags=flags)
    try:
        s.prepare(20)
        t0 = time.perf_counter()
        losses = s.step(20)
        s.sync()
        out[tag] = (np.asarray(losses), s.get_flat(), (time.perf_counter() - t0) / 20 * 1e3)
    finally:
        s.close()
rel = lambda a, b: float(np.max(np.abs(a - b)) / np.max(np.abs(b)))
(la, pa, ta), (lb, pb, tb) = out["default"], out["refine_all"]
print(f"losses rel {rel(la, lb):.2e}  params rel {rel(pa, pb):.2e}  (first loss {la[0]:.6e}, last {la[-1]:.6e})  "
      f"{ta:.2f} vs {tb:.2f} ms/step")
