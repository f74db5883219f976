"""Run K log-joint steps of a BASELINE config on one GPU (profiling driver)."""
import argparse, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np
from gpk.core import DeviceSolver
from gpk import problems

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C4")
ap.add_argument("--steps", type=int, default=50)
ap.add_argument("--flags", type=int, default=0, help="GPK_FLAG_* bits (include/gpk.h)")
a = ap.parse_args()
s = problems.make_solver(a.config, seed=0, flags=a.flags)
s.step(5)
s.sync(); t = time.perf_counter(); s.step(a.steps); s.sync(); dt = time.perf_counter() - t
print(f"{a.config} flags={a.flags}: {a.steps} steps {dt*1e3/a.steps:.3f} ms/step  {a.steps/dt:.1f} it/s")
print(s.profile_stages(10))
