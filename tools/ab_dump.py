"""Dump loss, gradient, a 2-step trajectory and predictions of a config with the library that
GPK_LIB_PATH selects (A/B bitwise checks between two builds).

    GPK_LIB_PATH=... python tools/ab_dump.py --config C5 --out gpurun_out/a.npz
"""
import argparse, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np
from gpk import problems

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C5")
ap.add_argument("--out", required=True)
ap.add_argument("--flags", type=int, default=0)
a = ap.parse_args()
s = problems.make_solver(a.config, seed=0, flags=a.flags)
try:
    loss, g = s.loss_grad()
    losses = s.step(2)
    s.sync()
    np.savez(a.out, loss=loss, grad=g, losses=losses, flat=s.get_flat())
finally:
    s.close()
