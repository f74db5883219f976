"""Steps/s of the 3-axis Kronecker solver (gpk_step3) on an n^3 grid, Q = 30 (profiling driver)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np
from oracle import gp_oracle as O
from gpk.model_GP_solver_3d import DeviceSolver3

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
prob = O.setup_3d("poisson_3d-mix_sin", (n, n, n), 2 * np.pi, "Matern52_Cos_1d")
s = DeviceSolver3("poisson", "Matern52_Cos_1d", (prob["x1"], prob["x2"], prob["x3"]), prob["src"],
                  prob["bvals"], Q=30, freq_scale=5.0)
flat = s.get_flat()
flat[:n ** 3] = 0.1 * np.random.default_rng(0).normal(size=n ** 3)
s.set_flat(flat)
s.step(3)
t = time.perf_counter()
losses = s.step(steps)
dt = time.perf_counter() - t
print(f"3-axis {n}^3 Matern52_Cos Q=30: {steps} steps {dt * 1e3 / steps:.3f} ms/step {steps / dt:.1f} it/s "
      f"final loss {losses[-1]:.6e}")
s.close()
