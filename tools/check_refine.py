"""Diagnostic: GPU vs oracle at ill-conditioned sizes (refinement check) + 20-step Adam trajectory."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from oracle import gp_oracle as O
from tests.helpers import device_solver, rel

O.set_backend(True)


def run(dim, name, n, scale, kind, fs, Q=30, steps=20, **kw):
    if dim == 1:
        prob, Xte, Yte = O.setup_1d(name, n, scale, kind)
        params = O.init_params_1d(n, Q, fs)
        params["u"] = 0.1 * np.random.default_rng(0).normal(size=params["u"].shape)
    else:
        prob, Xte, ute = O.setup_2d(name, n, scale, kind, n_col2=n, m_test=30, **kw)
        params = O.init_params_2d(n, n, Q, fs)
        params["U"] = 0.1 * np.random.default_rng(0).normal(size=(n, n))
    s = device_solver(prob, Q, fs)
    s.set_params(params)
    t = time.time()
    lg, gg = s.loss_grad()
    lo, go = (O.loss_grad_1d if dim == 1 else O.loss_grad_2d)(prob, params)
    print(f"{dim}D {name} n={n}: loss rel {abs(lg - lo) / abs(lo):.2e} grad rel {rel(gg, O.flatten_params(go)):.2e}",
          flush=True)
    opt = O.Adam(0.01)
    st = opt.init(params)
    p = params
    for i in range(steps):
        _, g = (O.loss_grad_1d if dim == 1 else O.loss_grad_2d)(prob, p)
        p, st = opt.update(g, st, p)
    losses = s.step(steps)
    pf = s.get_flat()
    print(f"   after {steps} Adam steps: params rel {rel(pf, O.flatten_params(p)):.2e}  "
          f"({time.time() - t:.1f}s)", flush=True)
    s.close()


if __name__ == "__main__":
    run(2, "advection-multiscale", 400, 1.0, "Matern52_Cos_1d", 40.0, llk_weight=500.0, beta=200.0)
    run(2, "poisson_2d-sin_sin", 256, 2 * np.pi, "Matern52_Cos_1d", 20.0)
    run(1, "poisson_1d-single_sin", 2048, 2 * np.pi, "Matern52_Cos_1d", 20.0, steps=5)
