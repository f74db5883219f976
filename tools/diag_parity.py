"""Diagnostic: GPU-vs-oracle and autograd-vs-oracle discrepancy against cond(K)."""
import sys, os, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from oracle import gp_oracle as O
from tests.helpers import device_solver, problem_1d, problem_2d, rel
from tests import autograd_ref as AR
O.set_backend(False)
rows = []
for dim in (1, 2):
    eqs = ["poisson", "allencahn"] + (["advection"] if dim == 2 else [])
    for eq in eqs:
        for kind in ["SE_Cos_1d", "Matern52_Cos_1d", "SE_1d", "Matern52_1d"]:
            if dim == 1:
                prob, params, _ = problem_1d(eq=eq, kind=kind, n=40, Q=5, seed=1); fs = 20.0
                lo, go = O.loss_grad_1d(prob, params); la, ga = AR.loss_grad_1d(prob, params)
                cond = np.linalg.cond(O.kernel_matrix(kind, prob["x"], params["kernel_paras"], 1e-6))
            else:
                prob, params, _, fs = problem_2d(eq=eq, kind=kind, n1=40, n2=36, Q=5, seed=4)
                lo, go = O.loss_grad_2d(prob, params); la, ga = AR.loss_grad_2d(prob, params)
                cond = max(np.linalg.cond(O.kernel_matrix(kind, prob["x1"], params["kernel_paras_1"], 1e-6)),
                           np.linalg.cond(O.kernel_matrix(kind, prob["x2"], params["kernel_paras_2"], 1e-6)))
            s = device_solver(prob, 5, fs); s.set_params(params); l, g = s.loss_grad(); s.close()
            gf, af = O.flatten_params(go), O.flatten_params(ga)
            print(f"{dim}D {eq:9s} {kind:16s} cond {cond:9.2e} | gpu-oracle loss {abs(l-lo)/abs(lo):8.1e} grad {rel(g, gf):8.1e} "
                  f"| autograd-oracle loss {abs(la-lo)/abs(lo):8.1e} grad {rel(af, gf):8.1e} | gpu-autograd grad {rel(g, af):8.1e}", flush=True)
