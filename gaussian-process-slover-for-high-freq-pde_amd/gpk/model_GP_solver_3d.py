"""3-axis Kronecker GP solver: the d > 2 generalisation of code/model_GP_solver_2d.py
(the reference itself stops at two axes).

Same log joint as GP_solver_2d_single (model_GP_solver_2d.py:87-183) with K = K1 (x) K2 (x) K3 on
a tensor grid: prior -1/2 c sum_k (prod_{j != k} N_j) logdet K_k - 1/2 <U, K^{-1} U> (the 2-axis
log-det weights :157-162), residual sum_k (D_k K_k^{-1}) x_k U - F [+ U(U^2-1)], boundary on the
six faces.  The whole step (assembly, SPD inverses, mode-k products, adjoints, Adam) runs on the
MI355X through gpk_create3 / gpk_step3 (include/gpk.h); there is no CPU fallback.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, dptr, f64
from .core import tree_flatten, tree_unflatten


def params_template_3d(n1, n2, n3, Q):
    kp = lambda: {"freq": np.zeros(Q), "log-ls": np.zeros(Q), "log-w": np.zeros(Q)}
    return {"U": np.zeros((n1, n2, n3)), "kernel_paras_1": kp(), "kernel_paras_2": kp(),
            "kernel_paras_3": kp(), "log_tau": 0.0, "log_v": 0.0}


def boundary_3d(U):
    """The six faces U[0], U[-1], U[:,0], U[:,-1], U[:,:,0], U[:,:,-1] (each row-major)."""
    U = np.asarray(U)
    return np.concatenate([U[0].ravel(), U[-1].ravel(), U[:, 0].ravel(), U[:, -1].ravel(),
                           U[:, :, 0].ravel(), U[:, :, -1].ravel()])


class DeviceSolver3:
    """One gpk_handle3: problem, params and Adam state resident on the device."""

    def __init__(self, eq, kind, xs, src, bvals, Q=30, jitter=1e-6, llk_weight=200.0, logdet=True,
                 lr=0.01, freq_scale=20.0, device=0, b1=0.9, b2=0.999, eps=1e-8):
        lib = _lib.load()
        if len(xs) != 3:
            raise ValueError("three coordinate axes")
        self._x = [f64(x).reshape(-1) for x in xs]
        self.ns = tuple(x.size for x in self._x)
        self._src = f64(src).reshape(-1)
        self._bvals = f64(bvals).reshape(-1)
        n1, n2, n3 = self.ns
        if self._src.size != n1 * n2 * n3:
            raise ValueError("src must have n1*n2*n3 entries")
        if self._bvals.size != 2 * (n2 * n3 + n1 * n3 + n1 * n2):
            raise ValueError("bvals must be the six faces of U (boundary_3d)")
        p = _lib.gpk_problem3()
        p.eq = _lib.EQ_IDS[eq]
        p.kind = _lib.KIND_IDS[kind] if isinstance(kind, str) else int(kind)
        p.n1, p.n2, p.n3, p.q = n1, n2, n3, int(Q)
        p.x1, p.x2, p.x3 = (dptr(x) for x in self._x)
        p.src, p.bvals = dptr(self._src), dptr(self._bvals)
        p.jitter, p.llk_weight, p.logdet = jitter, llk_weight, float(logdet)
        p.lr, p.b1, p.b2, p.eps = lr, b1, b2, eps
        p.device, p.flags = device, 0
        self._prob = p
        h = ctypes.c_void_p()
        check(lib.gpk_create3(ctypes.byref(p), float(freq_scale), ctypes.byref(h)))
        self._h = h
        n = ctypes.c_int64()
        check(lib.gpk_num_params3(h, ctypes.byref(n)))
        self.nparams = n.value
        self.Q = int(Q)
        self.template = params_template_3d(n1, n2, n3, self.Q)

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().gpk_destroy3(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def get_flat(self):
        out = np.empty(self.nparams)
        check(_lib.load().gpk_get_params3(self._h, dptr(out), self.nparams))
        return out

    def set_flat(self, flat):
        flat = f64(flat).reshape(-1)
        check(_lib.load().gpk_set_params3(self._h, dptr(flat), flat.size))

    def get_params(self):
        return tree_unflatten(self.template, self.get_flat())

    def set_params(self, params):
        self.set_flat(tree_flatten(params))

    def loss_grad(self):
        loss = ctypes.c_double()
        g = np.empty(self.nparams)
        check(_lib.load().gpk_loss_grad3(self._h, ctypes.byref(loss), dptr(g)))
        return loss.value, g

    def step(self, n=1):
        out = np.empty(max(int(n), 1))
        check(_lib.load().gpk_step3(self._h, int(n), dptr(out)))
        return out[:n]


class GP_solver_3d_single:
    """GP_solver_2d_single's interface (model_GP_solver_2d.py:40-48, :176-183) on three axes.

    bvals: boundary_3d(U) of the solution; X_col = (x, y, z); src_vals: N1 x N2 x N3;
    trick_paras: {'kernel': class, 'equation': 'poisson_3d-...' | 'allencahn_3d-...',
    'llk_weight', 'logdet', 'lr', 'Q', 'freq_scale'}."""

    eq_types = ("poisson_3d", "allencahn_3d")

    def __init__(self, bvals, X_col, src_vals, jitter, trick_paras, device=0):
        self.eq_type = trick_paras["equation"].split("-")[0]
        assert self.eq_type in self.eq_types
        self.cov_func = trick_paras["kernel"]()
        self.trick_paras = trick_paras
        eq = {"poisson_3d": "poisson", "allencahn_3d": "allencahn"}[self.eq_type]
        self.dev = DeviceSolver3(eq, self.cov_func.KIND, X_col, src_vals, bvals,
                                 Q=trick_paras.get("Q", 30), jitter=jitter,
                                 llk_weight=trick_paras["llk_weight"],
                                 logdet=trick_paras.get("logdet", True), lr=trick_paras.get("lr", 0.01),
                                 freq_scale=trick_paras.get("freq_scale", 20.0), device=device)

    @property
    def params(self):
        return self.dev.get_params()

    def loss(self, params):
        """Negative log joint at params (model_GP_solver_2d.py:145-174 on three axes)."""
        self.dev.set_params(params)
        return self.dev.loss_grad()[0]

    def value_and_grad(self, params):
        self.dev.set_params(params)
        loss, g = self.dev.loss_grad()
        return loss, tree_unflatten(self.dev.template, g)

    def step(self, n=1):
        """n Adam steps (step(), model_GP_solver_2d.py:176-183); the per-step losses."""
        return self.dev.step(n)
