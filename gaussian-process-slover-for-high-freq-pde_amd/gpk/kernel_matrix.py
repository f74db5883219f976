"""Drop-in mirror of the reference's kernel layer (code/kernel_matrix.py).

Same class names, constructor arguments and method names; every evaluation runs on the
MI355X through libgpk (`gpk_kernel_pairs`, closed-form fields instead of nested jax.grad).
Inputs may be scalars or arrays of pairs (the reference vmaps these methods over pairs,
code/kernel_matrix.py:26, code/model_GP_solver_2d.py:107-117).  `paras` is the reference's
dict of length-Q arrays {'log-w', 'log-ls', 'freq'}.
"""
import numpy as np

from .core import kernel_pairs


class Kernel_matrix(object):
    """Kernel_matrix(jitter, K_u) -- code/kernel_matrix.py:12-30."""

    def __init__(self, jitter, K_u):
        self.jitter = jitter
        self.K_u = K_u  # a Kernel_1d instance

    def get_kernel_matrix(self, X1, X2, paras):
        """vmap(kappa)(X1.flatten(), X2.flatten()).reshape(N, N) + jitter*I (:21-30).

        As in the reference, X1/X2 hold N^2 flattened (meshgrid) pairs and N = sqrt(size)."""
        N = int((np.asarray(X1).size) ** 0.5)
        K = self.K_u.kappa(np.asarray(X1).reshape(-1), np.asarray(X2).reshape(-1), paras)
        return K.reshape(N, N) + self.jitter * np.eye(N)


class Kernel_1d(object):
    """Base class: kappa and its x1-derivatives (code/kernel_matrix.py:35-82)."""

    KIND = None

    def __init__(self, fix_dict=None, fix_paras=None):
        # kept for signature compatibility; the reference's freezing is dead code (:84-104)
        self.fix_dict = fix_dict
        self.fix_paras = fix_paras

    def _eval(self, x1, y1, paras, deriv):
        if self.KIND is None:
            raise NotImplementedError
        x1a, y1a = np.broadcast_arrays(np.asarray(x1, np.float64), np.asarray(y1, np.float64))
        out = kernel_pairs(self.KIND, x1a, y1a, paras, deriv)
        return out.reshape(x1a.shape) if x1a.shape else float(out[0])

    def kappa(self, x1, y1, paras):
        return self._eval(x1, y1, paras, 0)

    def D_x1_kappa(self, x1, y1, paras):
        """cov(f'(x1), f(y1)) = grad(kappa, 0) (:49-52); abs'(0) = +1 as in JAX."""
        return self._eval(x1, y1, paras, 1)

    def DD_x1_kappa(self, x1, y1, paras):
        """cov(f''(x1), f(y1)) = grad(grad(kappa, 0), 0) (:54-57)."""
        return self._eval(x1, y1, paras, 2)


class SE_Cos_1d(Kernel_1d):
    """sum_q w_q exp(-d^2 e^{log-ls_q}) cos(2 pi f_q d)  (GP-HM-GM, :107-128)."""
    KIND = "SE_Cos_1d"


class Matern52_Cos_1d(Kernel_1d):
    """sum_q w_q Matern52(sqrt5 d e^{log-ls_q}) cos(2 pi f_q d)  (GP-HM-StM, :131-155)."""
    KIND = "Matern52_Cos_1d"


class Matern52_1d(Kernel_1d):
    """sum_q w_q Matern52(sqrt5 d e^{log-ls_q})  (GP-Matern, :158-176)."""
    KIND = "Matern52_1d"


class SE_1d(Kernel_1d):
    """sum_q w_q exp(-d^2 e^{log-ls_q})  (GP-SE, :179-193)."""
    KIND = "SE_1d"


KERNELS = {"Matern52_Cos_1d": Matern52_Cos_1d, "SE_Cos_1d": SE_Cos_1d,
           "Matern52_1d": Matern52_1d, "SE_1d": SE_1d}


def kernel_class(name):
    """The reference's kernel-name dispatch (model_GP_solver_2d.py:493-502)."""
    if name not in KERNELS:
        raise Exception('Invalid Kernel')
    return KERNELS[name]
