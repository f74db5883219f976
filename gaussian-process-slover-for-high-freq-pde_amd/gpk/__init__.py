"""gpk — MI355X-native (gfx950 HIP) hot path of the GP solver for high-frequency PDEs.

Drop-in surface mirroring the reference (xuangu-fang/Gaussian-Process-Slover-for-High-Freq-PDE):
  gpk.kernel_matrix          Kernel_matrix, SE_Cos_1d, Matern52_Cos_1d, Matern52_1d, SE_1d
  gpk.model_GP_solver_1d     GP_solver_1d_single, test, evals
  gpk.model_GP_solver_1d_extra  GP_solver_1d_extra (two-phase, extra Matern52 GP), test, evals
  gpk.model_GP_solver_2d     GP_solver_2d_single, test, evals
  gpk.model_GP_solver_advection  GP_solver_2d_single_advection, test, evals
Compute runs in libgpk.so (include/gpk.h) through ctypes; there is no CPU fallback.
"""
from .core import DeviceSolver, kernel_matrices, tree_flatten, tree_unflatten  # noqa: F401

__version__ = "0.1.0"
