"""Drop-in mirror of code/model_GP_solver_advection.py: beta*u_x + u_y = f on a space-time
Kronecker grid, first-derivative covariances D_x1_kappa (advection.py:87-121, :123-139).

CLI: `python -m gpk.model_GP_solver_advection -equation=advection-sin -kernel=Matern52_Cos_1d`.
"""
import sys

import numpy as np

from . import model_GP_solver_2d as m2d
from .cli import parse_flags
from .equations import EQUATIONS_ADV, boundary_2d
from .infras.exp_config import ExpConfig


class GP_solver_2d_single_advection(m2d.GP_solver_2d_single):
    """GP_solver_2d_single_advection (advection.py:30-351): eq_type 'advection', beta from
    trick_paras; early stopping is disabled in the reference (:323-328)."""

    eq_types = ("advection",)
    early_stop_enabled = False

    def __init__(self, bvals, X_col, src_vals, jitter, X_test, u_test, trick_paras=None,
                 fix_dict=None):
        self.beta = trick_paras["beta"]
        super().__init__(bvals, X_col, src_vals, jitter, X_test, u_test, trick_paras, fix_dict)

    def value_and_grad_kernel(self, params, key=None):
        """(K1, K2, K1inv_U, K2inv_Ut, U_x, U_y) (advection.py:87-121)."""
        return super().value_and_grad_kernel(params, key)

    def boundary_and_eq_gap(self, U, U_x, U_y):
        U = np.asarray(U)
        u_b = boundary_2d(U)
        boundary_gap = float(np.sum(np.square(u_b.reshape(-1) - self.bvals.reshape(-1))))
        eq_gap = float(np.sum(np.square(self.beta * U_x + U_y - self.src_vals)))
        return boundary_gap, eq_gap


def test(trick_paras):
    return m2d.test(trick_paras, solver_cls=GP_solver_2d_single_advection, beta=trick_paras["beta"])


def evals(**kwargs):
    """fire entry point (advection.py:466-509); other_paras gets '-beta-%d' like the reference."""
    args = ExpConfig()
    args.parse(kwargs)
    config = m2d.build_config(args, EQUATIONS_ADV, extra_suffix=lambda c: "-beta-%d" % c["beta"])
    return test(config)


def main(argv=None):
    return evals(**parse_flags(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    main()
