"""Drop-in mirror of code/model_GP_solver_1d.py: 1D Poisson / Allen-Cahn, single GP.

CLI: `python -m gpk.model_GP_solver_1d -equation=poisson_1d-single_sin -kernel=Matern52_Cos_1d`.
"""
import sys
import time

import numpy as np

from . import model_GP_solver_2d as m2d
from . import replicas, utils
from .cli import parse_flags
from .equations import EQUATIONS_1D, solution_1d
from .infras.exp_config import ExpConfig
from .kernel_matrix import Kernel_matrix
from .solver_common import SolverBase


class GP_solver_1d_single(SolverBase):
    """1D GP solver (model_GP_solver_1d.py:31-296).  Xind: indices of the boundary points in
    X_col; y: their values; src_col: source at the collocation points."""

    dim = 1
    early_stop_enabled = False  # commented out in the reference (1d.py:272-276)

    def __init__(self, Xind, y, X_col, src_col, jitter, X_test, Y_test, trick_paras=None,
                 fix_dict=None):
        self.Xind = np.asarray(Xind)
        self.y = np.asarray(y, np.float64)
        self.X_col = np.asarray(X_col, np.float64)
        self.src_col = np.asarray(src_col, np.float64)
        self.jitter = jitter
        self.X_con = self.X_col
        self.N = self.Xind.shape[0]
        self.N_con = self.X_con.shape[0]
        self.trick_paras = trick_paras
        self.llk_weight = trick_paras["llk_weight"]
        self.cov_func = trick_paras["kernel"]()
        self.kernel_matrix = Kernel_matrix(self.jitter, self.cov_func)
        self.Xte = X_test
        self.yte = Y_test
        self.params = None
        self.pred_func = None
        self.eq_type = trick_paras["equation"].split("-")[0]
        assert self.eq_type in ["poisson_1d", "allencahn_1d"]
        print("equation is: ", self.trick_paras["equation"])
        print("kernel is:", self.cov_func.__class__.__name__)
        eq = "poisson" if self.eq_type == "poisson_1d" else "allencahn"
        self._make_device(dim=1, eq=eq, kind=self.cov_func.KIND, x1=self.X_col.reshape(-1),
                          src=self.src_col.reshape(-1), bvals=self.y.reshape(-1),
                          bidx=self.Xind.reshape(-1))

    def value_and_grad_kernel(self, params, key=None):
        """(K, Kinv_u, u_xx) at params (1d.py:80-99), on the device."""
        self._sync(params)
        f = self.dev.forward_field
        return f("K"), f("Kinv_u"), f("u_xx")

    def boundary_and_eq_gap(self, u, u_xx):
        """(boundary_gap, eq_gap) from given fields (1d.py:101-121)."""
        u = np.asarray(u)
        boundary_gap = float(np.sum(np.square(u[self.Xind].reshape(-1) - self.y.reshape(-1))))
        if self.eq_type == "poisson_1d":
            eq_gap = float(np.sum(np.square(np.asarray(u_xx).flatten() - self.src_col.flatten())))
        elif self.eq_type == "allencahn_1d":
            eq_gap = float(np.sum(np.square(np.asarray(u_xx).flatten() + (u * (u ** 2 - 1)).flatten()
                                            - self.src_col.flatten())))
        else:
            raise NotImplementedError
        return boundary_gap, eq_gap

    def preds(self, params, Xte):
        """(Kmn K^{-1} u, K) (1d.py:160-180)."""
        self._sync(params)
        pred = self.dev.predict(np.asarray(Xte).reshape(-1)).reshape(-1, 1)
        return pred, self.dev.forward_field("K")

    def _err(self, params):
        self._sync(params)
        pred = self.dev.predict(np.asarray(self.Xte).reshape(-1))
        yte = np.asarray(self.yte).reshape(-1)
        return float(np.linalg.norm(pred - yte) / np.linalg.norm(yte))

    def _kernel_lists(self, params, log):
        kp = params["kernel_paras"]
        log.setdefault("w_list", []).append(np.exp(kp["log-w"]))
        log.setdefault("freq_list", []).append(np.asarray(kp["freq"]))
        log.setdefault("ls_list", []).append(np.exp(kp["log-ls"]))

    def _finish_log(self, log):
        keys = ["loss_list", "err_list", "w_list", "freq_list", "ls_list", "epoch_list"]
        return {k: log.get(k, []) for k in keys}


def get_source_val(src, x_vec, equation_type=None):
    """Source at the collocation points (1d.py:299-307); src is the source function."""
    return src(np.asarray(x_vec).reshape(-1))


def test(trick_paras):
    """1d.py:310-391."""
    u, src = solution_1d(trick_paras["equation"])
    M = 300
    scale = trick_paras["scale"]
    X_test = np.linspace(0, 1, num=M).reshape(-1, 1) * scale
    Y_test = u(X_test)
    N_col = trick_paras["N_col"]
    X_col = np.linspace(0, 1, num=N_col).reshape(-1, 1) * scale
    Xind = np.array([0, X_col.shape[0] - 1])
    y = np.array([u(X_col[Xind[0]]), u(X_col[Xind[1]])]).reshape(-1)
    src_vals = get_source_val(src, X_col.reshape(-1))
    # folds are independent problems: with WORLD_SIZE > 1 each rank trains its own folds on
    # its own GPU (gpk/replicas.py); results are gathered in fold order
    ctx = replicas.init()
    if ctx.world > 1:
        trick_paras = dict(trick_paras, device=ctx.local)
    results = {}
    start_time = time.time()
    model = None
    for fold in replicas.owned(trick_paras["num_fold"], ctx):
        print("fold %d training" % fold)
        model = GP_solver_1d_single(Xind, y, X_col, src_vals, 1e-6, X_test, Y_test, trick_paras)
        log_dict, early_stopping, min_err = model.train(trick_paras["nepoch"], fold)
        results[fold] = (min_err, early_stopping["epoch"])
        if fold == 0:
            utils.store_model(model, log_dict, trick_paras)
    allres = replicas.gather_by_index(results, trick_paras["num_fold"], ctx)
    err_list = [r[0] for r in allres]
    early_stopping_list = [r[1] for r in allres]
    end_time = time.time()
    err_dict = {"mean": np.mean(err_list), "std": np.std(err_list), "err_list": err_list,
                "stop_epoch_mean": np.mean(early_stopping_list), "used_time": end_time - start_time,
                "avg_time": (end_time - start_time) / trick_paras["num_fold"]}
    if ctx.rank == 0:
        utils.wrirte_log(model, err_dict, trick_paras)
        print("finish writing log ...")
    return err_dict


def evals(**kwargs):
    """fire entry point (1d.py:396-447)."""
    args = ExpConfig()
    args.parse(kwargs)
    config = m2d.build_config(args, EQUATIONS_1D)
    return test(config)


def main(argv=None):
    return evals(**parse_flags(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    main()
