"""Drop-in mirror of code/model_GP_solver_2d.py: 2D Poisson / Allen-Cahn on a Kronecker grid.

Same class (GP_solver_2d_single), constructor, methods, test()/evals() driver and CLI
(`python -m gpk.model_GP_solver_2d -equation=poisson_2d-sin_sin -kernel=Matern52_Cos_1d
-nepoch=1000`).  The log-joint step runs on the MI355X (libgpk); there is no CPU fallback.
"""
import os
import sys
import time

import numpy as np
import yaml

from . import init_func, replicas, utils
from .cli import parse_flags
from .core import DeviceSolver  # noqa: F401  (re-export for users of the handle)
from .equations import EQUATIONS_2D, boundary_2d, solution_2d
from .infras.exp_config import ExpConfig
from .kernel_matrix import Kernel_matrix, kernel_class
from .solver_common import SolverBase


class GP_solver_2d_single(SolverBase):
    """2D GP solver with a product (Kronecker) kernel (model_GP_solver_2d.py:31-352).

    bvals: boundary values hstack(U[0,:], U[-1,:], U[:,0], U[:,-1]);
    X_col = (x_pos, y_pos); src_vals: N1 x N2; X_test = (x_test, y_test); u_test: M1 x M2."""

    dim = 2
    eq_types = ("poisson_2d", "allencahn_2d")
    early_stop_enabled = True  # 2d.py:327-332 (tol > 0)

    def __init__(self, bvals, X_col, src_vals, jitter, X_test, u_test, trick_paras=None,
                 fix_dict=None):
        self.bvals = np.asarray(bvals, np.float64)
        self.X_col = X_col
        self.jitter = jitter
        self.Nb = self.bvals.size
        self.N1 = np.asarray(X_col[0]).size
        self.N2 = np.asarray(X_col[1]).size
        self.Nc = self.N1 * self.N2
        self.src_vals = np.asarray(src_vals, np.float64)
        self.trick_paras = trick_paras
        self.llk_weight = trick_paras["llk_weight"]
        self.cov_func = trick_paras["kernel"]()
        self.kernel_matrix = Kernel_matrix(self.jitter, self.cov_func)
        self.Xte = X_test
        self.ute = u_test
        self.params = None
        self.pred_func = None
        self.eq_type = trick_paras["equation"].split("-")[0]
        assert self.eq_type in self.eq_types
        print("equation is: ", self.trick_paras["equation"])
        print("kernel is:", self.cov_func.__class__.__name__)
        eq = {"poisson_2d": "poisson", "allencahn_2d": "allencahn", "advection": "advection"}[self.eq_type]
        self._make_device(dim=2, eq=eq, kind=self.cov_func.KIND, x1=X_col[0], x2=X_col[1],
                          src=self.src_vals, bvals=self.bvals, beta=float(trick_paras.get("beta", 1.0)))

    # -- reference methods -------------------------------------------------------------
    def value_and_grad_kernel(self, params, key=None):
        """(K1, K2, K1inv_U, K2inv_Ut, U_xx, U_yy) at params (2d.py:87-121), on the device."""
        self._sync(params)
        f = self.dev.forward_field
        return f("K1"), f("K2"), f("K1inv_U"), f("K2inv_Ut"), f("U_xx"), f("U_yy")

    def boundary_and_eq_gap(self, U, U_xx, U_yy):
        """(boundary_gap, eq_gap) from given fields (2d.py:123-143)."""
        U = np.asarray(U)
        u_b = boundary_2d(U)
        boundary_gap = float(np.sum(np.square(u_b.reshape(-1) - self.bvals.reshape(-1))))
        if self.eq_type == "poisson_2d":
            eq_gap = float(np.sum(np.square(U_xx + U_yy - self.src_vals)))
        elif self.eq_type == "allencahn_2d":
            eq_gap = float(np.sum(np.square(U_xx + U_yy + U * (U ** 2 - 1) - self.src_vals)))
        else:
            raise NotImplementedError
        return boundary_gap, eq_gap

    def preds(self, params):
        """U_pred = Kmn1 K1^{-1} U K2^{-1} Kmn2^T on the test grid (2d.py:185-220)."""
        self._sync(params)
        return self.dev.predict(self.Xte[0], self.Xte[1]), None

    def _err(self, params):
        preds, _ = self.preds(params)
        ute = np.asarray(self.ute)
        return float(np.linalg.norm(preds.reshape(-1) - ute.reshape(-1)) / np.linalg.norm(ute.reshape(-1)))

    def _kernel_lists(self, params, log):
        for ax, suffix in (("kernel_paras_1", "k1"), ("kernel_paras_2", "k2")):
            kp = params[ax]
            log.setdefault("w_list_" + suffix, []).append(np.exp(kp["log-w"]))
            log.setdefault("freq_list_" + suffix, []).append(np.asarray(kp["freq"]))
            log.setdefault("ls_list_" + suffix, []).append(np.exp(kp["log-ls"]))

    def _finish_log(self, log):
        keys = ["loss_list", "err_list", "w_list_k1", "freq_list_k1", "ls_list_k1", "w_list_k2",
                "freq_list_k2", "ls_list_k2", "epoch_list"]
        return {k: log.get(k, []) for k in keys}


# ---------------------------------------------------------------------------------------
# experiment driver (2d.py:355-464)
# ---------------------------------------------------------------------------------------
def get_source_val(u_src, x_pos, y_pos, equation_type=None):
    """Source values on the collocation mesh (2d.py:355-366); u_src is the source function."""
    x_mesh, y_mesh = np.meshgrid(x_pos, y_pos, indexing="ij")
    return u_src(x_mesh, y_mesh) * np.ones_like(x_mesh)


def get_mesh_data(u, M1, M2, scale):
    """(x_coor, y_coor, u_mesh) on linspace(0,1,M)*scale (2d.py:369-374)."""
    x_coor = np.linspace(0, 1, num=M1) * scale
    y_coor = np.linspace(0, 1, num=M2) * scale
    x_mesh, y_mesh = np.meshgrid(x_coor, y_coor, indexing="ij")
    return x_coor, y_coor, u(x_mesh, y_mesh)


def get_boundary_vals(u_mesh):
    return boundary_2d(u_mesh)


SOLVER = GP_solver_2d_single


def test(trick_paras, solver_cls=None, beta=None):
    """Run num_fold trainings of one equation and write result_log (2d.py:382-464)."""
    solver_cls = solver_cls or SOLVER
    u, src = solution_2d(trick_paras["equation"], beta)
    scale = trick_paras["scale"]
    M = 300
    x_pos_test, y_pos_test, u_test_mh = get_mesh_data(u, M, M, scale)
    N = trick_paras["N_col"]
    x_pos_tr, y_pos_tr, u_mh = get_mesh_data(u, N, N, scale)
    bvals = get_boundary_vals(u_mh)
    src_vals = get_source_val(src, x_pos_tr, y_pos_tr).reshape((x_pos_tr.size, y_pos_tr.size))
    X_test = (x_pos_test, y_pos_test)
    X_col = (x_pos_tr, y_pos_tr)
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
        model = solver_cls(bvals, X_col, src_vals, 1e-6, X_test, u_test_mh, trick_paras)
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


def load_config(equation):
    """./config/<equation>.yaml, falling back to the package's copy (2d.py:476-479)."""
    for base in (os.getcwd(), os.path.dirname(os.path.abspath(__file__))):
        p = os.path.join(base, "config", equation + ".yaml")
        if os.path.exists(p):
            with open(p, "r") as f:
                return yaml.safe_load(f)
    raise FileNotFoundError("config/" + equation + ".yaml")


def build_config(args, allowed, extra_suffix=None):
    assert args.equation in allowed
    config = load_config(args.equation)
    config["equation"] = args.equation
    config["init_u_trick"] = init_func.zeros
    config["kernel_extra"] = None
    config["scale"] = 2 * np.pi if config["scale"] == "2pi" else 1.0
    if args.nepoch is not None:
        config["nepoch"] = args.nepoch
    config["kernel"] = kernel_class(args.kernel)
    if getattr(args, "device", None) is not None:
        config["device"] = int(args.device)
    print("equation: %s, kernel: %s, freq_scale: %d" % (config["equation"], config["kernel"].__name__,
                                                        config["freq_scale"]))
    config["other_paras"] = config["other_paras"] + (extra_suffix(config) if extra_suffix else "") + \
        "-Ncol-%d" % config["N_col"]
    return config


def evals(**kwargs):
    """fire entry point (2d.py:467-510)."""
    args = ExpConfig()
    args.parse(kwargs)
    config = build_config(args, EQUATIONS_2D)
    return test(config)


def main(argv=None):
    return evals(**parse_flags(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    main()
