"""Drop-in mirror of code/model_GP_solver_1d_extra.py: 1D GP solver with an extra GP.

Two phases (model_GP_solver_1d_extra.py:198-339): the single GP of GP_solver_1d_single is
trained up to `change_point * nepoch`; then its params are frozen and a second ("extra") GP
with kernel `trick_paras['kernel_extra']` (Matern52_1d in the reference's evals, :476) is
trained on the residual: its loss (loss_extra, :101-137) is the 1D negative log-joint of the
extra GP with

    boundary gap  ||u[Xind] + u_e[Xind] - y||^2
    equation gap  ||u_xx + u_xx_e (+ (u+u_e)((u+u_e)^2-1)) - f||^2

where u, u_xx are the frozen first GP's.  On the device this is exactly the 1D step of libgpk on
shifted data -- y' = y - u[Xind], f' = f - u_xx -- plus, for Allen-Cahn, the frozen field u as the
offset of the nonlinear term (gpk_problem.uoff).  Both phases are libgpk handles; predictions
add the two GPs (preds_extra, :148-178).

CLI: `python -m gpk.model_GP_solver_1d_extra -equation=poisson_1d-mix_sin -kernel=Matern52_Cos_1d`.
"""
import copy
import sys
import time

import numpy as np

from . import model_GP_solver_2d as m2d
from . import replicas, utils
from .cli import parse_flags
from .core import DeviceSolver, tree_flatten, tree_unflatten
from .equations import EQUATIONS_1D, solution_1d
from .infras.exp_config import ExpConfig
from .kernel_matrix import Kernel_matrix, Matern52_1d
from .model_GP_solver_1d import GP_solver_1d_single, get_source_val
from .solver_common import record_epochs

try:
    import tqdm as _tqdm
except Exception:  # pragma: no cover
    _tqdm = None


class GP_solver_1d_extra(GP_solver_1d_single):
    """model_GP_solver_1d_extra.py:33-339."""

    def __init__(self, Xind, y, X_col, src_col, jitter, X_test, Y_test, trick_paras=None,
                 fix_dict=None):
        super().__init__(Xind, y, X_col, src_col, jitter, X_test, Y_test, trick_paras, fix_dict)
        self.cov_func_extra = trick_paras["kernel_extra"]()
        self.kernel_matrix_extra = Kernel_matrix(self.jitter, self.cov_func_extra)
        self.params = None
        self.params_extra = None
        self.dev_extra = None
        print("using extra GP with kernel:", self.cov_func_extra.__class__.__name__)

    # -- the extra GP on the device ------------------------------------------------------------
    def _frozen_fields(self, params):
        """(u, u_xx) of the frozen first GP (value_and_grad_kernel, :108)."""
        self._sync(params)
        u = np.asarray(self.dev.get_params()["u"], np.float64).reshape(-1)
        uxx = self.dev.forward_field("u_xx").reshape(-1)
        return u, uxx

    def _make_extra(self, params):
        """Second-phase handle on the shifted data of the frozen first GP at `params`."""
        u0, uxx0 = self._frozen_fields(params)
        self._u0, self._uxx0 = u0, uxx0
        xind = self.Xind.reshape(-1)
        bvals = self.y.reshape(-1) - u0[xind]
        src = self.src_col.reshape(-1) - uxx0
        tp = self.trick_paras
        eq = "poisson" if self.eq_type == "poisson_1d" else "allencahn"
        if self.dev_extra is not None:
            self.dev_extra.close()
        self.dev_extra = DeviceSolver(
            1, eq, self.cov_func_extra.KIND, self.X_col.reshape(-1), src, bvals, bidx=xind, Q=1,
            jitter=self.jitter, llk_weight=float(tp["llk_weight"]), logdet=bool(tp.get("logdet", True)),
            lr=float(tp["lr"]), freq_scale=0.0, device=int(tp.get("device", 0)),
            uoff=u0 if eq == "allencahn" else None)

    @staticmethod
    def _extra_tree(params_extra):
        """The reference's params_extra pytree {log_tau, log_v, kernel_paras{log-w, log-ls}, u}
        in the device layout (an unused 'freq' leaf: the extra kernel has no cosine)."""
        kp = params_extra["kernel_paras"]
        return {"kernel_paras": {"freq": np.zeros(1), "log-ls": np.asarray(kp["log-ls"], np.float64).reshape(1),
                                 "log-w": np.asarray(kp["log-w"], np.float64).reshape(1)},
                "log_tau": float(params_extra["log_tau"]), "log_v": float(params_extra["log_v"]),
                "u": np.asarray(params_extra["u"], np.float64).sum(axis=1).reshape(-1, 1)
                if np.ndim(params_extra["u"]) == 2 else np.asarray(params_extra["u"]).reshape(-1, 1)}

    def _set_extra(self, params_extra):
        self.dev_extra.set_flat(tree_flatten(self._extra_tree(params_extra)))

    def _get_extra(self):
        t = tree_unflatten(self.dev_extra.template, self.dev_extra.get_flat())
        return {"log_tau": t["log_tau"], "log_v": t["log_v"],
                "kernel_paras": {"log-w": t["kernel_paras"]["log-w"], "log-ls": t["kernel_paras"]["log-ls"]},
                "u": t["u"]}

    def value_and_grad_kernel_extra(self, params_extra, key=None):
        """(K_extra, Kinv_u_extra, u_xx_extra) (:57-77), on the device."""
        self._set_extra(params_extra)
        f = self.dev_extra.forward_field
        return f("K"), f("Kinv_u"), f("u_xx")

    def boundary_and_eq_gap_extra(self, u, u_extra, u_xx, u_xx_extra):
        """(boundary_gap, eq_gap) of the sum of the two GPs (:79-99)."""
        u = np.asarray(u).reshape(-1, 1)
        u_extra = np.asarray(u_extra).reshape(-1, 1)
        boundary_gap = float(np.sum(np.square(u[self.Xind].reshape(-1) + u_extra[self.Xind].reshape(-1)
                                              - self.y.reshape(-1))))
        if self.eq_type == "poisson_1d":
            eq_gap = float(np.sum(np.square(np.asarray(u_xx).flatten() + np.asarray(u_xx_extra).flatten()
                                            - self.src_col.flatten())))
        elif self.eq_type == "allencahn_1d":
            us = u + u_extra
            eq_gap = float(np.sum(np.square(np.asarray(u_xx).flatten() + np.asarray(u_xx_extra).flatten()
                                            + (us * (us ** 2 - 1)).flatten() - self.src_col.flatten())))
        else:
            raise NotImplementedError
        return boundary_gap, eq_gap

    def loss_extra(self, params_extra, key=None):
        """-log joint of the extra GP with the first GP frozen (:101-137)."""
        self._set_extra(params_extra)
        loss, _ = self.dev_extra.loss_grad()
        return loss

    def value_and_grad_extra(self, params_extra, key=None):
        """jax.value_and_grad(loss_extra)(params_extra) in the reference's pytree."""
        self._set_extra(params_extra)
        loss, g = self.dev_extra.loss_grad()
        t = tree_unflatten(self.dev_extra.template, g)
        return loss, {"log_tau": t["log_tau"], "log_v": t["log_v"],
                      "kernel_paras": {"log-w": t["kernel_paras"]["log-w"], "log-ls": t["kernel_paras"]["log-ls"]},
                      "u": t["u"]}

    def step_extra(self, params_extra, opt_state, key=None):
        """One Adam step of the extra GP (:139-146).  opt_state: None (fresh) or the device's."""
        if params_extra is not None:
            self._set_extra(params_extra)
        if opt_state is None:
            z = np.zeros(self.dev_extra.nparams)
            self.dev_extra.set_opt_state(0, z, z)
        loss = float(self.dev_extra.step(1)[0])
        return self._get_extra(), "device", loss

    def preds_extra(self, params_extra, Xte):
        """preds of the frozen first GP + Kmn_e K_e^{-1} u_e (:148-178)."""
        preds, _ = self.preds(self.params, Xte)
        if params_extra is self._EXTRA_ON_DEVICE:
            pe = self.dev_extra.predict(np.asarray(Xte).reshape(-1))
        else:
            # any params pytree with kernel_paras{log-w, log-ls} and u, through the extra kernel
            # (train() calls this once with the first GP's params at i == change_point)
            kp = params_extra["kernel_paras"]
            q = int(np.size(kp["log-w"]))
            tmp = DeviceSolver(1, "poisson", self.cov_func_extra.KIND, self.X_col.reshape(-1),
                               np.zeros(self.N_con), np.zeros(self.N), bidx=self.Xind.reshape(-1), Q=q,
                               jitter=self.jitter, device=int(self.trick_paras.get("device", 0)))
            try:
                t = tmp.get_params()
                t["kernel_paras"]["log-w"] = np.asarray(kp["log-w"], np.float64).reshape(q)
                t["kernel_paras"]["log-ls"] = np.asarray(kp["log-ls"], np.float64).reshape(q)
                t["u"] = np.asarray(params_extra["u"], np.float64).sum(axis=1).reshape(-1, 1) \
                    if np.ndim(params_extra["u"]) == 2 else np.asarray(params_extra["u"]).reshape(-1, 1)
                tmp.set_params(t)
                pe = tmp.predict(np.asarray(Xte).reshape(-1))
            finally:
                tmp.close()
        return preds + np.asarray(pe).reshape(-1, 1), None

    _EXTRA_ON_DEVICE = object()  # sentinel: "the extra GP's current device params"

    def compute_early_stopping_extra(self, params_extra, key=None):
        """boundary_gap/N + eq_gap/N_con of the two GPs together (:180-193)."""
        self._set_extra(params_extra)
        return self.dev_extra.criterion()

    # -- train (:195-339) ----------------------------------------------------------------------
    def train(self, nepoch, seed=0, verbose=True):
        early_stopping = {"flag": False, "epoch": self.trick_paras["nepoch"]}
        error_increase_count = 0
        params = self.init_params()
        self._sync(params)
        self.reset_optimizer()
        loss_list, err_list, w_list, freq_list, ls_list, epoch_list = [], [], [], [], [], []
        min_err, threshold = 2.0, 1e-3
        change_point = int(nepoch * self.trick_paras["change_point"])
        rec = set(record_epochs(nepoch))
        events = sorted(rec | ({change_point} if change_point < nepoch else set()))
        bar = _tqdm.tqdm(total=nepoch, disable=not verbose) if _tqdm is not None else None
        pred_is_extra = False
        frozen = None
        done = 0
        for i in events + [nepoch]:
            last = min(i, nepoch - 1)
            n = last - done + 1
            if n > 0:
                # an event list holds change_point, so no batch straddles the two phases
                if done <= change_point:
                    losses = self.steps(n)
                else:
                    losses = self.dev_extra.step(n)
                done += n
                if bar is not None:
                    bar.update(n)
                loss = float(losses[-1])
            if i >= nepoch:
                break
            if i == change_point:
                if verbose:
                    print("start to train the extra matern kernel")
                frozen = self.current().to_dict()
                self.params = copy.deepcopy(frozen)
                self._make_extra(frozen)
                init_extra = {"log_tau": copy.deepcopy(frozen["log_tau"]), "log_v": 0.0,
                              "kernel_paras": {"log-w": np.zeros(1), "log-ls": np.zeros(1)},
                              "u": np.zeros((self.N_con, 1))}
                self._set_extra(init_extra)
                z = np.zeros(self.dev_extra.nparams)
                self.dev_extra.set_opt_state(0, z, z)
                pred_is_extra = True
            if i not in rec:
                continue
            params = frozen if frozen is not None else self.current().to_dict()
            if i <= change_point:
                cur = params
            else:
                cur = self._EXTRA_ON_DEVICE
            if pred_is_extra:
                # at i == change_point the reference calls preds_extra with the first GP's params
                preds, _ = self.preds_extra(cur, self.Xte)
            else:
                preds, _ = self.preds(cur, self.Xte)
            yte = np.asarray(self.yte).reshape(-1)
            err = float(np.linalg.norm(np.asarray(preds).reshape(-1) - yte) / np.linalg.norm(yte))
            if err < min_err:
                min_err = err
            elif err - min_err > threshold:
                error_increase_count += 1
            if verbose:
                print("loss = %g" % loss)
                print("It ", i, "  loss = %g " % loss, " Relative L2 error", err, " min error", min_err)
            loss_list.append(np.log(loss) if loss > 1 else loss)
            err_list.append(err)
            w_list.append(np.exp(params["kernel_paras"]["log-w"]))
            freq_list.append(params["kernel_paras"]["freq"])
            ls_list.append(np.exp(params["kernel_paras"]["log-ls"]))
            epoch_list.append(i)
            # the reference evaluates the FIRST GP's criterion here in both phases (:300)
            criterion = self.compute_early_stopping(params)
            if verbose:
                print("criterion = %g" % criterion)
            if i > 0 and (criterion < self.trick_paras["tol"] or error_increase_count > 7):
                if verbose:
                    print("early stop at epoch %d" % (i))
                early_stopping["flag"] = True
                early_stopping["epoch"] = i
                break
        if bar is not None:
            bar.close()
        log_dict = {"loss_list": loss_list, "err_list": err_list, "w_list": w_list,
                    "freq_list": freq_list, "ls_list": ls_list, "epoch_list": epoch_list}
        if verbose:
            print("finish training ...")
        self.params_extra = copy.deepcopy(self._get_extra()) if self.dev_extra is not None else None
        return log_dict, early_stopping, min_err

    def close(self):
        if self.dev_extra is not None:
            self.dev_extra.close()
            self.dev_extra = None


def test(trick_paras):
    """model_GP_solver_1d_extra.py:353-436."""
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
    ctx = replicas.init()
    if ctx.world > 1:
        trick_paras = dict(trick_paras, device=ctx.local)
    results = {}
    start_time = time.time()
    model = None
    for fold in replicas.owned(trick_paras["num_fold"], ctx):
        print("fold %d training" % fold)
        model = GP_solver_1d_extra(Xind, y, X_col, src_vals, 1e-6, X_test, Y_test, trick_paras)
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


def build_config(args):
    """evals() of model_GP_solver_1d_extra.py:439-494: same config, kernel_extra = Matern52_1d,
    other_paras + '-Ncol-<N>change_point-<cp>-extra-GP'."""
    assert args.equation in EQUATIONS_1D
    config = m2d.load_config(args.equation)
    config["equation"] = args.equation
    from . import init_func
    config["init_u_trick"] = init_func.zeros
    config["kernel_extra"] = Matern52_1d
    config["scale"] = 2 * np.pi if config["scale"] == "2pi" else 1.0
    if args.nepoch is not None:
        config["nepoch"] = args.nepoch
    config["kernel"] = m2d.kernel_class(args.kernel)
    if getattr(args, "device", None) is not None:
        config["device"] = int(args.device)
    print("equation: %s, kernel: %s, freq_scale: %d" % (config["equation"], config["kernel"].__name__,
                                                        config["freq_scale"]))
    config["other_paras"] = config["other_paras"] + "-Ncol-%d" % config["N_col"] + \
        "change_point-%.1f" % config["change_point"] + "-extra-GP"
    return config


def evals(**kwargs):
    args = ExpConfig()
    args.parse(kwargs)
    return test(build_config(args))


def main(argv=None):
    return evals(**parse_flags(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    main()
