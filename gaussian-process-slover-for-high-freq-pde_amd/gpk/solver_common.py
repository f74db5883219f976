"""Shared machinery of the drop-in solver classes (1D, 2D, advection).

The reference's solvers keep params as a jax pytree and run one jitted `step` per Python
iteration (code/model_GP_solver_2d.py:176-183, :285-332).  Here params and the Adam state
live in HBM inside a libgpk handle; the Python objects handed back by `step` are lazy views
that fetch from the device only when read, so the reference's calling code keeps working:

    params, opt_state, loss = solver.step(params, opt_state, key)
    params['kernel_paras_1']['log-w']        # fetched on access

`train` batches the steps between two evaluation points into a single `gpk_step` call
(one hipGraph replay per step, one host sync per batch).
"""
from collections.abc import Mapping

import numpy as np

from .core import DeviceSolver, tree_flatten, tree_unflatten

try:  # progress bar like the reference (tqdm.tqdm(range(nepoch))), optional
    import tqdm as _tqdm
except Exception:  # pragma: no cover
    _tqdm = None


class LazyParams(Mapping):
    """Read-only view of the device-resident params at one step count."""

    def __init__(self, solver, version):
        self._solver = solver
        self._version = version
        self._cache = None

    def _tree(self):
        if self._cache is None:
            if self._version != self._solver._version:
                raise RuntimeError("stale params view: the solver has stepped since this view was made")
            self._cache = self._solver.dev.get_params()
        return self._cache

    def __getitem__(self, k):
        return self._tree()[k]

    def __iter__(self):
        return iter(self._tree())

    def __len__(self):
        return len(self._tree())

    def to_dict(self):
        return self._tree()


class OptStateToken(object):
    """Opaque stand-in for optax's ScaleByAdamState: the state lives on the device."""

    def __init__(self, solver, version):
        self._solver = solver
        self._version = version

    def fetch(self):
        count, mu, nu = self._solver.dev.get_opt_state()
        t = self._solver.dev.template
        return {"count": count, "mu": tree_unflatten(t, mu), "nu": tree_unflatten(t, nu)}


def record_epochs(nepoch):
    """The epochs i with i % (nepoch / 20) == 0 (Python float semantics, 2d.py:293)."""
    every = nepoch / 20
    return [i for i in range(nepoch) if i % every == 0]


class SolverBase(object):
    dim = None

    # -- device handle ------------------------------------------------------------------
    def _make_device(self, **kw):
        tp = self.trick_paras
        self.dev = DeviceSolver(
            Q=int(tp["Q"]), jitter=self.jitter, llk_weight=float(tp["llk_weight"]),
            logdet=bool(tp.get("logdet", True)), lr=float(tp["lr"]),
            freq_scale=float(tp["freq_scale"]), device=int(tp.get("device", 0)), **kw)
        self._version = 0

    def init_params(self):
        """train()'s initial params (model_GP_solver_2d.py:245-261 / 1d.py:203-213)."""
        Q, fs = int(self.trick_paras["Q"]), float(self.trick_paras["freq_scale"])
        kp = lambda: {"log-w": np.log(1 / Q) * np.ones(Q), "log-ls": np.zeros(Q),
                      "freq": np.linspace(0, 1, Q) * fs}
        if self.dim == 1:
            return {"log_tau": 0.0, "log_v": 0.0, "kernel_paras": kp(), "u": np.zeros((self.N_con, 1))}
        return {"log_tau": 0.0, "log_v": 0.0, "kernel_paras_1": kp(), "kernel_paras_2": kp(),
                "U": np.zeros((self.N1, self.N2))}

    def _sync(self, params, opt_state=None):
        """Make the device hold `params` (and `opt_state`) unless they already are its state."""
        if not (isinstance(params, LazyParams) and params._solver is self and params._version == self._version):
            tree = params.to_dict() if isinstance(params, LazyParams) else params
            self.dev.set_flat(tree_flatten(tree))
            self._version += 1
        if opt_state is None or (isinstance(opt_state, OptStateToken) and opt_state._solver is self):
            return
        if isinstance(opt_state, dict) and "mu" in opt_state:
            self.dev.set_opt_state(int(opt_state["count"]), tree_flatten(opt_state["mu"]),
                                   tree_flatten(opt_state["nu"]))

    def reset_optimizer(self):
        z = np.zeros(self.dev.nparams)
        self.dev.set_opt_state(0, z, z)
        return OptStateToken(self, self._version)

    def current(self):
        return LazyParams(self, self._version)

    # -- reference methods -----------------------------------------------------------------
    def loss(self, params, key=None):
        """-log joint at params (model_GP_solver_2d.py:145-174)."""
        self._sync(params)
        loss, _ = self.dev.loss_grad()
        return loss

    def value_and_grad(self, params, key=None):
        """jax.value_and_grad(self.loss)(params): (loss, grad pytree)."""
        self._sync(params)
        loss, g = self.dev.loss_grad()
        tree = params.to_dict() if isinstance(params, LazyParams) else params
        return loss, tree_unflatten(tree, g)

    def step(self, params, opt_state, key=None):
        """One Adam step on the log joint (model_GP_solver_2d.py:176-183)."""
        self._sync(params, opt_state)
        losses = self.dev.step(1)
        self._version += 1
        return LazyParams(self, self._version), OptStateToken(self, self._version), float(losses[0])

    def steps(self, n):
        """n steps in one device batch; returns the n losses (loss before each update)."""
        if n <= 0:
            return np.zeros(0)
        losses = self.dev.step(n)
        self._version += 1
        return losses

    def compute_early_stopping(self, params, key=None):
        """boundary_gap/Nb + eq_gap/Nc (model_GP_solver_2d.py:222-233)."""
        self._sync(params)
        return self.dev.criterion()

    # -- train loop ----------------------------------------------------------------------------
    def _kernel_lists(self, params, log):
        raise NotImplementedError

    def _err(self, params):
        raise NotImplementedError

    # -- checkpoint / resume (the reference only pickles the final params,
    # code/utils.py:580-597) ---------------------------------------------------------------
    def save_checkpoint(self, path, loop=None):
        """The training state as one NumPy .npz (plain arrays, no pickle): the flat params, the
        Adam count / mu / nu (the device's optimizer state) and, from train(), the loop position
        (epochs done, min error, error-increase count) and every record list."""
        count, mu, nu = self.dev.get_opt_state()
        arrs = {"params": self.dev.get_flat(), "count": np.int64(count), "mu": mu, "nu": nu}
        if loop is not None:
            done, min_err, inc, log = loop[:4]
            stopped = loop[4] if len(loop) > 4 else -1
            arrs.update(done=np.int64(done), min_err=np.float64(min_err), inc=np.int64(inc),
                        early_stop_epoch=np.int64(stopped))
            for k, v in log.items():
                arrs["log_" + k] = np.asarray(v)
        # written to a temporary file in the same directory and renamed onto `path` (exactly that
        # name: a file object keeps np.savez from appending ".npz"): a job killed mid-write leaves
        # the previous checkpoint intact
        import os
        tmp = "%s.tmp.%d" % (path, os.getpid())
        try:
            with open(tmp, "wb") as f:
                np.savez(f, **arrs)
            os.replace(tmp, path)
        finally:
            if os.path.exists(tmp):
                os.remove(tmp)

    def load_checkpoint(self, path):
        """Restore a save_checkpoint() file onto the device; returns the train-loop state or None."""
        with np.load(path, allow_pickle=False) as z:
            self.dev.set_flat(z["params"])
            self._version += 1
            self.dev.set_opt_state(int(z["count"]), z["mu"], z["nu"])
            if "done" not in z:
                return None
            # (per-record arrays stay arrays, scalars Python numbers: as train() appends them)
            log = {k[4:]: [x.copy() if x.ndim else x.item() for x in z[k]] for k in z.files if k.startswith("log_")}
            stopped = int(z["early_stop_epoch"]) if "early_stop_epoch" in z else -1
            return int(z["done"]), float(z["min_err"]), int(z["inc"]), log, stopped

    def train(self, nepoch, seed=0, verbose=True, checkpoint=None, resume=None, stop_at=None, perf_log=None):
        """train() (model_GP_solver_2d.py:235-352): same records, same early-stopping rule.

        Beyond the reference: `checkpoint` (path) saves the training state after every record
        epoch (save_checkpoint), `resume` (path) continues from such a file -- the same records
        and the same device state as the uninterrupted run -- and `stop_at` ends the loop after
        the first record at or past that many epochs (a time-boxed job, resumed later).
        `perf_log` (path) appends one JSON line per record: epoch, loss, error, criterion, and
        the device steps and wall time of the batch before it."""
        import json
        import time
        early_stopping = {"flag": False, "epoch": self.trick_paras["nepoch"]}
        params = self.init_params()
        self._sync(params)
        self.reset_optimizer()
        log = {"loss_list": [], "err_list": [], "epoch_list": []}
        min_err, threshold, error_increase_count = 2.0, 1e-3, 0
        done = 0
        if resume is not None:
            st = self.load_checkpoint(resume)
            if st is None:
                raise ValueError("resume: %s holds no train-loop state" % resume)
            done, min_err, error_increase_count, log, stopped = st
            if stopped >= 0:  # the checkpointed run had stopped early: nothing left to train
                early_stopping = {"flag": True, "epoch": stopped}
                self.params = self.current().to_dict()
                return self._finish_log(log), early_stopping, min_err
        rec = record_epochs(nepoch)
        bar = _tqdm.tqdm(total=nepoch, initial=done, disable=not verbose) if _tqdm is not None else None
        for i in rec + [nepoch]:
            if i < nepoch and i + 1 <= done:
                continue  # (recorded before the checkpoint this run resumed from)
            n = (i + 1 - done) if i < nepoch else (nepoch - done)
            t0 = time.perf_counter()
            losses = self.steps(n)
            self.dev.sync()
            dt = time.perf_counter() - t0
            done += n
            if bar is not None:
                bar.update(n)
            if i >= nepoch:
                break
            loss = float(losses[-1])
            params = self.current()
            err = self._err(params)
            if err < min_err:
                min_err = err
            elif err - min_err > threshold:
                error_increase_count += 1
            if verbose:
                print("loss = %g" % loss)
                print("It ", i, "  loss = %g " % loss, " Relative L2 error", err, " min error", min_err)
            log["loss_list"].append(np.log(loss) if loss > 1 else loss)
            log["err_list"].append(err)
            self._kernel_lists(params, log)
            log["epoch_list"].append(i)
            criterion = self.compute_early_stopping(params)
            if verbose:
                print("criterion = %g" % criterion)
            if perf_log is not None:
                with open(perf_log, "a") as f:
                    f.write(json.dumps({"epoch": i, "loss": loss, "err": float(err), "criterion": float(criterion),
                                        "steps": int(n), "seconds": dt, "steps_per_s": n / dt if dt > 0 else None}) + "\n")
            # the early-stop rule first (the uninterrupted run's order), and its outcome goes into
            # the checkpoint: a run resumed from this record stops exactly where it did
            stop = (self.early_stop_enabled and self.trick_paras.get("tol", -1) > 0
                    and criterion < self.trick_paras["tol"])
            if checkpoint is not None:
                self.save_checkpoint(checkpoint, (done, min_err, error_increase_count, log, i if stop else -1))
            if stop:
                if verbose:
                    print("early stop at epoch %d" % i)
                early_stopping["flag"] = True
                early_stopping["epoch"] = i
                break
            if stop_at is not None and done >= stop_at:
                break
        if bar is not None:
            bar.close()
        if verbose:
            print("finish training ...")
        self.params = self.current().to_dict()
        return self._finish_log(log), early_stopping, min_err

    early_stop_enabled = False

    def _finish_log(self, log):
        return log
