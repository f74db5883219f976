"""Where does the device's distance from the exact log-joint gradient come from?  (GPU box)

For a BASELINE config at its seeded bench params:
  * the device's K / D (the step's own K via gpk_forward_field, D via gpk_kernel_matrices)
    against the oracle's, in ulps;
  * device gradient vs the long-double yardstick on the ORACLE's K (tests/golden/ext_<cfg>.npz:
    what the parity tests assert) and vs the yardstick on the DEVICE's own K and D (the device
    algorithm's rounding alone, the input perturbation removed);
  * the fp64 LU oracle on the device's K vs that same yardstick (the reference algorithm's own
    rounding on identical inputs).
Prints one JSON line.   usage: python tools/gpu_accuracy_diag.py C2 [--flags N]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np

from oracle import gp_oracle as O
from tests.helpers import config_problem, rel
import tools.solve_accuracy as SA


def ulps(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    sp = np.spacing(np.maximum(np.abs(a), np.abs(b)))
    d = np.abs(a - b) / sp
    return {"max_ulp": float(np.max(d)), "mean_ulp": float(np.mean(d)),
            "max_rel": float(np.max(np.abs(a - b)) / np.max(np.abs(b)))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--quick", action="store_true", help="fixture comparison only (no yardstick on the device's K)")
    a = ap.parse_args()
    from gpk.core import kernel_matrices
    from gpk.problems import make_solver
    O.set_backend(True)
    cid = a.config
    prob, params, _, cfg = config_problem(cid)
    s = make_solver(cid, seed=0, flags=a.flags)
    try:
        assert np.array_equal(s.get_flat(), O.flatten_params(params))
        loss, g = s.loss_grad()
        Kdev = [s.forward_field("K")] if cfg["dim"] == 1 else [s.forward_field("K1"), s.forward_field("K2")]
        path = s.inverse_path()
    finally:
        s.close()
    gd = O.unflatten_params(params, g)
    gdev = {k: O.flatten_params(gd[k]) for k in gd}
    deriv = 1 if prob["eq"] == "advection" else 2
    axes = [("x", "kernel_paras")] if cfg["dim"] == 1 else [("x1", "kernel_paras_1"), ("x2", "kernel_paras_2")]
    dev_kd, kstats = {}, []
    for i, (xk, pk) in enumerate(axes):
        Ko, Do = O.kernel_kd(prob["kind"], prob[xk], params[pk], prob["jitter"], deriv)
        Kk, Dk = kernel_matrices(prob["kind"], prob[xk], prob[xk], params[pk], prob["jitter"], deriv)
        kstats.append({"K_step_vs_oracle": ulps(Kdev[i], Ko), "K_matrices_vs_step": ulps(Kk, Kdev[i]),
                       "D_vs_oracle": ulps(Dk, Do)})
        dev_kd[id(params[pk])] = (Kdev[i], Dk)   # keyed by the axis' parameter dict (loss_grad_* pass it through)
    out = {"config": cid, "path": path, "flags": a.flags, "kd": kstats}
    # yardstick on the oracle's inputs: the committed fixture
    fx = np.load(os.path.join(ROOT, "tests", "golden", f"ext_{cid}.npz"))
    fe = {}
    for k in gdev:
        v = gdev[k] if f"sample/{k}" not in fx else gdev[k][fx[f"sample/{k}"]]
        fe[k] = float(np.max(np.abs(v - fx[f"ext/{k}"])) / fx[f"maxabs/{k}"])
    fe["loss"] = abs(loss - float(fx["loss_ext"])) / abs(float(fx["loss_ext"]))
    out["dev_vs_ext_oracleK"] = fe
    out["lu_vs_ext_oracleK"] = {k[7:]: float(fx[k]) for k in fx.files if k.startswith("lu_err/")}
    if a.quick:
        print(json.dumps(out), flush=True)
        return
    # yardstick and LU on the device's own K and D
    kkd = O.kernel_kd

    def dev_kernel_kd(kind, x, kp, jitter, dv):
        return dev_kd[id(kp)]
    O.kernel_kd = dev_kernel_kd
    try:
        t = time.time()
        ext = SA.run_mode(prob, params, "ext")
        lu = SA.run_mode(prob, params, "lu")
        out["ext_seconds"] = time.time() - t
    finally:
        O.kernel_kd = kkd
    out["dev_vs_ext_devK"] = SA.distances((loss, gdev), ext)
    out["lu_vs_ext_devK"] = SA.distances(lu, ext)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
