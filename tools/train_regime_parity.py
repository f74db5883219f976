"""Accuracy of the step in C4's training regime, with and without the refinement GEMMs
(test infrastructure; round 5).

C4's refinement gate (gpk_internal.h REFINE_COND_LB: max_a K00 * max diag K_a^{-1} > LB) opens
during training, and the full graph's refinement stages then cost ~16 us per step.  This tool
measures what they buy at the params training actually reaches:

  --dump OUT.npz   (GPU) run C4's bench solver for 2000 Adam steps (code/model_GP_solver_2d.py:
                   285-332's loop), and at steps 0, 200, 1000, 2000 save the flat params, the
                   gate's bound and cond(K_a) per axis, and the device loss / gradient computed
                   (a) as the step computes them (refined when the gate is open) and (b) with
                   GPK_FLAG_NO_REFINE;
  --check IN.npz   (CPU) evaluate the extended-precision yardstick and the fp64 LU oracle (the
                   reference's algorithm) at each saved params and print every key's distance
                   from the yardstick for (a), (b) and the LU oracle, with the parity bar of
                   tests/test_gpu_accuracy.py (max(1e-10, 4 x LU distance)) -- once on the
                   oracle's K and D and once on the step's own (class-evaluated) K and D, which
                   removes the input perturbation of the two fp64 field evaluations.

usage: python tools/train_regime_parity.py --dump gpurun_out/r5/train_regime.npz
       python tools/train_regime_parity.py --check gpurun_out/r5/train_regime.npz [--json OUT]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np

POINTS = [0, 200, 1000, 2000]


def dump(path):
    from gpk import problems
    from gpk._lib import GPK_FLAG_NO_REFINE
    s = problems.make_solver("C4", seed=0)
    r = problems.make_solver("C4", seed=0, flags=GPK_FLAG_NO_REFINE)
    out = {}
    done = 0
    try:
        for i, target in enumerate(POINTS):
            if target > done:
                s.step(target - done)
                s.sync()
                done = target
            flat = s.get_flat()
            lb, cond = [], []
            for name in ("K1", "K2"):
                K = s.forward_field(name)
                cond.append(np.linalg.cond(K))
                lb.append(K[0, 0] * np.max(np.diag(np.linalg.inv(K))))
            fast, rb = s.graph_mode()
            loss_a, g_a = s.loss_grad()
            for name in ("K1inv_U", "K2inv_Ut", "G_K1", "G_D1", "G_K2", "G_D2", "K1inv", "K2inv",
                         "K1inv_D1t", "K2inv_D2t", "R", "X1", "X2", "S", "Kc1", "Kc2", "D1", "D2"):
                out[f"{i}/f/{name}"] = s.forward_field(name)
            # the device's K and D (gpk_kernel_matrices: bitwise the step's class-gathered ones)
            from gpk.core import kernel_matrices
            from gpk.problems import CONFIGS, problem_arrays
            arr = problem_arrays(CONFIGS["C4"])
            pr = s.get_params()
            for a, xk in ((1, "x1"), (2, "x2")):
                Kd, Dd = kernel_matrices(CONFIGS["C4"]["kernel"], arr[xk], arr[xk], pr[f"kernel_paras_{a}"], 1e-6, 2)
                out[f"{i}/f/K{a}dev"], out[f"{i}/f/D{a}dev"] = Kd, Dd
            r.set_flat(flat)
            loss_b, g_b = r.loss_grad()
            out.update({f"{i}/step": target, f"{i}/flat": flat, f"{i}/gate_lb": np.array(lb),
                        f"{i}/cond": np.array(cond), f"{i}/fast": int(fast), f"{i}/loss_a": loss_a,
                        f"{i}/grad_a": g_a, f"{i}/loss_b": loss_b, f"{i}/grad_b": g_b})
            print(f"C4 step {target:5d}: gate bound {max(lb):.3e} cond(K) {max(cond):.3e} fast graph {fast}",
                  flush=True)
    finally:
        s.close()
        r.close()
    np.savez_compressed(path, npoints=len(POINTS), **out)
    print(f"wrote {path}")


def check(path, out_json=None):
    from oracle import gp_oracle as O
    from tests.helpers import config_problem, rel
    from tools.solve_accuracy import run_mode
    O.set_backend(True)
    prob, params0, _, _ = config_problem("C4")
    z = np.load(path)
    report = []
    for i in range(int(z["npoints"])):
        params = O.unflatten_params(params0, z[f"{i}/flat"])
        ext = run_mode(prob, params, "ext")
        lu = run_mode(prob, params, "lu")
        row = {"step": int(z[f"{i}/step"]), "gate_bound": float(np.max(z[f"{i}/gate_lb"])),
               "cond": float(np.max(z[f"{i}/cond"])), "fast_graph": int(z[f"{i}/fast"])}
        for tag, dev in (("device_refined", (float(z[f"{i}/loss_a"]), z[f"{i}/grad_a"])),
                         ("device_no_refine", (float(z[f"{i}/loss_b"]), z[f"{i}/grad_b"])),
                         ("lu_oracle", None)):
            if dev is None:
                le, ge = lu
            else:
                gd = O.unflatten_params(params, dev[1])
                le, ge = dev[0], {k: O.flatten_params(gd[k]) for k in gd}
            d = {"loss": abs(le - ext[0]) / abs(ext[0])}
            for k in ext[1]:
                d[k] = rel(ge[k], ext[1][k])
            row[tag] = d
        # the same on the DEVICE's K and D (gpk_kernel_matrices): the input perturbation of the
        # two fp64 field evaluations (device libm vs the oracle's C libm; at trained params both are
        # ~275 ulp from a long-double evaluation, and the residual R = D1 A + Bt D2^T - F cancels
        # them against each other) removed, only the solve / product rounding left
        if f"{i}/f/K1dev" in z.files:
            kk = O.kernel_kd
            dev_kd = {}
            for a, pk in ((1, "kernel_paras_1"), (2, "kernel_paras_2")):
                if f"{i}/f/Kc{a}" in z.files:  # the step's own (class-evaluated) K and D
                    dev_kd[id(params[pk])] = (z[f"{i}/f/Kc{a}"], z[f"{i}/f/D{a}"])
                else:
                    dev_kd[id(params[pk])] = (z[f"{i}/f/K{a}dev"], z[f"{i}/f/D{a}dev"])
            O.kernel_kd = lambda kind, x, kp, jitter, dv: dev_kd[id(kp)]
            try:
                ext_d = run_mode(prob, params, "ext")
                lu_d = run_mode(prob, params, "lu")
            finally:
                O.kernel_kd = kk
            for tag, dev in (("device_refined_devKD", (float(z[f"{i}/loss_a"]), z[f"{i}/grad_a"])),
                             ("device_no_refine_devKD", (float(z[f"{i}/loss_b"]), z[f"{i}/grad_b"])),
                             ("lu_oracle_devKD", None)):
                if dev is None:
                    le, ge = lu_d
                else:
                    gd = O.unflatten_params(params, dev[1])
                    le, ge = dev[0], {k: O.flatten_params(gd[k]) for k in gd}
                d = {"loss": abs(le - ext_d[0]) / abs(ext_d[0])}
                for k in ext_d[1]:
                    d[k] = rel(ge[k], ext_d[1][k])
                row[tag] = d
            # the reference algorithm fed the step's K and D, measured against the yardstick on the
            # ORACLE's K and D: how far the field evaluations alone move the answer
            d = {"loss": abs(lu_d[0] - ext[0]) / abs(ext[0])}
            for k in ext[1]:
                d[k] = rel(lu_d[1][k], ext[1][k])
            row["lu_oracle_devKD_vs_oracleKD_yardstick"] = d
            bar_d = {k: max(1e-10, 4 * v) for k, v in row["lu_oracle_devKD"].items()}
            row["bar_devKD"] = bar_d
            row["worst_margin_devKD"] = max(row["device_refined_devKD"][k] / bar_d[k] for k in bar_d)
            row["worst_margin_no_refine_devKD"] = max(row["device_no_refine_devKD"][k] / bar_d[k] for k in bar_d)
        bar = {k: max(1e-10, 4 * v) for k, v in row["lu_oracle"].items()}
        row["bar"] = bar
        row["worst_margin_no_refine"] = max(row["device_no_refine"][k] / bar[k] for k in bar)
        row["worst_margin_refined"] = max(row["device_refined"][k] / bar[k] for k in bar)
        report.append(row)
        print(f"step {row['step']:5d} gate {row['gate_bound']:.3e} cond {row['cond']:.3e}: worst error/bar "
              f"refined {row['worst_margin_refined']:.3f}, no refinement {row['worst_margin_no_refine']:.3f}",
              flush=True)
        for tag in ("device_refined", "device_no_refine", "lu_oracle", "device_refined_devKD",
                    "device_no_refine_devKD", "lu_oracle_devKD", "lu_oracle_devKD_vs_oracleKD_yardstick"):
            if tag in row:
                print(f"   {tag[:26]:26s} " + " ".join(f"{k} {v:.2e}" for k, v in sorted(row[tag].items())), flush=True)
        if "worst_margin_devKD" in row:
            print(f"   on the device's own K, D: worst error/bar {row['worst_margin_devKD']:.3f} "
                  f"(no refinement: {row['worst_margin_no_refine_devKD']:.3f})", flush=True)
    if out_json:
        with open(out_json, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump")
    ap.add_argument("--check")
    ap.add_argument("--json")
    a = ap.parse_args()
    if a.dump:
        dump(a.dump)
    if a.check:
        check(a.check, a.json)
