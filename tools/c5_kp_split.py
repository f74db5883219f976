"""Where does C5's kernel_paras_2 error come from?  (test infrastructure; GPU box, ~5 min CPU)

VERDICT r4 item 2.  On the step's own K and D (gpk_forward_field Kc / D), the long-double
yardstick is run with its gradient contraction captured, which gives the exact-solve G_K2 and
G_D2 (oracle/gp_oracle.py loss_grad_2d: G_K2 = c N1/2 K2^{-1} - (S/2 + v X2)^T Bt, G_D2 =
v R^T Bt) and K2^{-1}.  The device's G_K2, G_D2, K2^{-1} (fields 8, 9, 11) differ from them; the
contraction is linear, so kernel_paras_2's error splits exactly into
  logdet : c N1/2 (K2^{-1}_dev - K2^{-1}_ext)            (the explicit inverse)
  quad   : the rest of G_K2_dev - G_K2_ext                ((S/2 + v X2)^T Bt)
  gd     : G_D2_dev - G_D2_ext
each reported as max-abs / max-abs of the yardstick's kernel_paras_2 (tests/helpers.rel), next to
the same split of the fp64 LU oracle (the reference algorithm) on the same K and D.

"contraction" separates the contraction's own rounding from the G matrices': each G is contracted
exactly (class sums over the distinct pair distances and the derivative fields in long double, the
reference's fp64 constants and exp(log-ls)), and the device gradient, the fp64 oracle contraction
(oracle/gp_oracle.py param_grad_contract) and the yardstick's own fp64 contraction are each
measured against the exact contraction of the G they contracted.
usage: python tools/c5_kp_split.py [C5] [2]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np

from oracle import gp_oracle as O
from tests.helpers import config_problem
import tools.solve_accuracy as SA


def contract_ld(kind, x, kp, GK, GD, deriv, sums64=False, fields64=False):
    """Exact (long-double) contraction of GK, GD with the derivative fields of kernel kind
    (oracle/gp_oracle.py param_grad_contract's formulas), summed per distinct pair distance."""
    k = O._kind_id(kind)
    x = np.asarray(x, np.float64)
    diff = x[:, None] - x[None, :]
    d = np.abs(diff).ravel()
    du, inv = np.unique(d, return_inverse=True)
    order = np.argsort(inv, kind="stable")
    starts = np.searchsorted(inv[order], np.arange(du.size))
    ld = np.longdouble
    sdt = np.float64 if sums64 else ld  # sums64 / fields64: that half in fp64 (diagnostics)
    SK = np.add.reduceat(GK.ravel()[order].astype(sdt), starts).astype(ld)
    SD = None
    if GD is not None:
        g = GD.ravel() * (np.where(diff >= 0.0, 1.0, -1.0).ravel() if deriv == 1 else 1.0)
        SD = np.add.reduceat(g[order].astype(sdt), starts).astype(ld)
    fdt = np.float64 if fields64 else ld
    w = np.exp(np.asarray(kp["log-w"], np.float64)).astype(ld)
    a = np.exp(np.asarray(kp["log-ls"], np.float64)).astype(fdt)
    f = np.asarray(kp["freq"], np.float64).astype(fdt)
    dd = du.astype(fdt)[:, None]
    m0, m1, m2, m0l, m1l, m2l = (v.astype(ld) for v in O._radial(k, dd, a, True))
    c0, c1, c2, c0f, c1f, c2f = (np.asarray(v).astype(ld) for v in O._cosine(k, dd, f, True))
    gw, gl, gf = SK @ (m0 * c0), SK @ (m0l * c0), SK @ (m0 * c0f)
    if SD is not None:
        if deriv == 2:
            Dw, Dl, Df = m2 * c0 + 2 * m1 * c1 + m0 * c2, m2l * c0 + 2 * m1l * c1 + m0l * c2, m2 * c0f + 2 * m1 * c1f + m0 * c2f
        else:
            Dw, Dl, Df = m1 * c0 + m0 * c1, m1l * c0 + m0l * c1, m1 * c0f + m0 * c1f
        gw, gl, gf = gw + SD @ Dw, gl + SD @ Dl, gf + SD @ Df
    if not O._has_cos(k):
        gf = gf * 0
    out = {"freq": gf * w, "log-ls": gl * w, "log-w": gw * w}
    return np.concatenate([out[n].reshape(-1) for n in sorted(out)])  # _flatten's order, long double


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="C5")
    ap.add_argument("axis", nargs="?", type=int, default=2)
    a = ap.parse_args()
    from gpk.problems import make_solver
    O.set_backend(True)
    prob, params, _, cfg = config_problem(a.config)
    ax = a.axis
    s = make_solver(a.config, seed=0)
    print("solver up", flush=True)
    try:
        loss, g = s.loss_grad()
        fld = {n: s.forward_field(n) for n in ("Kc1", "D1", "Kc2", "D2", f"G_K{ax}", f"G_D{ax}", f"K{ax}inv")}
    finally:
        s.close()
    kd = {id(params["kernel_paras_1"]): (fld["Kc1"], fld["D1"]),
          id(params["kernel_paras_2"]): (fld["Kc2"], fld["D2"])}
    saved_kd, saved_pc = O.kernel_kd, O.param_grad_contract
    cap = {}

    def capture(kind, x, kp, GK, GD, deriv):
        cap.setdefault(mode, []).append((kind, x, kp, GK.copy(), None if GD is None else GD.copy(), deriv))
        return saved_pc(kind, x, kp, GK, GD, deriv)
    O.kernel_kd = lambda kind, x, kp, jitter, dv: kd[id(kp)]
    O.param_grad_contract = capture
    try:
        res = {}
        for mode in ("ext", "lu"):
            res[mode] = SA.run_mode(prob, params, mode)
            print(f"{mode} done", flush=True)
    finally:
        O.kernel_kd, O.param_grad_contract = saved_kd, saved_pc
    key = f"kernel_paras_{ax}"
    gref = res["ext"][1][key]
    scale = float(np.max(np.abs(gref)))
    kind, x, kp, GKx, GDx, deriv = cap["ext"][ax - 1]
    K = fld[f"Kc{ax}"]
    N_other = (cfg["n"])  # square grid: N1 = N2
    c = float(prob["logdet"])
    # the yardstick's K^{-1}: the same long-double LU solve (oracle/ext_solve.c) against I
    O.set_extended(True)
    try:
        Kinv_ext = O._solve(O._lu(K), np.eye(K.shape[0]))
    finally:
        O.set_extended(False)
    print("yardstick K^-1 done", flush=True)

    def contract(GK, GD):
        return O.flatten_params(saved_pc(kind, x, kp, GK, GD, deriv))

    def split(GK, GD, Kinv):
        dl = 0.5 * c * N_other * (Kinv - Kinv_ext)
        out = {"logdet": float(np.max(np.abs(contract(dl, np.zeros_like(GD))))) / scale,
               "quad": float(np.max(np.abs(contract(GK - GKx - dl, np.zeros_like(GD))))) / scale,
               "gd": float(np.max(np.abs(contract(np.zeros_like(GK), GD - GDx)))) / scale,
               "total": float(np.max(np.abs(contract(GK - GKx, GD - GDx)))) / scale}
        return out
    dev_g = O.unflatten_params(params, g)
    _, _, _, GKl, GDl, _ = cap["lu"][ax - 1]
    Kinv_lu = np.linalg.solve(K, np.eye(K.shape[0]))
    report = {"config": a.config, "key": key,
              "device_total_vs_ext": float(np.max(np.abs(O.flatten_params(dev_g[key]) - gref))) / scale,
              "device": split(fld[f"G_K{ax}"], fld[f"G_D{ax}"], fld[f"K{ax}inv"]),
              "lu_oracle": split(GKl, GDl, Kinv_lu),
              "kinv_rel_err": {"device": float(np.max(np.abs(fld[f"K{ax}inv"] - Kinv_ext)) / np.max(np.abs(Kinv_ext))),
                               "lu": float(np.max(np.abs(Kinv_lu - Kinv_ext)) / np.max(np.abs(Kinv_ext)))}}
    # the contraction's own rounding, against the exact contraction of the G each one contracted
    ex_dev = contract_ld(kind, x, kp, fld[f"G_K{ax}"], fld[f"G_D{ax}"], deriv)
    ex_ext = contract_ld(kind, x, kp, GKx, GDx, deriv)
    ex_lu = contract_ld(kind, x, kp, GKl, GDl, deriv)
    print("exact contractions done", flush=True)

    def e(v, ref):
        return float(np.max(np.abs(np.asarray(v, np.longdouble) - ref))) / scale
    report["contraction"] = {
        "device_step_vs_exact_of_device_G": e(O.flatten_params(dev_g[key]), ex_dev),
        "oracle_fp64_vs_exact_of_device_G": e(contract(fld[f"G_K{ax}"], fld[f"G_D{ax}"]), ex_dev),
        "yardstick_fp64_vs_exact_of_its_G": e(gref, ex_ext),
        "lu_fp64_vs_exact_of_its_G": e(res["lu"][1][key], ex_lu),
        "exact_device_G_vs_exact_yardstick_G": e(ex_dev, ex_ext),
        "exact_lu_G_vs_exact_yardstick_G": e(ex_lu, ex_ext),
        "device_step_vs_exact_yardstick_G": e(O.flatten_params(dev_g[key]), ex_ext),
        "lu_fp64_vs_exact_yardstick_G": e(res["lu"][1][key], ex_ext),
        # which half of an fp64 contraction carries the rounding: fp64 class sums (sequential per
        # distance) with exact fields, and exact sums with fp64 fields
        "fp64_sums_exact_fields_of_device_G": e(contract_ld(kind, x, kp, fld[f"G_K{ax}"], fld[f"G_D{ax}"], deriv, sums64=True), ex_dev),
        "exact_sums_fp64_fields_of_device_G": e(contract_ld(kind, x, kp, fld[f"G_K{ax}"], fld[f"G_D{ax}"], deriv, fields64=True), ex_dev)}
    print(json.dumps(report, indent=1), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out", "r5"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "r5", f"kp_split_{a.config}_{ax}.json"), "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
