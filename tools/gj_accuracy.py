"""Where does the C5 dL/dU error come from, and how accurate is each SPD-inverse variant?  (CPU)

NumPy emulation of the device's large-factor path at a BASELINE config (default C5, the two
4096^2 advection factors at the seeded bench params), against the long-double yardstick
(oracle/ext_solve.c, the same solves tests/golden/ext_C5.npz is made of):

  * inverse variants: Gauss-Jordan sweeps of width W with Cholesky pivots (spdinv_big.hip), the
    pivot's L^{-1} formed from 32-blocks by the device's recursion ("rec") or by a triangular
    solve ("trsm"), the panel Z = L^{-1} X_P as an explicit-inverse product ("explicit") or by
    blocked forward substitution with the 32-blocks' own inverses ("fwd"); and the exact inverse
    rounded to fp64 ("exact");
  * per variant, the relative max-abs error of K^{-1} and of each dL/dU term of the device's
    formulas (S = A K2^{-1}, v X1 = v beta (K1^{-1} D1^T) R, v X2 = v R (K2^{-1} D2^T)^T, with
    A, Bt refined once as on the device), each over max |dL/dU|; and of S refined once.

The long-double pieces take ~5 minutes on 8 cores and are cached in --cache.
usage: python tools/gj_accuracy.py [--config C5] [--variants exact,128:rec:explicit,...]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np
import scipy.linalg as sla

from oracle import gp_oracle as O
from tests.helpers import config_problem


def chol_inv32(S):
    """the 32-pivot: L = chol(S), L^{-1} (triangular solve; the device's blocked MFMA form has
    the same accuracy class)"""
    L = np.linalg.cholesky(S)
    return L, sla.solve_triangular(L, np.eye(S.shape[0]), lower=True)


def linv_rec(S):
    """L^{-1} of an SPD block by the device's recursion: halves down to 32,
    L11^{-1} = rec(S11); V = L11^{-1} S12; L22^{-1} = rec(S22 - V^T V); (L^{-1})_21 = -L22^{-1} (V^T L11^{-1})"""
    w = S.shape[0]
    if w <= 32:
        return chol_inv32(S)[1]
    h = w // 2
    M1 = linv_rec(S[:h, :h])
    V = M1 @ S[:h, h:]
    M2 = linv_rec(S[h:, h:] - V.T @ V)
    out = np.zeros_like(S)
    out[:h, :h] = M1
    out[h:, h:] = M2
    out[h:, :h] = -M2 @ (V.T @ M1)
    return out


def blk_chol(S, b=32):
    """Blocked right-looking Cholesky of an SPD block, as a device pivot would run it: per
    32-block the pivot32 (chol + inverse of the diagonal block), the panel below as
    L_ji = (M_i S_ij)^T, the Schur update of the trailing blocks.  Returns (L, [M_i])."""
    w = S.shape[0]
    A = np.array(S)
    L = np.zeros_like(A)
    Ms = []
    for i in range(0, w, b):
        ii = slice(i, min(w, i + b))
        Li, Mi = chol_inv32(A[ii, ii])
        L[ii, ii] = Li
        Ms.append(Mi)
        rest = slice(ii.stop, w)
        if ii.stop < w:
            V = Mi @ A[ii, rest]          # = L_{rest,i}^T
            L[rest, ii] = V.T
            A[rest, rest] -= V.T @ V
    return L, Ms


def blk_fwd(L, Ms, B, b=32):
    """L^{-1} B by 32-block forward substitution with the diagonal blocks' inverses."""
    Z = np.empty_like(B)
    for k, i in enumerate(range(0, L.shape[0], b)):
        ii = slice(i, min(L.shape[0], i + b))
        Z[ii] = Ms[k] @ (B[ii] - L[ii, :i] @ Z[:i])
    return Z


def gj_inverse(K, W, linv="rec", panel="explicit"):
    """X <- -K^{-1} by W-wide Gauss-Jordan sweeps (full storage; the device updates the lower
    triangle and mirrors), then the sign flip."""
    X = np.array(K, dtype=np.float64)
    p = X.shape[0]
    for r0 in range(0, p, W):
        P = slice(r0, min(p, r0 + W))
        S = X[P, P].copy()
        if linv == "blk":   # device-implementable accurate form: blocked Cholesky, every panel
            L, Ms = blk_chol(S)   # column (the pivot's own: L^{-1} = fwd(I)) by forward substitution
            XP = X[P, :].copy()
            XP[:, P] = np.eye(S.shape[0])
            Z = blk_fwd(L, Ms, XP)
            inP = np.zeros(p, bool)
            inP[P] = True
            G = Z.T @ Z
            sgn = np.where(inP[:, None] != inP[None, :], -1.0, 1.0)
            base = np.where(inP[:, None] | inP[None, :], 0.0, X)
            X = sgn * (base - G)
            continue
        if linv == "rec":
            Li = linv_rec(S)
        else:
            Li = sla.solve_triangular(np.linalg.cholesky(S), np.eye(S.shape[0]), lower=True)
        XP = X[P, :].copy()
        if panel == "explicit":
            Z = Li @ XP
        else:  # blocked forward substitution, 32-wide diagonal blocks through their own inverses
            w = S.shape[0]
            L = np.linalg.cholesky(S)
            Z = np.empty_like(XP)
            for b in range(0, w, 32):
                bb = slice(b, min(w, b + 32))
                rhs = XP[bb] - L[bb, :b] @ Z[:b]
                Lb = sla.solve_triangular(L[bb, bb], np.eye(bb.stop - bb.start), lower=True)
                Z[bb] = Lb @ rhs
        Z[:, P] = Li
        inP = np.zeros(p, bool)
        inP[P] = True
        G = Z.T @ Z
        sgn = np.where(inP[:, None] != inP[None, :], -1.0, 1.0)
        base = np.where(inP[:, None] | inP[None, :], 0.0, X)
        X = sgn * (base - G)
    return -X


def rel(a, b, scale=None):
    return float(np.max(np.abs(a - b)) / (scale if scale is not None else np.max(np.abs(b))))


def exact_pieces(cid, cache):
    if os.path.exists(cache):
        z = np.load(cache)
        return {k: z[k] for k in z.files}
    prob, params, _, cfg = config_problem(cid)
    assert prob["eq"] == "advection"
    beta = float(prob["beta"])
    K1, D1 = O.kernel_kd(prob["kind"], prob["x1"], params["kernel_paras_1"], prob["jitter"], 1)
    K2, D2 = O.kernel_kd(prob["kind"], prob["x2"], params["kernel_paras_2"], prob["jitter"], 1)
    U = np.asarray(params["U"], np.float64)
    F = np.asarray(prob["src"], np.float64).reshape(U.shape)
    t = time.time()
    f1, f2 = O._ext_lu(K1), O._ext_lu(K2)
    I = np.eye(K1.shape[0])
    K1i, K2i = O._ext_solve(f1, I), O._ext_solve(f2, I)
    A = O._ext_solve(f1, U)
    Bt = O._ext_solve(f2, U.T).T
    S = O._ext_solve(f2, A.T).T
    R = beta * (D1 @ A) + Bt @ D2.T - F
    X1 = beta * O._ext_solve(f1, D1.T @ R)
    X2 = O._ext_solve(f2, (R @ D2).T).T
    print(f"long-double pieces: {time.time() - t:.0f} s", flush=True)
    out = dict(K1=K1, K2=K2, D1=D1, D2=D2, U=U, F=F, K1i=K1i, K2i=K2i, A=A, Bt=Bt, S=S, R=R, X1=X1, X2=X2,
               beta=np.float64(beta), v=np.float64(np.exp(params["log_v"])))
    np.savez(cache, **out)
    return out


def device_terms(e, K1i, K2i, refine_s=False):
    K1, K2, D1, D2, U, F = e["K1"], e["K2"], e["D1"], e["D2"], e["U"], e["F"]
    beta = float(e["beta"])
    A = K1i @ U
    A = A + K1i @ (U - K1 @ A)
    Bt = U @ K2i
    Bt = Bt + (U - Bt @ K2) @ K2i
    S = A @ K2i
    if refine_s:
        S = S + (A - S @ K2) @ K2i
    R = beta * (D1 @ A) + Bt @ D2.T - F
    X1 = beta * ((K1i @ D1.T) @ R)
    X2 = R @ (K2i @ D2.T).T
    return dict(A=A, Bt=Bt, S=S, R=R, X1=X1, X2=X2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--cache", default="/tmp/gj_accuracy_C5.npz")
    ap.add_argument("--variants", default="exact,32:rec:explicit,128:rec:explicit,128:rec:fwd,128:trsm:fwd,"
                                          "256:rec:explicit,256:rec:fwd")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    e = exact_pieces(a.config, a.cache)
    v = float(e["v"])
    gU = e["S"] + v * (e["X1"] + e["X2"])
    scale = float(np.max(np.abs(gU)))
    ex = {"S": e["S"], "vX1": v * e["X1"], "vX2": v * e["X2"]}
    report = {"config": a.config, "max_abs_gU": scale,
              "term_max_abs_over_gU": {k: float(np.max(np.abs(t)) / scale) for k, t in ex.items()}}
    for var in a.variants.split(","):
        t = time.time()
        if var == "exact":
            K1i, K2i = e["K1i"], e["K2i"]
        else:
            W, linv, panel = var.split(":")
            K1i = gj_inverse(e["K1"], int(W), linv, panel)
            K2i = gj_inverse(e["K2"], int(W), linv, panel)
        r = {"inv_rel_err": max(rel(K1i, e["K1i"]), rel(K2i, e["K2i"]))}
        for refine_s in (False, True):
            d = device_terms(e, K1i, K2i, refine_s)
            dv = {"S": d["S"], "vX1": v * d["X1"], "vX2": v * d["X2"]}
            g = dv["S"] + dv["vX1"] + dv["vX2"]
            key = "refS" if refine_s else "default"
            r[key] = {k: rel(dv[k], ex[k], scale) for k in dv}
            r[key]["gU"] = rel(g, gU, scale)
            r[key]["R"] = rel(d["R"], e["R"])
        r["seconds"] = time.time() - t
        report[var] = r
        print(var, json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
