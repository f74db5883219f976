"""How accurate are the solves of the log joint at a BASELINE config?  (test infrastructure)

Evaluates the loss and the full gradient of a config at its seeded bench params three ways,
all through the oracle's formulas (oracle/gp_oracle.py, code/model_GP_solver_{1d,2d}.py):

  lu   fp64 LU solves + slogdet (LAPACK getrf/getrs: what jnp.linalg.solve does, the reference)
  ext  the same solves in x87 80-bit long double (oracle/ext_solve.c): the "exact" yardstick
  inv  fp64 products with an explicit K^{-1} from a Cholesky factor: a CPU stand-in for the
       device's path, which forms K^{-1} (Gauss-Jordan sweeps with Cholesky pivots, spdinv*.hip)
       and applies it with GEMMs

and prints each one's distance from `ext` per gradient key (max-abs error / max-abs value, as
tests/helpers.rel).  With --fixture it writes tests/golden/ext_<config>.npz: the extended values
(every element, or for dL/dU above 2^20 elements a seeded sample of them plus the full max-abs)
and the LU oracle's own distance per key -- what the GPU parity tests measure the device against
(tests/test_gpu_accuracy.py).

usage: python tools/solve_accuracy.py C2 [C4 C5 T3072 ...] [--fixture] [--no-inv]
C5 (two 4096 factors, 7 long-double solves with 4096 right-hand sides) takes ~4 minutes on 8 cores.
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
from tests.helpers import config_problem, problem_2d, rel

# GPU tests' own problems with a yardstick fixture: T3072 is tests/test_gpu_fullsize.py's
# 3072^2 advection case (the 128x128-tile GEMM stages vs the 64x64 kernel, both checked against
# the yardstick instead of against each other)
TEST_PROBLEMS = {"T3072": dict(eq="advection", kind="Matern52_Cos_1d", n1=3072, n2=3072, Q=6, seed=3)}
SAMPLE = 16384          # dL/dU elements kept in a fixture when the field is larger than 2^20
SAMPLE_SEED = 1234


def sample_index(n):
    """The dL/dU positions a large fixture keeps (seeded, sorted, distinct)."""
    if n <= 1 << 20:
        return None
    return np.sort(np.random.default_rng(SAMPLE_SEED).choice(n, SAMPLE, replace=False))


def _fn(prob):
    return O.loss_grad_1d if "x" in prob else O.loss_grad_2d


def run_mode(prob, params, mode):
    """(loss, {key: flat gradient}) with the solves done the `mode` way."""
    fn = _fn(prob)
    saved = (O._lu, O._solve, O._slogdet_from_lu)
    try:
        if mode == "ext":
            O.set_extended(True)
        elif mode == "inv":
            def lu(K):
                c = sla.cho_factor(K, lower=True, check_finite=False)
                return ("inv", sla.cho_solve(c, np.eye(K.shape[0]), check_finite=False),
                        2.0 * float(np.sum(np.log(np.diag(c[0])))))

            def solve(f, B):
                return f[1] @ B if f[0] == "inv" else saved[1](f, B)

            def slogdet(f):
                return f[2] if f[0] == "inv" else saved[2](f)
            O._lu, O._solve, O._slogdet_from_lu = lu, solve, slogdet
        loss, g = fn(prob, params)
    finally:
        O.set_extended(False)
        O._lu, O._solve, O._slogdet_from_lu = saved
    return loss, {k: O.flatten_params(g[k]) for k in g}


def distances(a, b):
    la, ga = a
    lb, gb = b
    out = {"loss": abs(la - lb) / abs(lb)}
    for k in gb:
        out[k] = rel(ga[k], gb[k])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--fixture", action="store_true")
    ap.add_argument("--no-inv", action="store_true")
    ap.add_argument("--out", default=None, help="also write the distances as JSON here")
    a = ap.parse_args()
    O.set_backend(True)
    report = {}
    for cid in a.configs:
        if cid in TEST_PROBLEMS:  # a GPU test's own problem (not a BASELINE config)
            prob, params, _, _ = problem_2d(**TEST_PROBLEMS[cid])
        else:
            prob, params, _, cfg = config_problem(cid)
        res = {}
        for mode in ["lu", "ext"] + ([] if a.no_inv else ["inv"]):
            t = time.time()
            res[mode] = run_mode(prob, params, mode)
            print(f"{cid} {mode}: {time.time() - t:.1f} s", flush=True)
        d = {m: distances(res[m], res["ext"]) for m in res if m != "ext"}
        if "inv" in res:
            d["inv_vs_lu"] = distances(res["inv"], res["lu"])
        report[cid] = d
        for m, v in d.items():
            print(f"{cid} {m:10s} " + " ".join(f"{k} {e:.2e}" for k, e in sorted(v.items())), flush=True)
        if a.fixture:
            le, ge = res["ext"]
            fx = {"loss_ext": np.float64(le), "loss_lu_err": np.float64(d["lu"]["loss"])}
            for k, v in ge.items():
                idx = sample_index(v.size)
                fx[f"ext/{k}"] = v if idx is None else v[idx]
                fx[f"maxabs/{k}"] = np.float64(np.max(np.abs(v)))
                fx[f"lu_err/{k}"] = np.float64(d["lu"][k])
                if idx is not None:
                    fx[f"sample/{k}"] = idx.astype(np.int64)
            path = os.path.join(ROOT, "tests", "golden", f"ext_{cid}.npz")
            np.savez_compressed(path, **fx)
            print(f"wrote {path} ({os.path.getsize(path)} B)")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
