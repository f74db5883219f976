"""Rounding statistics of the step's fp64 MFMA GEMM kernels (gpk_dgemm) against long-double
products: mean (bias) and RMS of the error in ulps of the result, on positive operands (where
round-to-nearest errors average out and a directed rounding shows as a bias).  GPU box.
usage: python tools/gemm_rounding_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np

from gpk._lib import GEMM_BIG, GEMM_SMALL, GEMM_TILE128, dgemm

rng = np.random.default_rng(0)
n = 256
for dist in ("uniform(0,1)", "normal"):
    A = rng.uniform(0, 1, (n, n)) if dist != "normal" else rng.normal(size=(n, n))
    B = rng.uniform(0, 1, (n, n)) if dist != "normal" else rng.normal(size=(n, n))
    ex = np.asarray(A, np.longdouble) @ np.asarray(B, np.longdouble)
    sp = np.spacing(np.abs(np.asarray(ex, np.float64)))
    ref = {"numpy": A @ B}
    for name, v in (("small16", GEMM_SMALL), ("big64", GEMM_BIG), ("tile128", GEMM_TILE128)):
        ref[name] = dgemm(A, B, variant=v)[0]
    for name, C in ref.items():
        e = np.asarray(np.asarray(C, np.longdouble) - ex, np.float64) / sp
        print(f"{dist:13s} {name:8s}: error in ulps mean {e.mean():+.3f} rms {np.sqrt((e ** 2).mean()):.3f} "
              f"max {np.abs(e).max():.1f}", flush=True)
    # the MFMA's own rounding: one 16x16x4 block, K = 4 (a single instruction per element)
    A4, B4 = A[:, :32], B[:32, :]
    ex4 = np.asarray(A4, np.longdouble) @ np.asarray(B4, np.longdouble)
    sp4 = np.spacing(np.abs(np.asarray(ex4, np.float64)))
    for name, v in (("small16", GEMM_SMALL), ("tile128", GEMM_TILE128)):
        C = dgemm(A4, B4, variant=v)[0]
        e = np.asarray(np.asarray(C, np.longdouble) - ex4, np.float64) / sp4
        print(f"{dist:13s} {name:8s} K=32: mean {e.mean():+.3f} rms {np.sqrt((e ** 2).mean()):.3f}", flush=True)
    C = A4 @ B4
    e = np.asarray(np.asarray(C, np.longdouble) - ex4, np.float64) / sp4
    print(f"{dist:13s} numpy    K=32: mean {e.mean():+.3f} rms {np.sqrt((e ** 2).mean()):.3f}", flush=True)
