"""BASELINE.md §4 table on one MI355X box: per config the GPU step rate, the SPD factor+inverse
rate, the dense-part MFMA fraction, and the CPU oracle (the bench's cpu_baseline, child
processes) on all host cores and on one core.

    python tools/baseline_table.py [--configs C1,C2,C3,C4,C5] [--cpu-seconds 10] > table.json

Dense flops per step: 1D N^3, 2D 28 N^3 (factor + solves + the 13 N^3-size
products of the closed-form gradient).  CPU samples are bounded: at least one full step, then
steps until --cpu-seconds; C5's oracle step takes seconds to minutes, so it is timed over one
step with BLAS on the cores (its step is the dense LU solves and products).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="C1,C2,C3,C4,C5")
ap.add_argument("--cpu-seconds", type=float, default=10.0)
ap.add_argument("--cores", type=int, default=16)
ap.add_argument("--no-cpu", action="store_true")
a = ap.parse_args()

from gpk.problems import CONFIGS, make_solver  # noqa: E402

STEPS = {"C1": 500, "C2": 100, "C3": 500, "C4": 500, "C5": 10}
rows = {}
for c in a.configs.split(","):
    cfg = CONFIGS[c]
    n, dim = cfg["n"], cfg["dim"]
    s = make_solver(c, seed=0)
    try:
        k = STEPS[c]
        s.prepare(k)
        s.step(max(5, k // 10))
        s.sync()
        t0 = time.perf_counter()
        s.step(k)
        s.sync()
        dt = (time.perf_counter() - t0) / k
        inv_us = s.time_spd_inverse(5 if c == "C5" else 20)
        path = s.inverse_path()
    finally:
        s.close()
    nfac = 2 if dim == 2 else 1
    dense = 28 * n ** 3 if dim == 2 else n ** 3
    row = {"gpu_it_s": 1 / dt, "ms_per_step": dt * 1e3, "steps": k, "inverse_path": path,
           "spd_inverse_us": inv_us, "spd_inverse_gflops": nfac * n ** 3 / (inv_us * 1e-6) / 1e9,
           "dense_flops_per_step": dense,
           "mfma_frac_dense": dense / dt / 1e12 / bench.PEAK_F64_TFLOPS}
    print(json.dumps({c: row}), file=sys.stderr, flush=True)
    if not a.no_cpu:
        if c == "C5":
            row["cpu_all"] = bench.cpu_baseline_child(c, 0.0, a.cores, blas_threads=a.cores, warmup=False)
            row["cpu_1core"] = bench.cpu_baseline_child(c, 0.0, 1, blas_threads=1, warmup=False)
        else:
            row["cpu_all"] = bench.cpu_baseline_child(c, a.cpu_seconds, a.cores)
            row["cpu_1core"] = bench.cpu_baseline_child(c, a.cpu_seconds, 1)
        print(json.dumps({c: {"cpu_all": row["cpu_all"], "cpu_1core": row["cpu_1core"]}}),
              file=sys.stderr, flush=True)
    rows[c] = row
print(json.dumps(rows, indent=1))
