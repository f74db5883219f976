"""A/B of the 128-wide update's item order (quarter items first vs last, GPK_FLAG_NO_QUARTER_FIRST)
at C5, interleaved on one box: inverse of both 4096 factors (time_spd_inverse), the update launches
(gpk_bench_kernel "spd_updates": per launch, TF/s by the work their lists schedule), and whole steps.
    python tools/c5_qfirst_ab.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk._lib import GPK_FLAG_NO_QUARTER_FIRST
from gpk.problems import make_solver

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for rep in range(reps):
    for tag, flags in (("qfirst", 0), ("qlast", GPK_FLAG_NO_QUARTER_FIRST)):
        s = make_solver("C5", seed=0, flags=flags)
        try:
            s.prepare(5)
            s.step(1)
            s.sync()
            t0 = time.perf_counter()
            s.step(5)
            s.sync()
            step_ms = (time.perf_counter() - t0) / 5 * 1e3
            inv = s.time_spd_inverse(5)
            us, fl, _ = s.bench_kernel("spd_updates", 3)
        finally:
            s.close()
        print(f"rep {rep} {tag:6s}: inverse {inv / 1e3:6.3f} ms  update launch {us:6.1f} us "
              f"{fl / us / 1e6:5.1f} TF/s  step {step_ms:6.2f} ms", flush=True)
