"""Per-call overhead of gpk_step at C4: wall time of one prepared step(n) call (device synced on
both sides, as bench.py times it) for several n, and its split into a fixed part and a per-step
part (least squares).  The fixed part is what separates the driver's 20-step line from the
500-step rate.  Usage: python tools/call_overhead.py [--config C4] [--reps 30]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "gaussian-process-slover-for-high-freq-pde_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--ns", default="1,2,4,8,16,20,32,64")
    a = ap.parse_args()
    from gpk.problems import make_solver
    s = make_solver(a.config, seed=0, device=0)
    ns = [int(x) for x in a.ns.split(",")]
    for n in ns:
        s.prepare(n)
    s.step(20)
    s.sync()
    rows = []
    for n in ns:
        ts = []
        for _ in range(a.reps):
            s.sync()
            t0 = time.perf_counter()
            s.step(n)
            s.sync()
            ts.append(time.perf_counter() - t0)
        med = float(np.median(ts)) * 1e6
        rows.append((n, med))
        print(json.dumps({"n": n, "us_per_call": round(med, 1), "us_per_step": round(med / n, 2)}), flush=True)
    # the FIRST launch of a freshly prepared call graph (bench.py's timed call is one) against
    # its second launch
    for n in (12, 24):
        s.prepare(n)
        s.sync()
        tt = []
        for _ in range(2):
            t0 = time.perf_counter()
            s.step(n)
            s.sync()
            tt.append((time.perf_counter() - t0) * 1e6)
        print(json.dumps({"n": n, "first_call_us": round(tt[0], 1), "second_call_us": round(tt[1], 1)}), flush=True)
    x = np.array([r[0] for r in rows], float)
    y = np.array([r[1] for r in rows], float)
    b, c = np.polyfit(x, y, 1)
    print(json.dumps({"fit_us_per_step": round(float(b), 2), "fit_fixed_us": round(float(c), 1),
                      "residuals_us": [round(float(v), 1) for v in y - (b * x + c)]}), flush=True)


if __name__ == "__main__":
    main()
