"""Same-box A/B of handle flags on a BASELINE config's step rate (test infrastructure).

For each repetition and each flag set, a fresh solver (seed 0) runs W warm-up steps, then K
timed steps (wall clock around gpk_step + sync, as bench.py's timed region), at two shapes: the
driver's (K = 20) and a long run (K = 500).  Interleaved, so box drift hits both arms alike.
usage: python tools/ab_flags.py [--config C4] [--flags 0 131072] [--reps 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--flags", type=int, nargs="+", default=[0])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from gpk.problems import make_solver
    res = {f: [] for f in a.flags}
    for rep in range(a.reps):
        for f in a.flags:
            s = make_solver(a.config, seed=0, flags=f)
            try:
                row = []
                for w, k in ((5, 20), (20, 500)):
                    s.step(w)
                    s.sync()
                    t0 = time.perf_counter()
                    s.step(k)
                    s.sync()
                    row.append(k / (time.perf_counter() - t0))
            finally:
                s.close()
            res[f].append(row)
            print(f"{a.config} rep {rep} flags {f}: 20-step {row[0]:.1f} it/s, 500-step {row[1]:.1f} it/s", flush=True)
    for f in a.flags:
        r = res[f]
        print(f"{a.config} flags {f}: mean 20-step {sum(x[0] for x in r) / len(r):.1f}, 500-step {sum(x[1] for x in r) / len(r):.1f} it/s")


if __name__ == "__main__":
    main()
