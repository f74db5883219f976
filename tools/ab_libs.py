"""Same-box A/B of two or more libgpk builds on a BASELINE config's step rate (test infrastructure).

Each arm runs in a child process with GPK_LIB_PATH set to its library (the library is loaded once
per process); arms interleave per repetition, so box drift hits them alike.  Per arm and rep: a
fresh solver (seed 0), 5 warm-up steps + 20 timed (the driver's shape), then 20 more warm-up + 500
timed (wall clock around gpk_step + sync, as bench.py's timed region).
usage: python tools/ab_libs.py --config C4 --libs gpk/_lib/libgpk.so gpk/_lib/libgpk_x.so --reps 3
An arm "path@F" runs that library with handle flags F instead of --flags.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")


def child(config, flags):
    sys.path[:0] = [ROOT, PKG]
    from gpk.problems import make_solver
    s = make_solver(config, seed=0, flags=flags)
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
    print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a.config, a.flags)
    libs = list(a.libs)
    res = {p: [] for p in libs}
    for rep in range(a.reps):
        for arm in libs:
            p, _, fl = arm.partition("@")
            p = p if os.path.isabs(p) else os.path.join(PKG, p)
            env = dict(os.environ, GPK_LIB_PATH=p)
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--config", a.config,
                                  "--flags", fl or str(a.flags), "--libs", p], env=env, capture_output=True,
                                 text=True, timeout=300)
            if out.returncode != 0:
                print(out.stdout, out.stderr)
                raise SystemExit(f"arm {p} failed ({out.returncode})")
            row = json.loads(out.stdout.strip().splitlines()[-1])
            res[arm].append(row)
            print(f"{a.config} rep {rep} {os.path.basename(arm)}: 20-step {row[0]:.1f} it/s, 500-step {row[1]:.1f} it/s",
                  flush=True)
    for p in libs:
        r = res[p]
        print(f"{a.config} {os.path.basename(p)}: mean 20-step {sum(x[0] for x in r) / len(r):.1f}, "
              f"500-step {sum(x[1] for x in r) / len(r):.1f} it/s")


if __name__ == "__main__":
    main()
