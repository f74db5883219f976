"""C4 step(20) rate against the solver's age and its params (test infrastructure): does the
first ~50 steps' lower rate follow the params (training state) or the handle (first use)?
  A: fresh solver, 15 consecutive step(20) calls (after prepare + 5 warm-up steps)
  B: fresh solver whose params are set to A's params after 200 steps, then the same calls
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]


def calls(s, n=15, k=20):
    out = []
    for _ in range(n):
        s.sync()
        t = time.perf_counter()
        s.step(k)
        s.sync()
        out.append(k / (time.perf_counter() - t))
    return out


def main():
    from gpk.problems import make_solver
    s = make_solver("C4", seed=0)
    s.prepare(20)
    s.prepare(5)
    s.step(5)
    a = calls(s)
    print("A fresh, steps 5..305:", " ".join(f"{x:.0f}" for x in a), flush=True)
    flat = None
    s2 = make_solver("C4", seed=0)
    s2.prepare(20)
    s2.step(205)
    s2.sync()
    flat = s2.get_flat()
    s2.close()
    b = make_solver("C4", seed=0)
    b.prepare(20)
    b.prepare(5)
    b.set_flat(flat)
    b.step(5)
    r = calls(b)
    print("B fresh handle, params of step 205:", " ".join(f"{x:.0f}" for x in r), flush=True)
    s.close()
    b.close()


if __name__ == "__main__":
    main()
