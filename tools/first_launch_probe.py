"""First launch of a prepared step graph vs a warm one, with and without host idle before it (C4)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk import problems
s = problems.make_solver("C4", seed=0)
for n in (20, 24, 28):
    s.prepare(n)
s.step(5)
def call(n):
    s.sync(); t = time.perf_counter(); s.step(n); s.sync(); return (time.perf_counter() - t) * 1e6
w = [call(20) for _ in range(6)]
print("warm 20-step calls:", [round(x) for x in w])
print("first 24-step call right after (no idle):", round(call(24)), " second:", round(call(24)), " per-step est:", round((w[-1]-25)/20, 2))
time.sleep(0.05)
print("first 28-step call after 50 ms idle:", round(call(28)), " second:", round(call(28)))
