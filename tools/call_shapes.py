"""Per-call wall time of step(n) at C4 for several call sizes (prepared graphs), to split a call's
cost into a fixed part and a per-step part.  Run under `rocprofv3 --hip-trace --kernel-trace` to
see where the fixed part goes (graph launch API time, launch -> first kernel, last kernel -> sync).

    python tools/call_shapes.py [n ...]
"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np
from gpk import problems

sizes = [int(v) for v in sys.argv[1:]] or [1, 2, 4, 8, 16, 20, 32, 64]
# the bench's shape first: prepare(20), a 5-step warm-up, then the first 20-step call and the next
s = problems.make_solver("C4", seed=0)
s.prepare(20)
s.step(5)
for i in range(4):
    s.sync()
    t = time.perf_counter()
    s.step(20)
    s.sync()
    dt = time.perf_counter() - t
    print(f"bench shape call {i}: {dt * 1e6:9.1f} us = {20 / dt:7.1f} it/s", flush=True)
for i in range(3):  # a 20-step call right after a 5-step one (the exec launched before)
    s.step(5)
    s.sync()
    t = time.perf_counter()
    s.step(20)
    s.sync()
    dt = time.perf_counter() - t
    print(f"after step(5) {i}: {dt * 1e6:9.1f} us = {20 / dt:7.1f} it/s", flush=True)
for i in range(3):  # ... after an idle host pause
    time.sleep(0.05)
    s.sync()
    t = time.perf_counter()
    s.step(20)
    s.sync()
    dt = time.perf_counter() - t
    print(f"after 50 ms idle {i}: {dt * 1e6:9.1f} us = {20 / dt:7.1f} it/s", flush=True)
for n in sizes:
    s.prepare(n)
s.step(80)
for n in sizes:
    ts = []
    for _ in range(12):
        s.sync()
        t = time.perf_counter()
        s.step(n)
        s.sync()
        ts.append(time.perf_counter() - t)
    ts = np.array(ts[2:]) * 1e6
    print(f"step({n:3d}): median {np.median(ts):9.1f} us  min {ts.min():9.1f} us  "
          f"per step {np.median(ts) / n:7.2f} us", flush=True)
print("graph", s.graph_mode())
s.close()
