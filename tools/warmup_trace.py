"""The driver's bench shape on a fresh C4 handle, then more of the same calls: where do a fresh
handle's first ~80 steps lose their 2.5 %?  Run under
    rocprofv3 --kernel-trace -f csv -d DIR -o w -- python3 tools/warmup_trace.py
and analyse with tools/warmup_analyze.py DIR (per-step device span and per-kernel durations
against the step index).  Prints the wall time of every step(20) call."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk.problems import make_solver

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 16
s = make_solver("C4", seed=0)
try:
    s.prepare(20)            # bench.py: every graph the timed call can launch ...
    s.prepare(5)             # ... and the warm-up call's
    s.step(5)
    s.sync()
    for c in range(calls):
        fast, rb = s.graph_mode()
        t0 = time.perf_counter()
        s.step(20)
        s.sync()
        dt = time.perf_counter() - t0
        fast2, rb2 = s.graph_mode()
        print(f"call {c:3d} steps {5 + 20 * c:4d}-{5 + 20 * c + 19:4d}: {dt * 1e6:8.1f} us = {20 / dt:7.1f} it/s"
              f"  fast {int(fast)}->{int(fast2)} rollbacks {rb2 - rb}", flush=True)
finally:
    s.close()
