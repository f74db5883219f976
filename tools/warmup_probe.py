"""Is a fresh C4 handle's slow start the handle's or the device's?  Wall
time of step(20) calls (the driver's timed call) in four situations, untraced:
  fresh   : a fresh handle after the bench's prepare + 5-step warm-up (the driver's shape)
  busy    : the same, but the GPU is kept busy for ~30 ms (fp64 matmuls on torch's stream)
            right before the first timed call
  idle    : a handle already in steady state (300 steps done), then 50 ms of host sleep
  steady  : the same handle back to back
    python tools/warmup_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import torch

from gpk.problems import make_solver


def calls(s, n, pre=None):
    out = []
    for c in range(n):
        if pre is not None:
            pre(c)
        t0 = time.perf_counter()
        s.step(20)
        s.sync()
        out.append(20 / (time.perf_counter() - t0))
    return out


def busy(ms=30.0):
    a = torch.randn(2048, 2048, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        a = (a @ a) * 1e-3
        torch.cuda.synchronize()


def fresh(pre_busy):
    s = make_solver("C4", seed=0)
    try:
        s.prepare(20)
        s.prepare(5)
        s.step(5)
        s.sync()
        if pre_busy:
            busy()
        return calls(s, 6)
    finally:
        s.close()


torch.zeros(1, device="cuda")
busy(50.0)  # (torch / HIP initialisation out of the way)
for rep in range(3):
    for tag in ("fresh", "busy"):
        r = fresh(tag == "busy")
        print(f"{tag:6s} rep {rep}: " + " ".join(f"{v:7.0f}" for v in r), flush=True)
s = make_solver("C4", seed=0)
try:
    s.prepare(20)
    s.step(300)
    s.sync()
    for rep in range(3):
        r = calls(s, 4, pre=lambda c: time.sleep(0.05) if c == 0 else None)
        print(f"idle   rep {rep}: " + " ".join(f"{v:7.0f}" for v in r), flush=True)
        r = calls(s, 4)
        print(f"steady rep {rep}: " + " ".join(f"{v:7.0f}" for v in r), flush=True)
finally:
    s.close()
