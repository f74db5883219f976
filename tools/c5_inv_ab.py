"""C5's large-factor SPD inverse and step on the library GPK_LIB_PATH names (A/B driver):
inverse of both 4096 factors (time_spd_inverse), one update launch (spd_tiles) and whole steps."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk.problems import make_solver

s = make_solver("C5", seed=0)
try:
    s.prepare(3)
    s.step(1)
    s.sync()
    t0 = time.perf_counter()
    s.step(3)
    s.sync()
    step_ms = (time.perf_counter() - t0) / 3 * 1e3
    inv_us = s.time_spd_inverse(5)
    tus, tfl, _ = s.bench_kernel("spd_tiles", 5)
    gus, _, gby = s.bench_kernel("gather", 5)
    st = s.profile_stages(3)
    loss, _ = s.loss_grad()
finally:
    s.close()
print(f"{os.path.basename(os.path.dirname(os.environ.get('GPK_LIB_PATH', 'cur/x')))}: step {step_ms:.2f} ms  "
      f"inverse {inv_us / 1e3:.3f} ms ({2 * 4096 ** 3 / inv_us / 1e6:.1f} TF/s)  update launch {tus:.1f} us "
      f"({tfl / tus / 1e6:.1f} TF/s)  gather {gus:.1f} us ({gby / gus / 1e3:.0f} GB/s of K/Kc/D)  in-step assemble "
      f"{st['assemble']:.1f} us ({gby / st['assemble'] / 1e3:.0f} GB/s)  loss {loss!r}", flush=True)
