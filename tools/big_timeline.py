"""Device timeline of one 128-wide update launch of the C5 SPD inverse (sweep BIG_PROBE_SWEEP = 8,
factor 0) from the probe build (gpk_trace.h SLOT_BIG_*):

    GPK_LIB_PATH=.../libgpk_trace.so python tools/big_timeline.py [--reps 3]
"""
import argparse, ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np
from gpk import _lib, problems

NAMES = {240: "launch start (wg 0)", 241: "pivot wg: start .. its tile done", 242: "pivot128 done",
         243: "panel wgs: first start", 244: "panel done (last)", 245: "tile wgs: round 0 done (max)",
         246: "tile wgs: round 1 done (max)", 247: "quarter items: first start .. last end",
         248: "round 0: tile start (first .. last wg)", 249: "round 0: first K-step done (last wg)",
         250: "round 0: K-loop done (last wg)", 251: "round 1: tile start (first .. last wg)",
         252: "round 1: first K-step done (last wg)", 253: "round 1: K-loop done (last wg)"}
ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--flags", default="0", help="problem flags: an int or GPK_FLAG_* names joined by |")
a = ap.parse_args()
flags = 0
for f in a.flags.split("|"):
    flags |= int(f) if f.strip().isdigit() else getattr(_lib, f.strip())
lib = _lib.load()
s = problems.make_solver("C5", seed=0, flags=flags)
rows = []
try:
    s.loss_grad()
    for _ in range(a.reps):
        lib.gpk_trace_reset()
        s.loss_grad()
        lo = (ctypes.c_uint64 * 256)()
        hi = (ctypes.c_uint64 * 256)()
        if lib.gpk_trace_read(lo, hi, 256):
            sys.exit(_lib.load().gpk_last_error().decode())
        t0 = lo[240]
        rows.append({k: ((lo[k] - t0) / 100.0 if lo[k] != 2 ** 64 - 1 else np.nan,
                         (hi[k] - t0) / 100.0 if hi[k] else np.nan) for k in NAMES})
finally:
    s.close()
print(f"C5 wide update launch, sweep 8, factor 0, flags {a.flags} (us from the launch's first workgroup; mean of {a.reps})")
for k, nm in NAMES.items():
    l = np.nanmean([r[k][0] for r in rows]) if any(np.isfinite(r[k][0]) for r in rows) else np.nan
    h = np.nanmean([r[k][1] for r in rows]) if any(np.isfinite(r[k][1]) for r in rows) else np.nan
    print(f"  {nm:40s} {l:8.2f} .. {h:8.2f}")
