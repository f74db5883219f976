"""Time the SPD inverse (small 32-wide sweeps vs the large-factor 64-wide panel/update path) on
1D Matern52_Cos_1d factors of growing size, and full steps of C2 / C5 under both paths.

    python tools/spd_sweep.py [--sizes 256,512,...] [--steps]
"""
import argparse, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk import problems
from gpk._lib import GPK_FLAG_FORCE_BIG_SPD, GPK_FLAG_FORCE_SMALL_SPD

ap = argparse.ArgumentParser()
ap.add_argument("--sizes", default="256,512,768,1024,1536,2048,4096")
ap.add_argument("--steps", action="store_true", help="also time full C2 / C5 steps")
ap.add_argument("--small-max", type=int, default=2048, help="skip the small path above this size")
a = ap.parse_args()

paths = (("small", GPK_FLAG_FORCE_SMALL_SPD), ("big", GPK_FLAG_FORCE_BIG_SPD))
for n in [int(v) for v in a.sizes.split(",")]:
    cfg = dict(problems.CONFIGS["C2"], n=n)
    row = []
    for name, flags in paths:
        if name == "small" and n > a.small_max:
            continue
        s = problems.make_solver(cfg, flags=flags)
        us = s.time_spd_inverse(5)
        s.close()
        row.append(f"{name} {us:9.1f} us ({n ** 3 / us / 1e3:7.1f} GF/s)")
    print(f"n={n:5d}: " + " | ".join(row), flush=True)

if a.steps:
    for cfgname, nsteps in (("C2", 50), ("C5", 5)):
        for name, flags in paths:
            if cfgname == "C5" and name == "small":
                continue
            s = problems.make_solver(cfgname, flags=flags)
            s.step(2)
            t = time.perf_counter()
            s.step(nsteps)
            dt = time.perf_counter() - t
            print(f"{cfgname} [{name}]: {dt * 1e3 / nsteps:.3f} ms/step", flush=True)
            print(s.profile_stages(3), flush=True)
            s.close()
