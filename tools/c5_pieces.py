"""Per-launch times of the C5 large-factor SPD inverse pieces (both 4096 factors per launch):
pivot (128-pivot of block 0), standalone panel, the update's tile work alone, the update launch
with its pivot workgroup and fused panel (sweep 0), and the whole inverse.

    python tools/c5_pieces.py
"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk import problems

s = problems.make_solver("C5", seed=0)
try:
    for name in ("spd_pivot", "spd_panel", "spd_tiles", "sweep", "spd_updates"):
        us, fl, by = s.bench_kernel(name, 5)
        print(f"{name:10s} {us:9.2f} us" + (f"  {fl / us / 1e6:.1f} TF/s" if fl else ""), flush=True)
    inv = s.time_spd_inverse(5)
    print(f"inverse    {inv:9.1f} us  ({2 * 4096 ** 3 / inv / 1e6:.1f} TF/s, n^3 per factor)", flush=True)
finally:
    s.close()
