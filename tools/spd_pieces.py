"""Per-launch times of the large-factor SPD inverse pieces (pivot, panel, update) at several sizes,
64- and 128-wide sweeps (1D problems: one factor per launch).

    python tools/spd_pieces.py [sizes] [narrow|wide|both]
"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk import problems
from gpk._lib import GPK_FLAG_FORCE_BIG_SPD, GPK_FLAG_FORCE_WIDE_SPD, GPK_FLAG_FORCE_NARROW_SPD
from gpk.core import set_spd_big_workgroups

sizes = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "256,1024,2048,4096").split(",")]
which = sys.argv[2] if len(sys.argv) > 2 else "both"
widths = {"narrow": [False], "wide": [True], "both": [False, True]}[which]
set_spd_big_workgroups(int(sys.argv[3]) if len(sys.argv) > 3 else 0)  # 64-wide update workgroups
for n in sizes:
    for wide in widths:
        flags = GPK_FLAG_FORCE_BIG_SPD | (GPK_FLAG_FORCE_WIDE_SPD if wide else GPK_FLAG_FORCE_NARROW_SPD)
        s = problems.make_solver(dict(problems.CONFIGS["C2"], n=n), flags=flags)
        row = []
        for name in ("spd_pivot", "spd_panel", "spd_tiles", "sweep"):
            us, fl, by = s.bench_kernel(name, 5 if name == "spd_tiles" else 20)
            row.append(f"{name} {us:8.2f} us" + (f" ({fl / us / 1e6:.1f} TF/s, {by / us / 1e3:.0f} GB/s)" if fl else ""))
        inv = s.time_spd_inverse(5)
        print(f"n={n} {'W=128' if wide else 'W=64 '}: " + " | ".join(row)
              + f" | inverse {inv:9.1f} us ({n ** 3 / inv / 1e6:.1f} TF/s)", flush=True)
        s.close()
