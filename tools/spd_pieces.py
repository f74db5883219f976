"""Per-launch times of the large-factor SPD inverse pieces (pivot, panel, update) at several sizes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk import problems
from gpk._lib import GPK_FLAG_FORCE_BIG_SPD

sizes = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "256,1024,2048,4096").split(",")]
for n in sizes:
    s = problems.make_solver(dict(problems.CONFIGS["C2"], n=n), flags=GPK_FLAG_FORCE_BIG_SPD)
    row = []
    for name in ("spd_pivot", "spd_panel", "spd_tiles", "sweep"):
        us, fl, by = s.bench_kernel(name, 5 if name == "spd_tiles" else 20)
        row.append(f"{name} {us:8.2f} us" + (f" ({fl / us / 1e6:.1f} TF/s, {by / us / 1e3:.0f} GB/s)" if fl else ""))
    print(f"n={n}: " + " | ".join(row), flush=True)
    s.close()
