"""Driver for counter passes: the large-factor inverse's update launch alone (bench_kernel
'spd_tiles', sweep 0) on one n x n factor, 64- or 128-wide sweeps."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk import problems
from gpk._lib import GPK_FLAG_FORCE_BIG_SPD, GPK_FLAG_FORCE_WIDE_SPD, GPK_FLAG_FORCE_NARROW_SPD

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
wide = (sys.argv[2] if len(sys.argv) > 2 else "wide") == "wide"
flags = GPK_FLAG_FORCE_BIG_SPD | (GPK_FLAG_FORCE_WIDE_SPD if wide else GPK_FLAG_FORCE_NARROW_SPD)
s = problems.make_solver(dict(problems.CONFIGS["C2"], n=n), flags=flags)
us, fl, by = s.bench_kernel("spd_tiles", 5)
print(f"n={n} {'W=128' if wide else 'W=64'} update {us:.2f} us {fl / us / 1e6:.1f} TF/s")
s.close()
