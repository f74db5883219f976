"""C5 SPD inverse and step time of the loaded library (GPK_LIB_PATH selects it; test
infrastructure for same-box A/B runs of two builds)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]


def main():
    from gpk.problems import make_solver
    s = make_solver("C5", seed=0)
    try:
        inv = s.time_spd_inverse(10)
        s.step(2)
        s.sync()
        t = time.perf_counter()
        s.step(5)
        s.sync()
        ms = (time.perf_counter() - t) / 5 * 1e3
    finally:
        s.close()
    lib = os.path.basename(os.environ.get("GPK_LIB_PATH", "libgpk.so"))
    print(f"{lib}: inverse {inv / 1e3:.3f} ms, step {ms:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
