"""C5 SPD inverse time: the two-sweep update schedule (default) against GPK_FLAG_ONE_SWEEP_UPDATE,
interleaved on one box, and the step time of each (test infrastructure)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]


def main():
    from gpk._lib import GPK_FLAG_ONE_SWEEP_UPDATE
    from gpk.problems import make_solver
    for rep in range(2):
        for tag, flags in (("two-sweep", 0), ("one-sweep", GPK_FLAG_ONE_SWEEP_UPDATE)):
            s = make_solver("C5", seed=0, flags=flags)
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
            print(f"rep {rep} {tag}: inverse {inv / 1e3:.3f} ms, step {ms:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
