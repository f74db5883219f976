"""C5 step time and per-stage device times (HIP events around each stage, profile_stages) of
the loaded library (GPK_LIB_PATH selects it; test infrastructure for same-box A/B runs)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]


def main():
    from gpk.problems import make_solver
    s = make_solver("C5", seed=0)
    try:
        s.prepare(5)
        s.step(2)
        s.sync()
        t = time.perf_counter()
        s.step(5)
        s.sync()
        ms = (time.perf_counter() - t) / 5 * 1e3
        st = s.profile_stages(3)
    finally:
        s.close()
    lib = os.path.basename(os.environ.get("GPK_LIB_PATH", "libgpk.so"))
    keep = {k: round(v, 1) for k, v in st.items() if k in ("assemble", "spd_inverse", "pgrad_tail")}
    print(f"{lib}: step {ms:.2f} ms, stages us {keep}", flush=True)


if __name__ == "__main__":
    main()
