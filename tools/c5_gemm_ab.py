"""C5 GEMM stage kernel time (gpk_bench_kernel gemm_B, HIP events) and ms/step for the library
GPK_LIB_PATH selects (A/B of GEMM variants)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk import problems

s = problems.make_solver("C5", seed=0)
try:
    s.prepare(3)
    s.step(1)
    s.sync()
    t = time.perf_counter()
    s.step(3)
    s.sync()
    ms = (time.perf_counter() - t) / 3 * 1e3
    us, fl, _ = s.bench_kernel("gemm_B", 5)
    print(f"{os.path.basename(os.environ.get('GPK_LIB_PATH', 'libgpk.so'))}: step {ms:.2f} ms  gemm_B {us:.1f} us {fl / us / 1e6:.1f} TF/s", flush=True)
finally:
    s.close()
