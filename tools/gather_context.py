"""The C5 K-assembly launch (gather_wide_kernel) timed in several contexts on one handle: back to
back (gpk_bench_kernel "gather", HIP events), right after a C5 GEMM stage (gather_after_gemm) or
after an HBM-bound copy of the same bytes (gather_after_copy), and inside whole steps; run under
rocprofv3 --kernel-trace to get every dispatch's duration in order.

    rocprofv3 --kernel-trace -f csv -d DIR -- python3 tools/gather_context.py
"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk import problems

s = problems.make_solver("C5", seed=0)
try:
    s.step(1)
    us, fl, by = s.bench_kernel("gather", 5)
    print(f"bench gather (events): {us:.1f} us  {by / us / 1e3:.0f} GB/s", flush=True)
    s.step(3)
    s.sync()
    us, fl, by = s.bench_kernel("gather", 5)
    print(f"bench gather again (events): {us:.1f} us  {by / us / 1e3:.0f} GB/s", flush=True)
    for ctx in ("gather_after_gemm", "gather_after_copy", "gather", "write_stream", "write_stream_after_copy"):
        us, fl, by = s.bench_kernel(ctx, 5)
        print(f"{ctx:18s} (events around the gather alone): {us:.1f} us  {by / us / 1e3:.0f} GB/s", flush=True)
finally:
    s.close()
