"""Library fp64 GEMM rate on this device (torch.matmul -> rocBLAS / hipBLASLt) at the C5 stage
shape, for comparison with gemm_huge_kernel's rate in bench.py's `large_factors.gemm_tflops`.
Usage: python tools/dgemm_library.py [--n 4096] [--iters 20]"""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    n = a.n
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(n, n, dtype=torch.float64, device="cuda", generator=g)
    B = torch.randn(n, n, dtype=torch.float64, device="cuda", generator=g)
    C = torch.empty_like(A)
    out = {}
    for name, f in (("A@B", lambda: torch.matmul(A, B, out=C)),
                    ("A.T@B", lambda: torch.matmul(A.t(), B, out=C)),
                    ("A@B.T", lambda: torch.matmul(A, B.t(), out=C))):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        out[name] = {"ms": round(ms, 4), "tflops": round(2 * n ** 3 / (ms * 1e-3) / 1e12, 2)}
    print(json.dumps({"n": n, "dtype": "f64", "library": "torch.matmul (rocBLAS/hipBLASLt)",
                      "peak_tflops": 78.6, "results": out}), flush=True)


if __name__ == "__main__":
    main()
