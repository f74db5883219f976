"""CPU-baseline calibration at the reference's own run configs (GPU box).

The reference's committed runs (code/result_log/poisson_{1d-single_sin,2d-sin_sin}/
kernel_Matern52_Cos_1d/epoch_100/Q30/log.txt:2) are 1D N = 400 and 2D 400^2, Matern52_Cos_1d,
Q = 30.  BASELINE.md §4's credibility check asks the CPU baseline (the oracle, bench.py's
cpu_baseline leg, kind "port") to be no slower there than the reference's own proxies: >= 20 it/s
at 1D N = 400 and >= 11 it/s at 2D 400^2.  This times the oracle at exactly those configs on this
host (all cores = 16 OpenMP threads, and 1 core; bounded samples, child processes, as the bench
does) and the device step beside it, and prints one JSON object.

usage: python tools/cpu_calibration.py [--seconds 10] [--out profiles/r4_cpu_calibration.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]

PROXIES = {"R1": 20.0, "R2": 11.0}   # the reference's own it/s at these configs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--gpu-steps", type=int, default=200)
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import bench
    from gpk.problems import REFERENCE_RUNS
    out = {"note": "oracle (kind port) vs the reference's own it/s proxies at its committed run configs",
           "host_cpus": os.cpu_count(), "configs": {}}
    for cid, cfg in REFERENCE_RUNS.items():
        r = {"config": f"{cfg['equation']} {cfg['kernel']} N={cfg['n']}{'^2' if cfg['dim'] == 2 else ''} Q=30",
             "reference_proxy_its": PROXIES[cid]}
        print(f"{cid}: CPU {a.threads} threads ...", flush=True)
        r["cpu_all"] = bench.cpu_baseline_child(cid, a.seconds, a.threads)
        print(f"{cid}: CPU 1 thread ...", flush=True)
        r["cpu_1core"] = bench.cpu_baseline_child(cid, a.seconds, 1)
        v = r["cpu_all"].get("value")
        r["cpu_all_vs_proxy"] = v / PROXIES[cid] if v else None
        r["credible"] = bool(v and v >= PROXIES[cid])
        if not a.no_gpu:
            from gpk.problems import make_solver
            s = make_solver(cid, seed=0)
            try:
                s.prepare(a.gpu_steps)
                s.step(20)
                s.sync()
                t = time.perf_counter()
                s.step(a.gpu_steps)
                s.sync()
                dt = time.perf_counter() - t
                r["gpu"] = {"value": a.gpu_steps / dt, "unit": "iters/s", "steps": a.gpu_steps,
                            "inverse_path": s.inverse_path()}
            finally:
                s.close()
            r["gpu_vs_cpu_all"] = r["gpu"]["value"] / v if v else None
        out["configs"][cid] = r
        print(json.dumps({cid: r}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
