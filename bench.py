#!/usr/bin/env python3
"""bench.py — log-joint iters/sec of the MI355X-native GP-PDE step (BASELINE.json metric).

Workload (BASELINE.json configs[3], "C4"): 2D Poisson sin(100x)sin(100y) on a 256x256
Kronecker collocation grid, Matern52_Cos_1d (GP-HM-StM), Q = 30, fp64, jitter 1e-6, Adam lr
0.01.  One step = loss + full gradient + Adam update (step(),
/root/reference/code/model_GP_solver_2d.py:176-183), params and optimizer state resident in
HBM before the timed region starts.  Synthetic data: the reference's grid/source/boundary
construction with U ~ 0.1 N(0,1) (seed = rank).

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process per GPU, each
solving an independent 256^2 problem (replicas, weak scaling, no data-path collective; see
DESIGN.md §Multi-GPU).  Timing: barrier + device sync on both sides of exactly --steps steps,
max over ranks; value = total steps of all ranks / that time.

Also reported: the dominant kernel's roofline (HIP events on the library's stream, algorithmic
bytes/flops per launch), fp64 SPD factor+inverse GFLOP/s, the CPU
oracle timed on this host on a bounded sample (rank 0, N = 1 only), and `large_factors`: the
MFMA-bound kernels at C5's 4096^2 size (GEMM TF/s and fraction of the fp64 peak, the large SPD
inverse, C5 ms/step; rank 0, N = 1 only, --no-large to skip).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]

PEAK_HBM_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_F64_TFLOPS = 78.6    # MI355X fp64 dense matrix (= vector) peak, spec
METRIC = "log-joint iters/sec + fp64 Cholesky GFLOP/s, 2D Poisson 256^2, 1-8 GPU"
# launches per step of the fast step graph (sweep: T = p/32 in the per-sweep inverse; the
# persistent chain inverse is one launch; 3 GEMM stages with the augmented chain, else 5)
KERNEL_LAUNCHES = {"spd_chain": 1, "sweep": None, "gemm_B": 3, "pgrad": 1, "assemble": 1}


# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench (tools/gpu_round.sh), summarised by
# tools/pmc_summary.py: HBM-side bytes per launch (2*FETCH + WRITE, MI355X_MICROARCH.md §HBM)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r1_pmc_c4.json")
PMC_KERNEL = {"spd_chain": "gpk::chain_kernel<2, true>", "sweep": "gpk::sweep_kernel",
              "gemm_B": "gpk::gemm_small_kernel<true>", "pgrad": "gpk::pgrad_kernel<true, true, 2, false, true>",
              "assemble": "gpk::class_eval_kernel<true, true, 2>"}


def pmc_traffic(kernel):
    """Bytes per launch of `kernel` from the committed PMC summary (None if absent)."""
    try:
        with open(PMC_SUMMARY) as f:
            k = json.load(f)["kernels"].get(kernel)
        return None if k is None else k["traffic_bytes"]
    except (OSError, ValueError, KeyError):
        return None


def cpu_baseline(config, seconds, max_steps=400):
    """The CPU oracle (oracle/gp_oracle.py: NumPy/SciPy LU + OpenMP C fields) on the same
    workload, bounded sample of `seconds` of work (test infrastructure; never the product)."""
    import numpy as np
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    os.environ["OMP_NUM_THREADS"] = str(threads)
    os.environ.setdefault("OMP_WAIT_POLICY", "PASSIVE")
    try:
        # OpenMP (C fields) gets the cores; BLAS runs single-threaded: a multithreaded
        # OpenBLAS contending with the OpenMP pool made a 256^2 step 6x slower (measured)
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(limits=1, user_api="blas")
    except Exception:  # pragma: no cover
        limiter = None
    from oracle import gp_oracle as O
    from gpk.problems import CONFIGS
    cfg = CONFIGS[config]
    prob, _, _ = O.setup_2d(cfg["equation"], cfg["n"], cfg["scale"], cfg["kernel"],
                            llk_weight=cfg["llk_weight"], beta=cfg.get("beta"), m_test=8)
    params = O.init_params_2d(cfg["n"], cfg["n"], 30, cfg["freq_scale"])
    params["U"] = 0.1 * np.random.default_rng(0).normal(size=(cfg["n"], cfg["n"]))
    opt = O.Adam(0.01)
    st = opt.init(params)
    lo, g = O.loss_grad_2d(prob, params)          # warm-up (thread pools, page-in)
    t0 = time.perf_counter()
    steps = 0
    while steps < max_steps and (time.perf_counter() - t0) < seconds:
        lo, g = O.loss_grad_2d(prob, params)
        params, st = opt.update(g, st, params)
        steps += 1
    dt = time.perf_counter() - t0
    if limiter is not None:
        limiter.unregister() if hasattr(limiter, "unregister") else None
    return {"value": steps / dt, "unit": "iters/s", "cores": threads, "kind": "port",
            "sample": f"{steps} full steps (loss+grad+Adam) of {config} {cfg['n']}x{cfg['n']}, "
                      f"{dt:.1f} s, oracle/gp_oracle.py (SciPy LU, 1 BLAS thread + OpenMP/libmvec "
                      f"C fields on {threads} threads)"}


def large_factors(steps=3):
    """The MFMA-bound end of the path on C5's 4096^2 grid (BASELINE.json configs[4]): the
    128x128-tile GEMM stage gemm_B (S = A K2^{-1} and the residual R = beta D1 A + Bt D2^T - F:
    three 4096^3 products), the 64-wide SPD inverse of both 4096 factors (n^3 flops each =
    potrf + potri) and whole steps.  Not the headline; shows fp64 MFMA utilisation at size."""
    from gpk.problems import make_solver
    s = make_solver("C5", seed=0)
    try:
        s.step(1)
        t0 = time.perf_counter()
        s.step(steps)
        step_ms = (time.perf_counter() - t0) / steps * 1e3
        us, fl, _ = s.bench_kernel("gemm_B", 5)
        inv_us = s.time_spd_inverse(3)
        n = 4096
        tus, tfl, _ = s.bench_kernel("spd_tiles", 3)
    finally:
        s.close()
    gemm_tf = fl / (us * 1e-6) / 1e12
    return {"config": "C5: advection 4096x4096, Matern52_Cos_1d, Q=30, fp64", "step_ms": step_ms,
            "gemm_B_us": us, "gemm_tflops": gemm_tf, "gemm_mfma_frac": gemm_tf / PEAK_F64_TFLOPS,
            "spd_inverse_ms": inv_us / 1e3, "cholesky_gflops": 2 * n ** 3 / (inv_us * 1e-6) / 1e9,
            "spd_update_tflops": tfl / (tus * 1e-6) / 1e12}


def main_sharded(a):
    """One 2D problem (--config) row-sharded over all ranks (gpk/shard.py): every rank runs its
    rows of every product, RCCL all-gathers / all-reduces inside the step graph.  value = steps
    of the single problem per second (strong scaling)."""
    from gpk import replicas, shard
    from gpk.problems import CONFIGS
    ctx = replicas.init("nccl")
    cfg = CONFIGS[a.config]
    s = shard.make_sharded_solver(a.config, ctx, seed=0)
    s.step(a.warmup)
    replicas.barrier(ctx)
    t0 = time.perf_counter()
    losses = s.step(a.steps)
    t1 = time.perf_counter()
    replicas.barrier(ctx)
    dt = replicas.max_over_ranks(t1 - t0, ctx)
    if ctx.rank == 0:
        n = cfg["n"]
        print(json.dumps({
            "metric": METRIC, "value": a.steps / dt, "unit": "iters/s", "n_gpus": ctx.world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: reference grid/source/boundary, U ~ 0.1 N(0,1) (seed 0, same on every rank)",
            "config": {"workload": f"{a.config}: one {n}x{n} 2D problem row-sharded over {ctx.world} GPU(s)",
                       "grid": [n, n], "Q": 30, "kernel": cfg["kernel"], "equation": cfg["equation"],
                       "parallelism": f"row-sharded x{ctx.world} (RCCL all-gather / all-reduce)"},
            "roofline": None, "cpu_baseline": None, "final_loss": float(losses[-1])}), flush=True)
    s.close()
    replicas.shutdown(ctx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--no-large", action="store_true", help="skip the C5-size MFMA section")
    ap.add_argument("--mode", choices=["replicas", "sharded"], default="replicas",
                    help="replicas: one independent problem per GPU (weak scaling, the default); "
                         "sharded: ONE 2D problem row-sharded over the GPUs with RCCL (strong scaling)")
    a = ap.parse_args()
    if a.mode == "sharded":
        return main_sharded(a)

    from gpk import replicas
    from gpk.problems import CONFIGS, make_solver
    ctx = replicas.init("nccl")
    world, rank, local = ctx.world, ctx.rank, ctx.local
    cfg = CONFIGS[a.config]
    s = make_solver(a.config, seed=rank, device=local)
    s.step(a.warmup)                     # warm-up: graph capture + caches
    replicas.barrier(ctx)
    t0 = time.perf_counter()
    fast_graph, rb0 = s.graph_mode()     # graph the timed batch starts on (refinement gate closed?)
    losses = s.step(a.steps)             # exactly K steps; returns after a device sync
    t1 = time.perf_counter()
    replicas.barrier(ctx)
    fast_end, rb1 = s.graph_mode()       # graph it ends on; chunks rerun inside the timed batch
    rollbacks = rb1 - rb0
    dt = replicas.max_over_ranks(t1 - t0, ctx)
    value = world * a.steps / dt

    # fp64 SPD factor+inverse rate: potrf + potri = n^3 flops per Kronecker factor
    inv_us = s.time_spd_inverse(20)
    n = cfg["n"]
    nfac = 2 if cfg["dim"] == 2 else 1
    chol_gflops = nfac * n ** 3 / (inv_us * 1e-6) / 1e9

    # per-kernel timings; the dominant kernel = largest device time per step
    T = (n + 31) // 32
    kern = {}
    try:  # the step's SPD inverse: the persistent chain launch when the factors are small
        s.bench_kernel("spd_chain", 1)
        spd = "spd_chain"
    except Exception:
        spd = "sweep"
    for name in ([spd, "gemm_B", "pgrad", "assemble"] if cfg["dim"] == 2 else [spd, "assemble"]):
        us, fl, by = s.bench_kernel(name, a.kernel_iters)
        launches = T if name == "sweep" else KERNEL_LAUNCHES[name]
        kern[name] = dict(us=us, flops=fl, bytes=by, per_step_us=us * launches)
    dom = max(kern, key=lambda k: kern[k]["per_step_us"])
    d = kern[dom]
    ai = d["flops"] / d["bytes"] if d["bytes"] else float("inf")
    ridge = PEAK_F64_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)
    if ai < ridge:
        roof = {"kernel": dom, "bound": "hbm", "achieved": d["bytes"] / (d["us"] * 1e-6) / 1e9,
                "peak": PEAK_HBM_GBS, "unit": "GB/s"}
    else:
        roof = {"kernel": dom, "bound": "mfma", "achieved": d["flops"] / (d["us"] * 1e-6) / 1e12,
                "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s"}
    roof["frac"] = roof["achieved"] / roof["peak"]
    roof["traffic"] = pmc_traffic(PMC_KERNEL[dom])
    roof["avg_launch_us"] = d["us"]
    roof["alg_flops_per_launch"] = d["flops"]
    roof["alg_bytes_per_launch"] = d["bytes"]

    large = None
    if rank == 0 and world == 1 and not a.no_large:
        try:
            large = large_factors()
        except Exception as e:  # reported, never required
            large = {"error": f"{type(e).__name__}: {e}"}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            cpu = cpu_baseline(a.config, a.cpu_seconds)
        except Exception as e:  # the baseline is reported, never required
            cpu = {"value": None, "error": f"{type(e).__name__}: {e}"}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "iters/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: reference grid/source/boundary of poisson_2d-sin_sin, U ~ 0.1 N(0,1) seeded per rank",
            "config": {"workload": f"{a.config}: 2D Poisson 256x256 Kronecker grid, Matern52_Cos_1d, Q=30, fp64"
                       if a.config == "C4" else a.config,
                       "grid": [n, n] if cfg["dim"] == 2 else [n], "Q": 30, "kernel": cfg["kernel"],
                       "equation": cfg["equation"],
                       "parallelism": f"replicas x{world} (one independent problem per GPU)"},
            "cholesky_gflops": chol_gflops,
            "spd_inverse_us": inv_us,
            "roofline": roof,
            "kernels_us": {k: round(v["us"], 3) for k, v in kern.items()},
            "cpu_baseline": cpu,
            "large_factors": large,
            "final_loss": float(losses[-1]),
            # step graph of the timed batch: "fast" = refinement GEMM stages left out (gate closed,
            # checked every step; a step needing refinement reruns its 64-step chunk on the full
            # graph, counted in rollbacks); "fast_at_end" = the graph the last chunk ran
            "step_graph": {"fast": bool(fast_graph), "fast_at_end": bool(fast_end), "rollbacks": int(rollbacks)},
        }
        print(json.dumps(out), flush=True)
    s.close()
    replicas.shutdown(ctx)


if __name__ == "__main__":
    main()
