#!/usr/bin/env python3
"""bench.py — log-joint iters/sec of the MI355X-native GP-PDE step (BASELINE.json metric).

Workload (BASELINE.json configs[3], "C4"): 2D Poisson sin(100x)sin(100y) on a 256x256
Kronecker collocation grid, Matern52_Cos_1d (GP-HM-StM), Q = 30, fp64, jitter 1e-6, Adam lr
0.01.  One step = loss + full gradient + Adam update (step(),
/root/reference/code/model_GP_solver_2d.py:176-183), params and optimizer state resident in
HBM before the timed region starts.  Synthetic data: the reference's grid/source/boundary
construction with U ~ 0.1 N(0,1) (seed = rank).

Multi-GPU: `bench.py --gpus N` starts N ranks of itself (one process per GPU, the
torch.distributed.run environment: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*) before anything
touches a GPU, or runs as one of the ranks when launched by torch.distributed.run (then --gpus
must equal WORLD_SIZE).  Each rank solves an independent 256^2 problem (replicas, weak scaling,
no data-path collective).  Timing: barrier + device sync on both sides of exactly
--steps steps, max over ranks; value = total steps of all ranks / that time.  With N > 1 the
line also carries `sharded`: ONE C4 and ONE C5 problem row-sharded over the N ranks with RCCL
(strong scaling of a single problem).

Also reported: the dominant kernel's roofline (HIP events on the library's stream, algorithmic
bytes/flops per launch), fp64 SPD factor+inverse GFLOP/s, a step(1)-per-call
rate (the reference's loop shape), the CPU oracle timed on this host on bounded samples (all
cores and 1 core; rank 0, N = 1 only; child processes, so no thread setting leaks into the GPU
process), and `large_factors`: the MFMA-bound kernels at C5's 4096^2 size (rank 0, N = 1).
"""
import argparse
import json
import os
import subprocess
import sys
import threading
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
# (the newest round's summary; the line names it and the source tree it was measured on, so a
# traffic figure older than the kernel it prices is visible as such)
def _newest_pmc():
    import glob
    import re
    files = glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_c4.json"))
    files.sort(key=lambda f: int(re.match(r"r(\d+)_", os.path.basename(f)).group(1)))
    return files[-1] if files else None


PMC_SUMMARY = _newest_pmc()
PMC_KERNEL = {"spd_chain": "gpk::chain_kernel<2, true>", "sweep": "gpk::sweep_kernel",
              "gemm_B": "gpk::gemm_small_kernel<true>", "pgrad": "gpk::pgrad_kernel<true, true, 2, false, true>",
              "assemble": "gpk::class_eval_kernel<true, true, 2>"}


def pmc_traffic(kernel):
    """(bytes per launch of `kernel` from the committed PMC summary or None, the summary's
    provenance: file, the source tree it was measured on, how)."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
        k = d["kernels"].get(kernel)
        src = {"file": os.path.relpath(PMC_SUMMARY, ROOT), "tree": d.get("tree"), "how": d.get("source")}
        return (None if k is None else k["traffic_bytes"]), src
    except (OSError, ValueError, KeyError, TypeError):
        return None, None


# ------------------------------------------------------------------------------------------
# CPU baseline (test infrastructure: the oracle, never the product)
# ------------------------------------------------------------------------------------------
def cpu_baseline(config, seconds, threads, max_steps=400, min_steps=1, warmup=True, blas_threads=1):
    """The CPU oracle (oracle/gp_oracle.py: NumPy/SciPy LU + OpenMP C fields) on the same
    workload, a bounded sample of `seconds` of work.  Runs in a child process of rank 0
    (`--cpu-baseline-only`): OMP / BLAS thread counts are fixed before NumPy loads."""
    import numpy as np
    try:
        # OpenMP (C fields) gets the cores; BLAS runs single-threaded: a multithreaded
        # OpenBLAS contending with the OpenMP pool made a 256^2 step 6x slower (measured)
        from threadpoolctl import threadpool_limits
        threadpool_limits(limits=blas_threads, user_api="blas")
    except Exception:  # pragma: no cover
        pass
    from oracle import gp_oracle as O
    from gpk.problems import get_config
    cfg = get_config(config)
    n = cfg["n"]
    if cfg["dim"] == 1:
        prob, _, _ = O.setup_1d(cfg["equation"], n, cfg["scale"], cfg["kernel"],
                                llk_weight=cfg["llk_weight"], m_test=8)
        params = O.init_params_1d(n, 30, cfg["freq_scale"])
        params["u"] = 0.1 * np.random.default_rng(0).normal(size=(n, 1))
        loss_grad = O.loss_grad_1d
    else:
        prob, _, _ = O.setup_2d(cfg["equation"], n, cfg["scale"], cfg["kernel"],
                                llk_weight=cfg["llk_weight"], beta=cfg.get("beta"), m_test=8)
        params = O.init_params_2d(n, n, 30, cfg["freq_scale"])
        params["U"] = 0.1 * np.random.default_rng(0).normal(size=(n, n))
        loss_grad = O.loss_grad_2d
    opt = O.Adam(0.01)
    st = opt.init(params)
    if warmup:
        lo, g = loss_grad(prob, params)           # warm-up (thread pools, page-in)
    t0 = time.perf_counter()
    steps = 0
    while steps < max(1, min_steps) or (steps < max_steps and (time.perf_counter() - t0) < seconds):
        lo, g = loss_grad(prob, params)
        params, st = opt.update(g, st, params)
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": steps / dt, "unit": "iters/s", "cores": max(threads, blas_threads), "kind": "port",
            "sample": f"{steps} full steps (loss+grad+Adam) of {config} {'x'.join([str(n)] * cfg['dim'])}, "
                      f"{dt:.1f} s, oracle/gp_oracle.py (SciPy LU, {blas_threads} BLAS thread(s) + OpenMP/libmvec "
                      f"C fields on {threads} thread(s))"}


def cpu_baseline_child(config, seconds, threads, blas_threads=1, warmup=True):
    """blas_threads > 1: BLAS gets the cores instead of the OpenMP fields (the large configs,
    whose step is dominated by the dense LU solves and products)."""
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_WAIT_POLICY="PASSIVE",
               OPENBLAS_NUM_THREADS=str(blas_threads), HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--config", config,
           "--cpu-seconds", str(seconds), "--cpu-threads", str(threads),
           "--cpu-blas-threads", str(blas_threads)] + ([] if warmup else ["--cpu-no-warmup"])
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=10 * seconds + 300)
    if r.returncode != 0:
        return {"value": None, "error": r.stderr.strip().splitlines()[-1:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


# ------------------------------------------------------------------------------------------
# GPU sections
# ------------------------------------------------------------------------------------------
def large_factors(steps=3):
    """The MFMA-bound end of the path on C5's 4096^2 grid (BASELINE.json configs[4]): the
    128x128-tile GEMM stage gemm_B (S = A K2^{-1} and the residual R = beta D1 A + Bt D2^T - F:
    three 4096^3 products), the SPD factor + inverse of both 4096 factors (n^3 flops each =
    potrf + potri) and whole steps.  Not the headline; shows fp64 MFMA utilisation at size."""
    from gpk.problems import make_solver
    s = make_solver("C5", seed=0)
    try:
        s.prepare(steps)
        s.step(1)
        s.sync()
        t0 = time.perf_counter()
        s.step(steps)
        s.sync()
        step_ms = (time.perf_counter() - t0) / steps * 1e3
        us, fl, _ = s.bench_kernel("gemm_B", 5)
        inv_us = s.time_spd_inverse(3)
        n = 4096
        # every update launch of one inverse (even and odd launches of the two-sweep schedule),
        # credited the MFMA work their tile lists schedule (gpk_bench_kernel "spd_updates")
        tus, tfl, _ = s.bench_kernel("spd_updates", 3)
        gus, _, gby = s.bench_kernel("gather", 5)
        # the same launch inside whole steps (stage 'assemble' = class_eval + the gather, HIP
        # events around the stage): the first gather after a step's GEMMs runs ~2x slower than
        # back to back, so both are reported
        stages = s.profile_stages(3)
        path = s.inverse_path()
    finally:
        s.close()
    gemm_tf = fl / (us * 1e-6) / 1e12
    return {"config": "C5: advection 4096x4096, Matern52_Cos_1d, Q=30, fp64", "step_ms": step_ms,
            "inverse_path": path, "gemm_B_us": us, "gemm_tflops": gemm_tf,
            "gemm_mfma_frac": gemm_tf / PEAK_F64_TFLOPS, "spd_inverse_ms": inv_us / 1e3,
            "spd_inverse_gflops": 2 * n ** 3 / (inv_us * 1e-6) / 1e9,
            "spd_update_tflops": tfl / (tus * 1e-6) / 1e12,
            "spd_update_us": tus,
            "spd_update_flops": "per update launch, averaged over one inverse's launches: the tile "
                                "products its lists schedule (2 w_I w_J K, K = 128 or 256) + next pivot + panel",
            # K-assembly at size: gather_kernel writes K (+ its kept copy) and D of both 4096^2
            # factors from the class values and reads each element's class-id variant byte (the
            # bytes it moves: 839 MB at C5)
            "assembly": {"kernel": "gather_wide_kernel (K, Kc, D of both factors from class values, nontemporal stores)",
                         "us": gus, "bytes": gby, "hbm_gbs": gby / (gus * 1e-6) / 1e9,
                         "hbm_frac": gby / (gus * 1e-6) / 1e9 / PEAK_HBM_GBS,
                         "timing": "back to back, HIP events",
                         "in_step": {"stage": "assemble (class_eval + gather)",
                                     "us": stages.get("assemble"),
                                     "hbm_gbs": gby / (stages["assemble"] * 1e-6) / 1e9
                                     if stages.get("assemble") else None}}}


def sharded_section(a, ctx, configs=("C4", "C5", "C5_split"), make_sharded=None, make_single=None):
    """ONE problem per config row-sharded over all ranks (gpk/shard.py: rows of every product
    per rank, RCCL all-gathers / all-reduces inside the step graph).  value = steps/s of the
    single problem (strong scaling).  C5_split: one Kronecker factor inverted per rank half,
    broadcast over RCCL (GPK_FLAG_SPLIT_FACTORS) instead of both factors on every rank.
    make_sharded(cid, flags) / make_single(cid): solver factories (the dry run passes stand-ins,
    so the launcher tests run this very code on CPU)."""
    from gpk import replicas
    from gpk.shard import plan_collectives
    if make_sharded is None:
        from gpk import shard
        from gpk._lib import GPK_FLAG_SPLIT_FACTORS
        from gpk.problems import make_solver
        make_sharded = lambda cid, flags: shard.make_sharded_solver(cid, ctx, seed=0, flags=flags)  # noqa: E731
        make_single = lambda cid: make_solver(cid, seed=0)  # noqa: E731
        split_flag = GPK_FLAG_SPLIT_FACTORS
    else:
        split_flag = 1
    out, single = {}, {}
    for key in configs:
        cid = key.split("_")[0]
        flags = split_flag if key.endswith("_split") else 0
        steps = a.sharded_steps if cid == "C4" else max(2, a.sharded_steps // 10)
        STAGE["name"] = f"sharded {key}: create"
        s = make_sharded(cid, flags)
        plan = s.shard_plan() if hasattr(s, "shard_plan") else None
        try:
            STAGE["name"] = f"sharded {key}: prepare + warm-up"
            s.prepare(steps)
            s.step(2)
            s.sync()
            replicas.barrier(ctx)
            STAGE["name"] = f"sharded {key}: {steps} timed steps"
            t0 = time.perf_counter()
            s.step(steps)
            s.sync()
            t1 = time.perf_counter()
            replicas.barrier(ctx)
        finally:
            s.close()
        dt = replicas.max_over_ranks(t1 - t0, ctx)
        out[key] = {"value": steps / dt, "unit": "iters/s", "ms_per_step": dt / steps * 1e3,
                    "steps": steps, "ranks": ctx.world, "plan": plan,
                    "collectives_per_step": None if plan is None else plan_collectives(plan)}
        if cid not in single:
            STAGE["name"] = f"sharded {key}: single-GPU reference on rank 0"
            single[cid] = single_gpu_reference(lambda: make_single(cid), steps, ctx)
        out[key].update(single[cid])
        out[key]["speedup_vs_1gpu"] = single[cid]["single_gpu_ms_per_step"] / out[key]["ms_per_step"]
        STAGE["name"] = f"sharded {key}: collective latency"
        out[key]["ceiling"] = strong_scaling_ceiling(out[key], collective_latency_us(ctx, cid), ctx.world)
    # C5 is reported both ways: both factors inverted on every rank, or one factor
    # per rank half + a broadcast of K^{-1}; the default is the replicated form
    out["C5_default"] = "C5 (replicated inverse); C5_split = GPK_FLAG_SPLIT_FACTORS"
    return out


STAGE = {"name": "start"}   # what the sharded section is doing (reported when it fails)


def single_gpu_reference(make, steps, ctx):
    """The same problem unsharded on ONE GPU (rank 0, its own device; the other ranks wait at the
    barrier): ms per step of `steps` timed steps after a prepared warm-up, the denominator of a
    sharded entry's speedup_vs_1gpu (strong scaling, measured in the same run)."""
    from gpk import replicas
    ms, rep = None, None
    if ctx.rank == 0:
        s = make()
        try:
            s.prepare(steps)
            s.step(2)
            s.sync()
            t0 = time.perf_counter()
            s.step(steps)
            s.sync()
            ms = (time.perf_counter() - t0) / steps * 1e3
            if hasattr(s, "profile_stages"):
                # the part of the step every rank repeats in a sharded run: assembly + the SPD
                # inverse of both factors (+ the step constants), HIP events per stage
                st = s.profile_stages(3)
                rep = sum(st.get(k, 0.0) for k in ("prep", "assemble", "spd_inverse")) / 1e3
        finally:
            s.close()
    # every rank gets rank 0's time (the others contribute 0 to the MAX): each rank computes the
    # same speedup and leaves the section together
    ms = replicas.max_over_ranks(ms if ms is not None else 0.0, ctx)
    rep = replicas.max_over_ranks(rep if rep is not None else -1.0, ctx)
    return {"single_gpu_ms_per_step": ms, "single_gpu_steps": steps,
            "single_gpu_replicated_ms": rep if rep >= 0.0 else None}


def collective_latency_us(ctx, cid, iters=20):
    """The price of one of the sharded step's collectives on this group, measured here: an
    all-gather of the config's row block (h rows x P columns of fp64 per rank: the R / U
    gathers) and an all-reduce of the step's reduction vector size, torch.distributed on the
    same devices and backend (RCCL over xGMI on GPU ranks), average of `iters` after a warm-up."""
    from gpk import replicas
    if ctx.world == 1:
        return None
    import torch
    import torch.distributed as dist
    from gpk.problems import CONFIGS
    n = CONFIGS[cid]["n"]
    m = 32 * ctx.world
    p = (n + m - 1) // m * m
    dev = f"cuda:{ctx.local}" if ctx.backend == "nccl" else "cpu"
    blk = torch.zeros(p // ctx.world * p, dtype=torch.float64, device=dev)
    parts = [torch.empty_like(blk) for _ in range(ctx.world)]
    red = torch.zeros(2 + 6 * 64 + 2 * (p // 16) ** 2, dtype=torch.float64, device=dev)

    def timed(fn):
        fn()
        if dev != "cpu":
            torch.cuda.synchronize()
        replicas.barrier(ctx)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        if dev != "cpu":
            torch.cuda.synchronize()
        return replicas.max_over_ranks((time.perf_counter() - t0) / iters * 1e6, ctx)
    return {"allgather_us": timed(lambda: dist.all_gather(parts, blk)),
            "allreduce_us": timed(lambda: dist.all_reduce(red)),
            "allgather_bytes_per_rank": blk.numel() * 8}


def strong_scaling_ceiling(entry, lat, world):
    """A-priori strong-scaling bound of a sharded entry from measured pieces: T_N >= T_rep +
    (T_1 - T_rep) / N + gathers x t_allgather + t_allreduce, where T_rep (assembly + SPD
    inverse, single GPU) is repeated on every rank and the rest of the 1-GPU step divides
    perfectly over N ranks."""
    t1, rep, plan = entry.get("single_gpu_ms_per_step"), entry.get("single_gpu_replicated_ms"), entry.get("plan")
    if not t1 or rep is None or plan is None or lat is None:
        return None
    ngather = sum(1 for tok in plan.split() if tok.startswith("g"))
    coll_ms = (ngather * lat["allgather_us"] + lat["allreduce_us"]) / 1e3
    tn = rep + (t1 - rep) / world + coll_ms
    return {"replicated_ms": rep, "parallel_ms_per_rank": (t1 - rep) / world, "gathers": ngather,
            "allreduces": 1, "collectives_ms": coll_ms, **lat, "ms_per_step_bound": tn,
            "speedup_ceiling": t1 / tn}


def dry_run_sharded_section(a, ctx):
    """--dry-run --dry-run-sharded ok|hang|raise: sharded_section itself on stand-in solvers
    (same barriers, max-over-ranks, single-GPU reference and speedup on every rank); 'hang'
    blocks rank 1's timed steps (a stuck collective), 'raise' fails them.  Tests check that
    bench.py exits 0 on every rank for 'ok' and non-zero otherwise."""
    mode = a.dry_run_sharded

    class Sharded(_DryRunSolver):
        def step(self, n):
            if ctx.rank == 1 and mode == "hang" and n > 2:
                time.sleep(3600)
            if ctx.rank == 1 and mode == "raise" and n > 2:
                raise RuntimeError("stand-in collective failed")
            return super().step(n)

    return sharded_section(a, ctx, configs=("C4", "C5_split"),
                           make_sharded=lambda cid, flags: Sharded(ctx.rank),
                           make_single=lambda cid: _DryRunSolver(0))


def kernel_roofline(s, cfg, iters):
    """Per-kernel device timings (HIP events on the library's stream); the dominant kernel =
    largest device time per step, priced against its roofline."""
    n = cfg["n"]
    T = (n + 31) // 32
    kern = {}
    spd = "spd_chain" if s.inverse_path() in ("chain", "chain_aug") else "sweep"
    for name in ([spd, "gemm_B", "pgrad", "assemble"] if cfg["dim"] == 2 else [spd, "assemble"]):
        us, fl, by = s.bench_kernel(name, iters)
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
    roof["traffic"], roof["traffic_source"] = pmc_traffic(PMC_KERNEL[dom])
    roof["avg_launch_us"] = d["us"]
    roof["alg_flops_per_launch"] = d["flops"]
    roof["alg_bytes_per_launch"] = d["bytes"]
    # the step's assembly launch at this config, priced at the bytes it really moves: with the
    # chain inverse that is the class-value launch (K and D at every distance class; the chain
    # gathers K itself), a latency-bound launch whose GB/s is small by construction -- the
    # HBM-bound K-assembly is measured at C5 size (large_factors.assembly)
    a = kern.get("assemble")
    asm = None
    if a:
        asm = {"kernel": "class_eval_kernel" if s.inverse_path() in ("chain", "chain_aug", "chain_multi")
               else "assemble", "us": a["us"], "bytes": a["bytes"],
               "hbm_gbs": a["bytes"] / (a["us"] * 1e-6) / 1e9}
    return roof, {k: round(v["us"], 3) for k, v in kern.items()}, asm


class _DryRunSolver:
    """--dry-run: a stand-in with the solver's stepping interface and no GPU (tests of the
    launcher / rank plumbing on CPU).  Its numbers are not measurements."""

    def __init__(self, seed):
        self.seed = seed

    def prepare(self, n):
        pass

    def step(self, n):
        time.sleep(1e-4 * n)
        return [float(self.seed)] * n

    def sync(self):
        pass

    def graph_mode(self):
        return False, 0

    def inverse_path(self):
        return "dry-run"

    def close(self):
        pass


def spawn_ranks(n):
    """One process per GPU, started before this process touches a GPU (children get the
    torch.distributed.run environment); exits with the worst child status."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    sys.exit(bad[0] if bad else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-blas-threads", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-no-warmup", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--step1-calls", type=int, default=200)
    ap.add_argument("--no-prepare-warmup", action="store_true",
                    help="run the warm-up steps without a prepared whole-call graph (A/B)")
    ap.add_argument("--no-large", action="store_true", help="skip the C5-size MFMA section")
    ap.add_argument("--no-sharded", action="store_true", help="N > 1: skip the row-sharded section")
    ap.add_argument("--sharded-steps", type=int, default=50)
    ap.add_argument("--train-warmup", type=int, default=200,
                    help="Adam steps before the train_regime timing (after the timed batch)")
    ap.add_argument("--sharded-timeout", type=float, default=240.0)
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/rank plumbing only: gloo, stand-in solver, no GPU (tests)")
    ap.add_argument("--dry-run-sharded", choices=["ok", "hang", "raise"], default=None,
                    help=argparse.SUPPRESS)  # with --dry-run: a stand-in sharded section (tests)
    a = ap.parse_args()
    if a.cpu_baseline_only:
        print(json.dumps(cpu_baseline(a.config, a.cpu_seconds, a.cpu_threads, warmup=not a.cpu_no_warmup,
                                      blas_threads=a.cpu_blas_threads)), flush=True)
        return
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        return spawn_ranks(a.gpus)
    if env_world is not None and int(env_world) != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={env_world}")

    from gpk import replicas
    from gpk.problems import CONFIGS, make_solver
    ctx = replicas.init("gloo" if a.dry_run else "nccl")
    world, rank, local = ctx.world, ctx.rank, ctx.local
    cfg = CONFIGS[a.config]
    s = _DryRunSolver(rank) if a.dry_run else make_solver(a.config, seed=rank, device=local)
    s.prepare(a.steps)                   # every graph the timed call can launch, built untimed
    if a.warmup > 1 and not a.no_prepare_warmup:
        s.prepare(a.warmup)              # ... and the warm-up call's (one graph launch, not W)
    s.step(a.warmup)                     # warm-up steps
    s.sync()
    replicas.barrier(ctx)
    t0 = time.perf_counter()
    fast_graph, rb0 = s.graph_mode()     # graph the timed batch starts on (refinement gate closed?)
    losses = s.step(a.steps)             # exactly K steps (returns once their losses are final)
    s.sync()                             # ... and the device has finished the last update
    t1 = time.perf_counter()
    replicas.barrier(ctx)
    fast_end, rb1 = s.graph_mode()       # graph it ends on; chunks rerun inside the timed batch
    rollbacks = rb1 - rb0
    dt = replicas.max_over_ranks(t1 - t0, ctx)
    value = world * a.steps / dt

    extra = {}
    if not a.dry_run:
        # the training regime (model_GP_solver_2d.py:285-332 runs nepoch steps): the same
        # step(K) call after >= 200 more Adam steps, with the graph it ran on (the refinement gate
        # follows the params, so the first 25 steps alone do not show a long run's rate)
        s.step(a.train_warmup)
        s.sync()
        tr_fast, tr_rb0 = s.graph_mode()
        t = time.perf_counter()
        s.step(a.steps)
        s.sync()
        dtr = time.perf_counter() - t
        tr_fast_end, tr_rb1 = s.graph_mode()
        extra["train_regime"] = {"value": a.steps / dtr, "unit": "iters/s", "ms_per_step": dtr / a.steps * 1e3,
                                 "steps": a.steps, "after_steps": a.warmup + a.steps + a.train_warmup,
                                 "step_graph": {"fast": bool(tr_fast), "fast_at_end": bool(tr_fast_end),
                                                "rollbacks": int(tr_rb1 - tr_rb0)}}
        # the reference's loop shape: one step() call per iteration (model_GP_solver_2d.py:285-300)
        s.step(5)
        s.sync()
        t = time.perf_counter()
        for _ in range(a.step1_calls):
            s.step(1)
        s.sync()
        extra["step1_per_call"] = {"value": a.step1_calls / (time.perf_counter() - t), "unit": "iters/s",
                                   "calls": a.step1_calls}
        # fp64 SPD inverse rate.  The path forms K^{-1} itself (Gauss-Jordan sweeps with Cholesky
        # pivots: the log-det gradient needs c N/2 K^{-1}), so what is timed is potrf + potri
        # together, priced at n^3 flops per Kronecker factor (potrf n^3/3 + potri 2n^3/3); there is
        # no separate potrf launch to time alone
        inv_us = s.time_spd_inverse(20)
        n = cfg["n"]
        nfac = 2 if cfg["dim"] == 2 else 1
        extra["spd_inverse_gflops"] = nfac * n ** 3 / (inv_us * 1e-6) / 1e9
        extra["spd_inverse_us"] = inv_us
        roof, kus, asm = kernel_roofline(s, cfg, a.kernel_iters)
        extra["roofline"] = roof
        extra["kernels_us"] = kus
        extra["assembly"] = asm
    final_loss = float(losses[-1])
    path = s.inverse_path()
    s.close()

    failed = None
    if world > 1 and (a.dry_run_sharded or (not a.dry_run and not a.no_sharded)):
        # strong scaling of ONE problem.  A failure or a stuck collective is a FAILED run: the
        # line is still printed (rank 0, the replicas' value + the error), the failing rank and
        # stage go to stderr, and the process exits non-zero -- never a clean-looking rc 0.
        done = threading.Event()
        result = {}

        def watchdog():
            if not done.wait(a.sharded_timeout):
                msg = f"rank {rank}: timeout after {a.sharded_timeout:.0f} s in stage '{STAGE['name']}'"
                print(f"bench.py: sharded section FAILED: {msg}", file=sys.stderr, flush=True)
                if rank == 0:
                    result["sharded"] = {"error": msg}
                    emit(a, value, dt, world, fast_graph, fast_end, rollbacks, final_loss, path, extra, result)
                os._exit(3)   # (no re-exec, no cleanup: a collective may hold the GPU)
        threading.Thread(target=watchdog, daemon=True).start()
        try:
            if a.dry_run_sharded:
                result["sharded"] = dry_run_sharded_section(a, ctx)
            else:
                result["sharded"] = sharded_section(a, ctx)
        except Exception as e:
            failed = f"rank {rank}: {type(e).__name__}: {e} in stage '{STAGE['name']}'"
            print(f"bench.py: sharded section FAILED: {failed}", file=sys.stderr, flush=True)
            result["sharded"] = {"error": failed}
        done.set()
        extra.update(result)

    if rank == 0 and world == 1 and not a.dry_run:
        if not a.no_large:
            try:
                extra["large_factors"] = large_factors()
            except Exception as e:  # reported, never required
                extra["large_factors"] = {"error": f"{type(e).__name__}: {e}"}
        if not a.no_cpu_baseline:
            extra["cpu_baseline"] = cpu_baseline_child(a.config, a.cpu_seconds, a.cpu_threads)
            extra["cpu_baseline_1core"] = cpu_baseline_child(a.config, a.cpu_seconds, 1)

    if rank == 0:
        emit(a, value, dt, world, fast_graph, fast_end, rollbacks, final_loss, path, extra)
    if failed:
        sys.exit(3)
    replicas.shutdown(ctx)


def emit(a, value, dt, world, fast_graph, fast_end, rollbacks, final_loss, path, extra, more=None):
    from gpk.problems import CONFIGS
    cfg = CONFIGS[a.config]
    n = cfg["n"]
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
        "data": ("dry-run stand-in solver, NOT a measurement" if a.dry_run else
                 "synthetic: reference grid/source/boundary of poisson_2d-sin_sin, U ~ 0.1 N(0,1) seeded per rank"),
        "config": {"workload": f"{a.config}: 2D Poisson 256x256 Kronecker grid, Matern52_Cos_1d, Q=30, fp64"
                   if a.config == "C4" else a.config,
                   "grid": [n, n] if cfg["dim"] == 2 else [n], "Q": 30, "kernel": cfg["kernel"],
                   "equation": cfg["equation"],
                   "parallelism": f"replicas x{world} (one independent problem per GPU)"},
        "inverse_path": path,
        "spd_inverse_gflops": extra.get("spd_inverse_gflops"),
        "spd_inverse_flops": "n^3 per Kronecker factor = potrf n^3/3 + potri 2n^3/3 (K^{-1} formed, "
                             "the log-det gradient needs it); the metric's 'Cholesky GFLOP/s'",
        "spd_inverse_us": extra.get("spd_inverse_us"),
        "roofline": extra.get("roofline"),
        "kernels_us": extra.get("kernels_us"),
        "assembly": extra.get("assembly"),
        "train_regime": extra.get("train_regime"),
        "step1_per_call": extra.get("step1_per_call"),
        "cpu_baseline": extra.get("cpu_baseline"),
        "cpu_baseline_1core": extra.get("cpu_baseline_1core"),
        "large_factors": extra.get("large_factors"),
        "sharded": (more or extra).get("sharded"),
        "final_loss": final_loss,
        # step graph of the timed batch: "fast" = refinement GEMM stages left out (gate closed,
        # checked every step; a step needing refinement reruns its 64-step chunk on the full
        # graph, counted in rollbacks); "fast_at_end" = the graph the last chunk ran
        "step_graph": {"fast": bool(fast_graph), "fast_at_end": bool(fast_end), "rollbacks": int(rollbacks)},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
