"""bench.py's multi-GPU launcher on CPU (gloo, --dry-run stand-in solver, no GPU): `--gpus N`
without a launcher starts N ranks of itself with the torch.distributed.run environment, the
ranks form one process group (world N), and rank 0 prints ONE JSON line with n_gpus = N;
launched by torch.distributed.run, --gpus must equal WORLD_SIZE."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "4", "--warmup", "1",
                        "--dry-run"], env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["steps"] == 4 and out["value"] > 0
    assert "NOT a measurement" in out["data"]


def test_gpus_must_match_world_size():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "2", "--dry-run"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


@pytest.mark.parametrize("config", ["C1", "C3"])
def test_cpu_baseline_child_1d_and_2d(config):
    """The bench's cpu_baseline leg (the oracle on the host, a child process) runs 1D and 2D
    configs and reports a bounded sample: at least one full step, the thread counts used."""
    sys.path.insert(0, ROOT)
    import bench
    r = bench.cpu_baseline_child(config, 0.2, 2)
    assert r.get("value") and r["value"] > 0, r
    assert r["cores"] == 2 and r["kind"] == "port" and config in r["sample"]


def test_sharded_section_ok_exits_zero():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--dry-run", "--dry-run-sharded", "ok"], env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    # bench.sharded_section itself ran on stand-in solvers: every sharded entry carries the same
    # problem's single-GPU time (rank 0, same run, shared with every rank) and the strong-scaling
    # speedup over it, and every rank left the section (exit 0)
    for key in ("C4", "C5_split"):
        d = out["sharded"][key]
        assert d["ranks"] == 2
        assert d["single_gpu_ms_per_step"] > 0 and d["speedup_vs_1gpu"] > 0, d
        assert abs(d["speedup_vs_1gpu"] - d["single_gpu_ms_per_step"] / d["ms_per_step"]) < 1e-9


@pytest.mark.parametrize("mode", ["hang", "raise"])
def test_sharded_section_failure_exits_nonzero(mode):
    """A stuck collective (the watchdog fires) or a failing rank in the sharded section makes
    bench.py --gpus 2 exit non-zero, naming the rank and the stage on stderr; rank 0 still prints
    its line, with the error in `sharded`."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--dry-run", "--dry-run-sharded", mode, "--sharded-timeout", "8"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0, (r.stdout, r.stderr)
    assert "sharded section FAILED" in r.stderr, r.stderr
    assert "rank 1" in r.stderr or "rank 0" in r.stderr, r.stderr
    assert "sharded C4" in r.stderr, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert "error" in json.loads(lines[0])["sharded"]
