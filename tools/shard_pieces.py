"""Measured single-GPU pieces of the strong-scaling bound: per config, the
unsharded step (ms), its replicated part (prep + assembly + SPD inverse of both factors: every
rank of a sharded run repeats it), and a ONE-rank RCCL sharded handle of the same problem (its
plan and ms/step: the sharded step's own overheads -- row-sliced descriptors, whole 'f' stages,
in-graph collectives on one rank).
    python tools/shard_pieces.py [C4 C5]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk import replicas, shard
from gpk.problems import make_solver


def timed(s, steps):
    s.prepare(steps)
    s.step(2)
    s.sync()
    t0 = time.perf_counter()
    s.step(steps)
    s.sync()
    return (time.perf_counter() - t0) / steps * 1e3


out = {}
for cid in (sys.argv[1:] or ["C4", "C5"]):
    steps = 200 if cid == "C4" else 5
    s = make_solver(cid, seed=0)
    try:
        ms = timed(s, steps)
        st = s.profile_stages(5 if cid == "C4" else 2)
        path = s.inverse_path()
    finally:
        s.close()
    rep = sum(st.get(k, 0.0) for k in ("prep", "assemble", "spd_inverse")) / 1e3
    r = shard.make_sharded_solver(cid, replicas.Ctx(1, 0, 0, ""), seed=0)
    try:
        plan = r.shard_plan()
        ms1 = timed(r, steps)
        path1 = r.inverse_path()
    finally:
        r.close()
    out[cid] = {"single_ms": ms, "inverse_path": path, "stages_us": st, "replicated_ms": rep,
                "sharded_1rank_ms": ms1, "sharded_path": path1, "plan": plan,
                "gathers": sum(1 for t in plan.split() if t.startswith("g")), "allreduces": 1}
    print(cid, json.dumps(out[cid]), flush=True)
