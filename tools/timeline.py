"""One step's device timeline from the probe build (csrc/gpk_trace.h; `make -C ... trace`).

    GPK_LIB_PATH=.../libgpk_trace.so python tools/timeline.py [--config C4] [--steps 3]

Prints, per probed slot, [first arrival, last departure] in microseconds relative to the first
probe of the step (100 MHz device clock, 10 ns resolution), averaged over --steps single steps.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np

NS = 256  # gpk_trace.h TRACE_SLOTS

# single-workgroup probes (gpk_trace.h): "first" = workgroup 0, "last" = the last in the grid
NAMES = {0: "class_eval first wg", 1: "gather pivot wg | chain wg(0,0)", 2: "pivot0 wait done", 3: "pivot0 factor",
         40: "class_sum first wg", 41: "pgrad first wg start", 42: "pg first wg contracted",
         43: "pg group tails", 44: "pg top tail", 45: "pg U plane wg0", 46: "pg finalize",
         47: "pg last grad wg", 48: "pg first wg staged", 49: "class_sum last wg",
         50: "class_eval last wg", 51: "gather last wg", 52: "class_sum wg0 loaded", 53: "chain: last wg done",
         54: "chain: factor-1 pivot chain done", 55: "fin: loads issued", 56: "fin: sums done",
         57: "fin: loss done", 58: "chain last sweep: L word seen", 59: "chain last sweep: L in LDS",
         60: "chain last sweep: products done", 61: "chain last sweep: tile out + done",
         62: "chain last sweep: aug tile out + done", 36: "chain: prefetch missed (first..last)",
         37: "pg group complete (first..last)", 38: "pg U plane last wg"}
for k in range(16):
    NAMES[64 + 4 * k] = f"gemm stage {k} first wg"
    NAMES[65 + 4 * k] = f"  gemm {k} first wg loaded"
    NAMES[66 + 4 * k] = f"  gemm {k} first wg mfma done"
    NAMES[67 + 4 * k] = f"  gemm {k} last wg"
for k in range(16):
    NAMES[128 + k] = f"mc sweep {k}: panel loads issued"
    NAMES[144 + k] = f"mc sweep {k}: L words in"
    NAMES[160 + k] = f"mc sweep {k}: L + panel in LDS"
    NAMES[176 + k] = f"mc sweep {k}: V in LDS"
    NAMES[192 + k] = f"mc sweep {k}: pass-0 published"
    NAMES[208 + k] = f"mc sweep {k}: sweep done"
    NAMES[224 + k] = f"mc sweep {k}: pass-0 products done"
for k in range(16):
    NAMES[4 + k] = f"sweep {k} (pivot wg)"
    NAMES[20 + k] = f"  pivot in sweep {k}"

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C4")
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--flags", type=int, default=0, help="GPK_FLAG_* bits of the handle")
a = ap.parse_args()
if a.config in ("C1", "C2"):  # 1D: gpk_trace.h SLOT_MCP_IN / SLOT_MCP_OUT reuse the GEMM / update slots
    for k in range(16):
        for j in range(4):
            NAMES.pop(64 + 4 * k + j, None)
    for k in range(16):
        NAMES[64 + k] = f"row {k + 1} publishers (sweep {k}): inputs in (first..last)"
        NAMES[240 + k] = f"row {k + 1} publishers (sweep {k}): published (first..last)"
if "GPK_LIB_PATH" not in os.environ:
    os.environ["GPK_LIB_PATH"] = os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd",
                                              "gpk", "_lib", "libgpk_trace.so")
from gpk import _lib, problems  # noqa: E402

lib = _lib.load()
s = problems.make_solver(a.config, seed=0, flags=a.flags)
s.step(20)
U64 = ctypes.c_uint64 * NS
who = []


def who_role(wg, mpos):
    """chain_multi_kernel workgroup -> (macro row R, column pair c0, diagonal tiles) (spdinv.hip multi_role)"""
    g = wg - (1 if wg > mpos else 0)
    if g == 0:
        return (0, -1, "d3")
    r, first = 1, 1
    while first + r <= g:
        first += r
        r += 1
    c0 = g - first
    o4, o5, o6 = (r - 2 if r >= 2 else 0), (r - 3 if r >= 3 else 0), r - 1
    dm = "".join(n for n, o in (("(2R,2R)", o4), ("(2R+1,2R)", o5), ("(2R+1,2R+1)", o6)) if c0 == o)
    return (r, c0, dm)
acc_lo, acc_hi, cnt = np.zeros(NS), np.zeros(NS), np.zeros(NS)
for _ in range(a.steps):
    _lib.check(lib.gpk_trace_reset())
    s.step(1)
    lo, hi = U64(), U64()
    _lib.check(lib.gpk_trace_read(lo, hi, NS))
    if a.config in ("C1", "C2"):  # last publishers (clock << 16 | blockIdx.x), decoded as ids
        raw = [int(v) for v in hi[:]]
        mpos = raw[112] & 0xFFFF
        who.append([(who_role(raw[80 + k] & 0xFFFF, mpos) if raw[80 + k] else None,
                     who_role(raw[96 + k] & 0xFFFF, mpos) if raw[96 + k] else None) for k in range(16)])
        for i in list(range(80, 113)):
            hi[i] = 0
    lo = np.array(lo[:], dtype=np.float64)
    hi = np.array(hi[:], dtype=np.float64)
    valid_lo = lo < 2 ** 63
    t0 = lo[valid_lo].min()
    for i in range(NS):
        if hi[i] > 0 or valid_lo[i]:
            acc_lo[i] += (lo[i] - t0) / 100.0 if valid_lo[i] else np.nan
            acc_hi[i] += (hi[i] - t0) / 100.0 if hi[i] > 0 else np.nan
            cnt[i] += 1
print(f"{a.config} flags {a.flags}: one step, device timeline (us, mean of {a.steps})")
for i in sorted(range(NS), key=lambda i: (acc_lo[i] / max(cnt[i], 1)) if cnt[i] and not np.isnan(acc_lo[i]) else 1e9):
    if cnt[i]:
        l, h = acc_lo[i] / cnt[i], acc_hi[i] / cnt[i]
        print(f"  {str(NAMES.get(i, i)):24s} {l:9.2f} .. {h:9.2f}   ({h - l:7.2f})")
if who:
    print("last publisher of each panel row (macro row R, column pair c0, diagonal tiles held), per step:")
    for k in range(16):
        print(f"  row {k + 1:2d} (sweep {k:2d}): last in " + "; ".join(str(w[k][0]) for w in who)
              + " | last out " + "; ".join(str(w[k][1]) for w in who))
