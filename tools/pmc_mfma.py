"""fp64 MFMA utilisation per kernel from rocprofv3 counter passes (MI355X_MICROARCH.md §rocprofv3).

Inputs (one command profiled three times, each pass a run of its own):
  --trace DIR   rocprofv3 --kernel-trace --stats (average duration per kernel)
  --mops DIR    rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
  --util DIR    rocprofv3 --pmc MfmaUtil   (the derived metric: sum(BUSY) / (max(GUI_ACTIVE) * SIMDs))
Per kernel (mean over its dispatches):
  mfma_flops        = SQ_INSTS_VALU_MFMA_MOPS_F64 * 512      (fp64 MFMA flops the hardware executed)
  counter_tflops    = mfma_flops / average duration (trace)   vs the 78.6 TF/s fp64 matrix peak
  mfma_busy_pct     = MfmaUtil                                (matrix-pipe busy share of the kernel's
                                                               active cycles, all 1024 SIMDs)
usage: python tools/pmc_mfma.py --trace D --mops D --util D --out profiles/r3_pmc_mfma_<cfg>.json
"""
import argparse
import collections
import csv
import glob
import json
import os

PEAK_F64 = 78.6e12


def kname(full):
    """'void gpk::(anonymous namespace)::k<1>(args)' -> 'gpk::k<1>'"""
    return full.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")


def _name(r):
    return kname(r["Kernel_Name"])


def counters(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        # one row per (dispatch, counter[, instance]): sum instances per dispatch first
        key = (r.get("Dispatch_Id") or r.get("Correlation_Id") or "", _name(r))
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    for (disp, name), cs in per.items():
        for c, v in cs.items():
            acc[name][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"dispatches": len(next(iter(cs.values())))}
            for k, cs in acc.items()}


def durations(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(f)):
        out[kname(r["Name"])] = (float(r["AverageNs"]), int(r["Calls"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--mops", required=True)
    ap.add_argument("--util", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    dur, mops, util = durations(a.trace), counters(a.mops), counters(a.util)
    res = {}
    for k, c in mops.items():
        fl = c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) * 512.0
        if fl <= 0:
            continue
        ns = dur.get(k, (None, 0))[0]
        e = {"mfma_flops_per_dispatch": fl, "dispatches": c["dispatches"],
             "busy_cycles": c.get("SQ_VALU_MFMA_BUSY_CYCLES"), "gui_active": c.get("GRBM_GUI_ACTIVE"),
             "mfma_busy_pct": util.get(k, {}).get("MfmaUtil")}
        if ns:
            e["avg_ns"] = ns
            e["counter_tflops"] = fl / (ns * 1e-9) / 1e12
            e["frac_of_peak"] = fl / (ns * 1e-9) / PEAK_F64
        res[k] = e
    with open(a.out, "w") as f:
        json.dump({"label": a.label,
                   "source": "rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES "
                             "GRBM_GUI_ACTIVE | --pmc MfmaUtil | --kernel-trace --stats, separate runs "
                             "of the same command; flops = MOPS_F64 * 512; peak 78.6 TF/s fp64",
                   "kernels": res}, f, indent=1)
    for k, e in sorted(res.items(), key=lambda kv: -kv[1]["mfma_flops_per_dispatch"]):
        print(f"{k[:60]:60s} {e['mfma_flops_per_dispatch']:.3e} flop  "
              f"{e.get('counter_tflops', float('nan')):7.2f} TF/s  busy {e['mfma_busy_pct']}")


if __name__ == "__main__":
    main()
