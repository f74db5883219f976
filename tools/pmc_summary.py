"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes per launch.

Corrections per /opt/skills/guides/MI355X_MICROARCH.md §HBM: counters are in KiB; FETCH_SIZE
counts 64 B per 128-B request on gfx950 for wide coalesced reads, so it is doubled ("fetch_x2");
the raw value is kept too because our loads are 8-B-per-lane (uncalibrated width).  Counters come
from the L2 memory side and include Infinity-Cache hits, so at working sets < 256 MiB they are an
upper bound on DRAM bytes.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json> [tree]
(tree: the source tree the passes measured, e.g. its git head -- recorded in the summary so the
bench line's roofline.traffic names what it was measured on)
"""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            # ('void gpk::(anonymous namespace)::k<1>(args)' -> 'gpk::k<1>': the anonymous-namespace
            # kernels of spdinv_big.hip were all lumped into 'gpk::' before)
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            acc[name].append(float(r["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    fetch, write, out = sys.argv[1:4]
    tree = sys.argv[4] if len(sys.argv) > 4 else None
    fr, wr = per_kernel(fetch, "FETCH_SIZE"), per_kernel(write, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fr) | set(wr)):
        fb = fr.get(k, (0.0, 0))[0]
        wb = wr.get(k, (0.0, 0))[0]
        res[k] = {"fetch_bytes_raw": fb, "fetch_bytes_x2": 2 * fb, "write_bytes": wb,
                  "traffic_bytes": 2 * fb + wb, "launches": fr.get(k, (0, 0))[1]}
    with open(out, "w") as f:
        json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) "
                             "of bench.py; traffic_bytes = 2*FETCH + WRITE per launch",
                   "tree": tree, "kernels": res}, f, indent=1)
    for k, v in res.items():
        print(f"{k:40s} fetch {v['fetch_bytes_x2'] / 1e6:9.3f} MB  write {v['write_bytes'] / 1e6:9.3f} MB")


if __name__ == "__main__":
    main()
