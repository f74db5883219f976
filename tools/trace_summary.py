"""Median duration per (kernel, grid) of a rocprofv3 --kernel-trace run.

    python tools/trace_summary.py <rocprof output dir>
"""
import collections
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    grid = (int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    d[(name, grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for (name, grid), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{name[:60]:60s} grid {str(grid):18s} n {len(v):6d}  median {v[len(v) // 2] / 1000:8.2f} us  min {v[0] / 1000:8.2f}")
