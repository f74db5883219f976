"""Per-step device timeline of a tools/warmup_trace.py kernel trace: each step starts at its
class_eval_kernel dispatch; prints, per bucket of step indices, the mean step period (start to
next start), the step's busy span (first start to last end) and each kernel's mean duration.
    python tools/warmup_analyze.py <rocprofv3 output dir>"""
import collections
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = []
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].replace("gpk::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
steps, cur = [], None
for st, en, nm in rows:
    if nm.startswith("class_eval"):
        cur = []
        steps.append(cur)
    if cur is not None:
        cur.append((st, en, nm))
print(f"{len(steps)} steps")
buckets = [(0, 5), (5, 25), (25, 45), (45, 85), (85, 125), (125, 205), (205, 10 ** 9)]
for b0, b1 in buckets:
    sel = list(range(b0, min(b1, len(steps) - 1)))
    if not sel:
        continue
    per = [steps[i + 1][0][0] - steps[i][0][0] for i in sel]
    span = [max(e for _, e, _ in steps[i]) - steps[i][0][0] for i in sel]
    kd = collections.defaultdict(list)
    for i in sel:
        c = collections.Counter()
        for st, en, nm in steps[i]:
            kd[(nm, c[nm])].append(en - st)
            c[nm] += 1
    ks = " ".join(f"{nm}#{k}:{sum(v) / len(v) / 1e3:.2f}" for (nm, k), v in sorted(kd.items(), key=lambda kv: kv[0]))
    print(f"steps {b0:4d}-{min(b1, len(steps) - 1) - 1:4d}: period {sum(per) / len(per) / 1e3:7.2f} us  "
          f"span {sum(span) / len(span) / 1e3:7.2f} us  kernels/step {len(steps[sel[0]])}  | {ks}")
