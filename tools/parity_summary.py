"""Collect the GPU parity tests' observed errors (tests/helpers.record_parity lines) into one JSON:
per test and config, the error of every key, its bar, and the LU oracle's own error where known.
usage: python tools/parity_summary.py <parity.jsonl> <out.json> [label]"""
import json
import sys

rows = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
out = {"label": sys.argv[3] if len(sys.argv) > 3 else "",
       "source": "tests/test_gpu_accuracy.py (+ any test calling tests/helpers.record_parity) on an MI355X; "
                 "errors are max-abs / max-abs per key (tests/helpers.rel) against the long-double "
                 "yardstick fixtures tests/golden/ext_<cfg>.npz, preds as relative L2 vs the fp64 oracle",
       "results": rows}
with open(sys.argv[2], "w") as f:
    json.dump(out, f, indent=1)
for r in rows:
    tol = r.get("tol")
    worst = max((v / (tol[k] if isinstance(tol, dict) else tol), k) for k, v in r["errors"].items()) if tol else None
    print(f"{r['test'][:44]:44s} {r['config']:3s} worst error/bar {worst[0]:.3f} ({worst[1]})" if worst else r)
