#!/bin/bash
# driver-shape bench with and without a prepared whole-call graph for the warm-up steps
set -o pipefail
mkdir -p gpurun_out/warm
export TMPDIR=/tmp
for rep in 1 2 3 4; do
  for fl in "" "--no-prepare-warmup"; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-large --kernel-iters 5 --step1-calls 50 $fl > gpurun_out/warm/b.json 2>/dev/null || { echo bench failed; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/warm/b.json')); print('${fl:-prepared}', round(d['value'],1))"
  done
done
