#!/bin/bash
# round 4: the driver's 20-step line after 5 vs 50 warm-up steps (same box, interleaved)
set -o pipefail
mkdir -p gpurun_out/r4
for rep in 1 2 3; do
  for w in 5 50 200; do
    timeout -k 10 200 python bench.py --steps 20 --warmup $w --no-cpu-baseline --no-large --kernel-iters 5 --step1-calls 5 > gpurun_out/ab.json 2>/dev/null || { echo bench failed; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('C4 steps 20 warmup $w', round(d['value'],1))"
  done
done
