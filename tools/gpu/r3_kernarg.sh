#!/bin/bash
# C4 bench with kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs default, interleaved
set -o pipefail
export TMPDIR=/tmp
for rep in 1 2 3; do
  for e in 0 1; do
    if [ $e = 1 ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
    for a in "--steps 20 --warmup 5" "--steps 500 --warmup 20"; do
      timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-large --kernel-iters 5 --step1-calls 100 > /tmp/b.json 2>/dev/null || { echo bench failed; exit 1; }
      python3 -c "import json; d=json.load(open('/tmp/b.json')); print('devkernarg=$e', '$a', round(d['value'],1), round(d['step1_per_call']['value'],1))"
    done
  done
done
