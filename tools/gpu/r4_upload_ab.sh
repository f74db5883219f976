#!/bin/bash
# round 4: graph upload at instantiation (libgpk.so) vs without (libgpk_ab.so): per-call
# overhead (tools/call_overhead.py) and C4 bench lines at the driver's shape, interleaved
set -o pipefail
mkdir -p gpurun_out/r4
L=gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for lib in libgpk.so libgpk_ab.so; do
  echo "== $lib"
  GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python -u tools/call_overhead.py --reps 20 || { echo overhead failed; exit 1; }
done
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_ab.so; do
    for a in "--steps 20 --warmup 5" "--steps 500 --warmup 20"; do
      GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-large --kernel-iters 5 > gpurun_out/ab.json 2>/dev/null || { echo bench failed; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('C4', '$lib', '$a', round(d['value'],1), round(d['step1_per_call']['value'],1))"
    done
  done
done
