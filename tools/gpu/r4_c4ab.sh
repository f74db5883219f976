#!/bin/bash
# round 4: C4 A/B (libgpk.so vs libgpk_ab.so) at the driver's shape and at 500 steps, and C2
# ms/step, interleaved; then the GPU tests that cover the changed kernels
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
L=gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_ab.so; do
    for a in "--steps 20 --warmup 5" "--steps 500 --warmup 20"; do
      GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-large --kernel-iters 5 > gpurun_out/ab.json 2>/dev/null || { echo bench failed; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('C4', '$lib', '$a', round(d['value'],1), round(d['step1_per_call']['value'],1))"
    done
    GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python bench.py --config C2 --steps 200 --warmup 10 --no-cpu-baseline --no-large --kernel-iters 5 --step1-calls 5 > gpurun_out/ab.json 2>/dev/null || { echo C2 bench failed; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('C2', '$lib', round(d['ms_per_step'],4))"
  done
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/c4ab_tests.log 2>&1 || { tail -30 gpurun_out/r4/c4ab_tests.log; exit 1; }
tail -3 gpurun_out/r4/c4ab_tests.log
