#!/bin/bash
# round 4: the whole GPU suite on the current tree, then C4 A/B (libgpk.so vs libgpk_ab.so = the
# last committed tree) at the driver's shape and at 500 steps, then the gather A/B (r4_gab.sh)
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
L=gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/all_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r4/all_suite.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r4/all_suite.log | head -30; exit $rc; }
for rep in 1 2; do
  for lib in libgpk.so libgpk_ab.so; do
    for a in "--steps 20 --warmup 5" "--steps 500 --warmup 20"; do
      GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-large --kernel-iters 5 > gpurun_out/ab.json 2>/dev/null || { echo bench failed; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('C4', '$lib', '$a', round(d['value'],1), round(d['step1_per_call']['value'],1))"
    done
  done
done
bash tools/gpu/r4_gab.sh
