#!/bin/bash
# round 4: C2 (chain_multi) tests, then ms/step A/B of libgpk.so vs libgpk_ab.so, interleaved
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
L=gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "multi or C2 or 2048 or timeout" > gpurun_out/r4/c2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4/c2_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r4/c2_tests.log | head -20; exit $rc; }
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_ab.so; do
    GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python bench.py --config C2 --steps 200 --warmup 10 --no-cpu-baseline --no-large --kernel-iters 5 --step1-calls 5 > gpurun_out/ab.json 2>/dev/null || { echo C2 bench failed; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('C2', '$lib', round(d['ms_per_step'],4))"
  done
done
