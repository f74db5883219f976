#!/bin/bash
# chain_multi with L_k^{-1} as self-validating words (no pivot flags): C2 tests, timeline, A/B vs HEAD
set -o pipefail
mkdir -p gpurun_out/r3lw
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain_multi.py tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3lw/pytest.log 2>&1 || { tail -30 gpurun_out/r3lw/pytest.log; exit 1; }
tail -1 gpurun_out/r3lw/pytest.log
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
GPK_LIB_PATH=$L/libgpk_trace.so timeout -k 10 200 python tools/timeline.py --config C2 --steps 5 > gpurun_out/r3lw/c2.txt 2>&1 || exit 1
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_ab.so; do
    GPK_LIB_PATH=$L/$lib timeout -k 10 200 python bench.py --config C2 --steps 100 --warmup 10 --no-cpu-baseline --no-large --kernel-iters 5 --step1-calls 5 > gpurun_out/ab.json 2>/dev/null || { echo C2 bench failed; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('C2', '$lib', round(d['ms_per_step'],4))"
  done
done
