#!/bin/bash
# round 4: plain C5 stage products on rocBLAS (libgpk.so) vs all on gemm_huge_kernel (libgpk_ab.so):
# the C5-size GPU tests first, then the C5 step (bench.py large_factors) interleaved
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
L=gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_accuracy.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/libgemm_tests.log 2>&1 || { tail -30 gpurun_out/r4/libgemm_tests.log; exit 1; }
tail -2 gpurun_out/r4/libgemm_tests.log
for rep in 1 2; do
  for lib in libgpk.so libgpk_ab.so; do
    GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-iters 5 --step1-calls 5 > gpurun_out/ab.json 2>gpurun_out/r4/libgemm_bench.err || { tail -20 gpurun_out/r4/libgemm_bench.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); lf=d['large_factors']; print('$lib', 'C4', round(d['value'],1), 'C5 step_ms', round(lf['step_ms'],3), 'inverse_ms', round(lf['spd_inverse_ms'],3), 'gemm_B_us', round(lf['gemm_B_us'],1))"
  done
done
