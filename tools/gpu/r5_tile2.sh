# round 5: the pipelined 128x128 tile inside libgpk (gemm_huge_kernel) -- probe rates, GEMM tests,
# C5 / C4 step times; outputs under gpurun_out/r5
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
#timeout -k 10 300 tools/probes/bin/gemm_tile_probe 4096 > gpurun_out/r5/tile_probe2.txt 2>&1 || { cat gpurun_out/r5/tile_probe2.txt; exit 1; }
#cat gpurun_out/r5/tile_probe2.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r5/gemm_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r5/gemm_tests.log
[ $rc -eq 0 ] || exit 1
for c in C5 C4; do timeout -k 10 300 python tools/run_steps.py --config $c --steps 20 > gpurun_out/r5/steps_$c.txt 2>&1 || { cat gpurun_out/r5/steps_$c.txt; exit 1; }; head -3 gpurun_out/r5/steps_$c.txt; done
