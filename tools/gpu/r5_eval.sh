# round 5: the chain launch's fused class evaluation -- bitwise test, A/B against NO_CHAIN_EVAL,
# and the C4 timeline (probe build)
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dclass.py -k "fused_eval or class_path" -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5/eval_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r5/eval_tests.log | tail -20
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r5/eval_tests.log | head -30; exit 1; }
timeout -k 10 300 python -u tools/ab_flags.py --config C4 --flags 0 131072 --reps 3
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib/libgpk_trace.so
GPK_LIB_PATH=$L timeout -k 10 120 python -u tools/timeline.py --config C4 --steps 5 > gpurun_out/r5/timeline_C4_eval.txt 2>&1 || { cat gpurun_out/r5/timeline_C4_eval.txt; exit 1; }
head -12 gpurun_out/r5/timeline_C4_eval.txt
