# round 5: two-sweep update schedule of the C5 inverse -- tests, A/B, MFMA counters of the update
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp GPK_PARITY_LOG=$PWD/gpurun_out/r5/parity_sched.jsonl
rm -f $GPK_PARITY_LOG
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_accuracy.py -k "quarter or tile128 or c5 or C5 or big" -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/sched_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r5/sched_tests.log | tail -30
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r5/sched_tests.log | head -30; exit 1; }
timeout -k 10 300 python -u tools/c5_inv_sched_ab.py || exit 1
C5="tools/run_steps.py --config C5 --steps 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r5/sched_trace -o t -- python3 $C5 > gpurun_out/r5/sched_trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d gpurun_out/r5/sched_mops -o m -- python3 $C5 > gpurun_out/r5/sched_mops.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc MfmaUtil -f csv -d gpurun_out/r5/sched_util -o u -- python3 $C5 > gpurun_out/r5/sched_util.log 2>&1 || exit 1
python3 tools/pmc_mfma.py --trace gpurun_out/r5/sched_trace --mops gpurun_out/r5/sched_mops --util gpurun_out/r5/sched_util --out gpurun_out/r5/pmc_mfma_c5_sched.json --label "C5 two-sweep schedule: $C5" | grep -E "wide_update|gemm_huge|panel|pivot"
rm -rf gpurun_out/r5/sched_mops gpurun_out/r5/sched_util
