# round 5: double-double kernel-parameter contraction -- tests, C5 split, C5 step time A/B
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp GPK_PARITY_LOG=$PWD/gpurun_out/r5/parity_ddc.jsonl
rm -f $GPK_PARITY_LOG
timeout -k 10 600 python -u -m pytest tests/test_gpu_accuracy.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/ddc_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r5/ddc_tests.log | tail -20
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r5/ddc_tests.log | head -30; exit 1; }
python3 tools/parity_summary.py $GPK_PARITY_LOG gpurun_out/r5/parity_ddc.json ddc | sort -k4 | tail -12
export OMP_NUM_THREADS=16
for ax in 2 1; do
  timeout -k 10 400 python -u tools/c5_kp_split.py C5 $ax > gpurun_out/r5/contract_ddc_C5_$ax.log 2>&1 || { tail -20 gpurun_out/r5/contract_ddc_C5_$ax.log; exit 1; }
  grep -A14 '"contraction"' gpurun_out/r5/contract_ddc_C5_$ax.log | head -4
done
timeout -k 10 300 python -u tools/ab_flags.py --config C5 --flags 0 262144 --reps 1 2>&1 | tail -2 || true
