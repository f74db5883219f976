# round 5: double-double phase / radial arguments in the device field evaluation, against the
# exact-field yardstick -- the whole GPU suite (parity log -> gpurun_out/r5/parity.jsonl), then
# the C5 kernel-parameter split on both axes
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp GPK_PARITY_LOG=$PWD/gpurun_out/r5/parity.jsonl
rm -f $GPK_PARITY_LOG
timeout -k 10 800 python -u -m pytest tests -m gpu --maxfail=12 -v --timeout 300 --timeout-method thread > gpurun_out/r5/dd_suite.log 2>&1; rc=$?
tail -3 gpurun_out/r5/dd_suite.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/r5/dd_suite.log | head -30; exit 1; }
export OMP_NUM_THREADS=16
for ax in 2 1; do
  timeout -k 10 400 python -u tools/c5_kp_split.py C5 $ax > gpurun_out/r5/contract_dd_C5_$ax.log 2>&1 || { tail -20 gpurun_out/r5/contract_dd_C5_$ax.log; exit 1; }
  grep -A14 '"contraction"' gpurun_out/r5/contract_dd_C5_$ax.log
done
