# round 5: the C5 kernel-parameter split on both axes (exact-field yardstick, dd device fields)
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp OMP_NUM_THREADS=16
for ax in 2 1; do
  timeout -k 10 400 python -u tools/c5_kp_split.py C5 $ax > gpurun_out/r5/contract_dd_C5_$ax.log 2>&1 || { tail -20 gpurun_out/r5/contract_dd_C5_$ax.log; exit 1; }
  grep -B30 -A14 '"contraction"' gpurun_out/r5/contract_dd_C5_$ax.log
done
