# round 5: fp64 contraction rounding vs the exact (long-double) contraction, C5 and C4, both axes
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp OMP_NUM_THREADS=16
for c in "C5 2" "C5 1" "C4 1" "C4 2"; do
  timeout -k 10 600 python -u tools/c5_kp_split.py $c > gpurun_out/r5/contract_${c// /_}.log 2>&1 || { tail -20 gpurun_out/r5/contract_${c// /_}.log; exit 1; }
  grep -A12 '"contraction"' gpurun_out/r5/contract_${c// /_}.log
done
