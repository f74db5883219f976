set -o pipefail
mkdir -p gpurun_out/r5
export OMP_NUM_THREADS=16
timeout -k 10 1000 python -u tools/step_fields_parity.py C1 C3 C4 C2 C5 --out gpurun_out/r5/step_fields_parity.json
