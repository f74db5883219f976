# round 5: DD contraction diagnostics -- small-size test, then the C5 split on axis 2
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp GPK_PARITY_LOG=$PWD/gpurun_out/r5/parity_ddc2.jsonl
rm -f $GPK_PARITY_LOG
timeout -k 10 300 python -u -m pytest tests/test_gpu_accuracy.py -k "dd_contraction" -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/ddc2_tests.log 2>&1
grep -E "PASSED|FAILED|ERROR|^E " gpurun_out/r5/ddc2_tests.log | head -20
python3 -c "
import json
for l in open('$GPK_PARITY_LOG'):
    r=json.loads(l); print(r['config'], 'dd', {k:'%.2e'%v for k,v in r['errors'].items() if k.startswith('kern')}, 'fp64', {k:'%.2e'%v for k,v in r['fp64_contraction_err'].items() if k.startswith('kern')})
"
export OMP_NUM_THREADS=16
timeout -k 10 400 python -u tools/c5_kp_split.py C5 2 > gpurun_out/r5/contract_ddc_C5_2.log 2>&1 || { tail -20 gpurun_out/r5/contract_ddc_C5_2.log; exit 1; }
grep -A14 '"contraction"' gpurun_out/r5/contract_ddc_C5_2.log
