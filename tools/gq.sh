set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "big_spd" -x -q --timeout 120 --timeout-method thread > gpurun_out/q7_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/q7_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/q7_pytest.log | head -30; exit 1; fi
timeout -k 10 300 python tools/spd_pieces.py 4096 wide > gpurun_out/q7_pieces.txt 2>&1 || { cat gpurun_out/q7_pieces.txt; exit 1; }
cat gpurun_out/q7_pieces.txt
timeout -k 10 200 python tools/run_steps.py --config C5 --steps 10 > gpurun_out/q7_c5.txt 2>&1 || { cat gpurun_out/q7_c5.txt; exit 1; }
cat gpurun_out/q7_c5.txt
