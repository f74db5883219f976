set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "big_spd or c2_size" -x -q --timeout 120 --timeout-method thread > gpurun_out/q9_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/q9_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/q9_pytest.log | head -30; exit 1; fi
timeout -k 10 300 python tools/spd_pieces.py 2048,4096 both > gpurun_out/q9_pieces.txt 2>&1 || { cat gpurun_out/q9_pieces.txt; exit 1; }
cat gpurun_out/q9_pieces.txt
for c in C2 C5; do timeout -k 10 200 python tools/run_steps.py --config $c --steps 10 > gpurun_out/q9_$c.txt 2>&1 || { cat gpurun_out/q9_$c.txt; exit 1; }; cat gpurun_out/q9_$c.txt; done
