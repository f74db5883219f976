# large-factor (wide) inverse iteration: its parity tests, C5 stage times, SPD pieces
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest "tests/test_gpu_parity.py::test_loss_grad_big_spd_path" "tests/test_gpu_parity.py::test_big_spd_long_tile_runs" "tests/test_gpu_parity.py::test_big_spd_adam_and_predict_match_small" tests/test_gpu_fullsize.py tests/test_shard.py -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_wide.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error|Timeout" gpurun_out/pytest_wide.log | head -30; exit 1; fi
timeout -k 10 300 python tools/spd_pieces.py 4096 both > gpurun_out/pieces.txt 2>&1 &&
timeout -k 10 200 python tools/run_steps.py --config C5 --steps 10 > gpurun_out/c5_stages.txt 2>&1 || { echo step failed; tail -5 gpurun_out/pieces.txt gpurun_out/c5_stages.txt; exit 1; }
cat gpurun_out/pieces.txt; cat gpurun_out/c5_stages.txt
