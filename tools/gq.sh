set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/spd_pieces.py 2048,4096 both > gpurun_out/q2_pieces.txt 2>&1 || { cat gpurun_out/q2_pieces.txt; exit 1; }
cat gpurun_out/q2_pieces.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/q2_prof -o c5 -- python3 tools/run_steps.py --config C5 --steps 3 > gpurun_out/q2_prof.log 2>&1 || { tail -20 gpurun_out/q2_prof.log; exit 1; }
python3 tools/trace_summary.py gpurun_out/q2_prof | head -20
