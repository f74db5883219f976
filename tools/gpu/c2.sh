# C2 per-stage times (64-wide and 128-wide large-factor inverse) + a rocprof kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/run_steps.py --config C2 --steps 50 > gpurun_out/c2_stages.txt 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c2 -o c2 -- python3 tools/run_steps.py --config C2 --steps 10 > gpurun_out/prof_c2.log 2>&1
rc=$?; cat gpurun_out/c2_stages.txt; exit $rc
