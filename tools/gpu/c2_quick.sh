# C2 only: timeline (probe build) + stage times, no tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/timeline.py --config C2 --steps 3 > gpurun_out/tl_c2.txt 2>&1 &&
timeout -k 10 120 python tools/run_steps.py --config C2 --steps 50 > gpurun_out/c2_stages.txt 2>&1 || { echo step failed; tail -5 gpurun_out/tl_c2.txt gpurun_out/c2_stages.txt; exit 1; }
head -1 gpurun_out/c2_stages.txt
