# round 5: C4 one-step device timeline (probe build) + the kernel trace of the same steps
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib/libgpk_trace.so
GPK_LIB_PATH=$L timeout -k 10 120 python -u tools/timeline.py --config C4 --steps 5 > gpurun_out/r5/timeline_C4.txt 2>&1 || { cat gpurun_out/r5/timeline_C4.txt; exit 1; }
cat gpurun_out/r5/timeline_C4.txt
