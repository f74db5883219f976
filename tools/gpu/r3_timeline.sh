#!/bin/bash
# device timelines of one C4 and one C2 step from the probe build
set -o pipefail
mkdir -p gpurun_out/r3tl
export TMPDIR=/tmp
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib/libgpk_trace.so
GPK_LIB_PATH=$L timeout -k 10 200 python tools/timeline.py --config C4 --steps 5 > gpurun_out/r3tl/c4.txt 2>&1 &&
GPK_LIB_PATH=$L timeout -k 10 200 python tools/timeline.py --config C2 --steps 5 > gpurun_out/r3tl/c2.txt 2>&1
