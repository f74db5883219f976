#!/bin/bash
# round 4: the C5 FETCH / WRITE passes again (per-kernel HBM bytes, the large-factor inverse's
# kernels by name), summarised by tools/pmc_summary.py
set -o pipefail
OUT=gpurun_out/r4p
mkdir -p $OUT
export TMPDIR=/tmp
C5="tools/run_steps.py --config C5 --steps 3"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch_C5 -o fetch_C5 -- python3 $C5 > $OUT/fetch_C5.log 2>&1 || { tail -20 $OUT/fetch_C5.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write_C5 -o write_C5 -- python3 $C5 > $OUT/write_C5.log 2>&1 || { tail -20 $OUT/write_C5.log; exit 1; }
python3 tools/pmc_summary.py $OUT/fetch_C5 $OUT/write_C5 $OUT/pmc_c5.json
rm -rf $OUT/fetch_C5 $OUT/write_C5
