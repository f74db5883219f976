#!/bin/bash
# C2 class-sum row chunk size sweep (GPK_CSUM_RB), ms/step and the kernel stats of each
set -o pipefail
mkdir -p gpurun_out/csumrb
export TMPDIR=/tmp
for rb in ${RBS:-32 64 128 256 32}; do
  GPK_CSUM_RB=$rb timeout -k 10 200 python tools/run_steps.py --config C2 --steps 100 > gpurun_out/csumrb/steps_$rb.txt 2>&1 || { cat gpurun_out/csumrb/steps_$rb.txt; exit 1; }
  echo "rb=$rb $(head -1 gpurun_out/csumrb/steps_$rb.txt)"
done
for rb in 32 128; do
  GPK_CSUM_RB=$rb timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/csumrb/prof_$rb -o run -- python3 tools/run_steps.py --config C2 --steps 30 > gpurun_out/csumrb/prof_$rb.log 2>&1 || { tail gpurun_out/csumrb/prof_$rb.log; exit 1; }
  f=$(find gpurun_out/csumrb/prof_$rb -name "*kernel_stats.csv" | head -1)
  echo "== rb=$rb"; python3 -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])): print(f\"{r['Name'][:64]:64s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.2f} us\")
" "$f"
done
