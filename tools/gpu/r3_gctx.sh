#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/gctx
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/gctx/tr -o tr -- python3 tools/gather_context.py > gpurun_out/gctx/log.txt 2>&1 || { tail -20 gpurun_out/gctx/log.txt; exit 1; }
grep "bench gather" gpurun_out/gctx/log.txt
f=$(find gpurun_out/gctx/tr -name "*kernel_trace.csv" | head -1)
python3 -c "
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
prev = None
for r in rows:
    n = r['Kernel_Name']
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    if 'gather' in n or 'class_eval' in n:
        print(f'{n[:40]:40s} {d:9.1f} us   (previous kernel: {prev})')
    prev = n[:40]
" "$f"
rm -rf gpurun_out/gctx/tr
