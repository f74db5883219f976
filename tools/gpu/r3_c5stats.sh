#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/c5s
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c5s/tr -o tr -- python3 tools/run_steps.py --config C5 --steps 3 > gpurun_out/c5s/log.txt 2>&1 || { tail gpurun_out/c5s/log.txt; exit 1; }
head -1 gpurun_out/c5s/log.txt
f=$(find gpurun_out/c5s/tr -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/c5s/C5_kernel_stats.csv
python3 -c "
import csv, sys, json
fl = {k: v['mfma_flops_per_dispatch'] for k, v in json.load(open('profiles/r3_pmc_mfma_c5.json'))['kernels'].items()}
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '')
    us = float(r['AverageNs']) / 1e3
    f = fl.get(n)
    print(f\"{n[:50]:50s} {int(r['Calls']):5d} {us:9.1f} us\" + (f'  {f / us / 1e6:6.1f} TF/s  {f / us / 1e6 / 78.6 * 100:5.1f} %' if f else ''))
" gpurun_out/c5s/C5_kernel_stats.csv
rm -rf gpurun_out/c5s/tr
