#!/bin/bash
# 1D class sums over folded lower pairs + LDS-bin chunking: 1D GPU tests, C2 ms/step vs the
# previous build, kernel stats
set -o pipefail
mkdir -p gpurun_out/f1d
export TMPDIR=/tmp
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 700 python -u -m pytest tests/test_gpu_chain_multi.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_accuracy.py tests/test_gpu_fastgraph.py tests/test_gpu_dclass.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/f1d/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/f1d/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/f1d/pytest.log | head -30; exit 1; fi
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_ab.so; do
    GPK_LIB_PATH=$L/$lib timeout -k 10 200 python tools/run_steps.py --config C2 --steps 100 > gpurun_out/f1d/steps.txt 2>&1 || { cat gpurun_out/f1d/steps.txt; exit 1; }
    echo "$lib $(head -1 gpurun_out/f1d/steps.txt)"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/f1d/prof -o run -- python3 tools/run_steps.py --config C2 --steps 30 > gpurun_out/f1d/prof.log 2>&1 || { tail gpurun_out/f1d/prof.log; exit 1; }
f=$(find gpurun_out/f1d/prof -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])): print(f\"{r['Name'][:64]:64s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.2f} us\")
" "$f"
