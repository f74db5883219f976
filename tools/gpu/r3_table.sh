#!/bin/bash
# BASELINE.md §4 table at the round-3 HEAD (GPU rates + CPU oracle on the box's host cores)
set -o pipefail
mkdir -p gpurun_out/r3table
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/baseline_table.py > gpurun_out/r3table/table.json 2> gpurun_out/r3table/progress.txt || { tail -20 gpurun_out/r3table/progress.txt; exit 1; }
cat gpurun_out/r3table/table.json
