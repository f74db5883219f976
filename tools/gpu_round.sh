#!/bin/bash
# One GPU session: parity tests, smoke, bench line, rocprof kernel stats + HBM PMC passes.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${1:-r1}
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
tail -3 $OUT/pytest_gpu.log
# rc 1 = ordinary test failures; anything else (abort, segfault, time limit) ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; tail -40 $OUT/pytest_gpu.log; exit 1; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$TAG -o bench -- python3 bench.py --no-cpu-baseline --no-large > $OUT/prof_$TAG.log 2>&1 || { echo rocprof failed; tail -20 $OUT/prof_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/pmc_fetch_$TAG -o pmc -- python3 bench.py --no-cpu-baseline --no-large --steps 50 --warmup 5 --kernel-iters 5 > $OUT/pmc_fetch_$TAG.log 2>&1 || { echo pmc fetch failed; tail -20 $OUT/pmc_fetch_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/pmc_write_$TAG -o pmc -- python3 bench.py --no-cpu-baseline --no-large --steps 50 --warmup 5 --kernel-iters 5 > $OUT/pmc_write_$TAG.log 2>&1 || { echo pmc write failed; tail -20 $OUT/pmc_write_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_c5_$TAG -o c5 -- python3 tools/run_steps.py --config C5 --steps 3 > $OUT/prof_c5_$TAG.log 2>&1 || { echo rocprof c5 failed; tail -20 $OUT/prof_c5_$TAG.log; exit 1; }
find $OUT/prof_$TAG $OUT/prof_c5_$TAG $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG -name "*.csv" | head -20
