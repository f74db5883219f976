# round 6: the fresh-handle warm-up gap: wall per step(20) call and a kernel
# trace of the same run
set -o pipefail
OUT=${OUT:-gpurun_out/r6w}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/warmup_trace.py 16 > $OUT/wall_plain.txt 2>&1 || { tail $OUT/wall_plain.txt; exit 1; }
cat $OUT/wall_plain.txt
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/prof -o w -- python3 tools/warmup_trace.py 16 > $OUT/wall_traced.txt 2>&1 || { tail $OUT/wall_traced.txt; exit 1; }
python3 tools/warmup_analyze.py $OUT/prof > $OUT/analysis.txt && cat $OUT/analysis.txt
