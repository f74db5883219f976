# round 5: one-level pgrad tail (32 classes per contraction block) -- dispatch probe, GPU suite,
# A/B against the previous tree's library (gpk/_lib/prev), C4 timeline
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 5 60 tools/probes/bin/dispatch_probe 579 50 60 > gpurun_out/r5/dispatch_50.txt 2>&1 && timeout -k 5 60 tools/probes/bin/dispatch_probe 579 8 60 > gpurun_out/r5/dispatch_8.txt 2>&1 && timeout -k 5 60 tools/probes/bin/dispatch_probe 193 50 60 > gpurun_out/r5/dispatch_193.txt 2>&1 || { echo probe failed; exit 1; }
head -3 gpurun_out/r5/dispatch_50.txt; grep "CUs with" gpurun_out/r5/dispatch_*.txt
export GPK_PARITY_LOG=$PWD/gpurun_out/r5/parity_tail.jsonl
rm -f $GPK_PARITY_LOG
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/tail_suite.log 2>&1; rc=$?
tail -3 gpurun_out/r5/tail_suite.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " gpurun_out/r5/tail_suite.log | head -30; exit 1; }
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for rep in 1 2; do
  for lib in $L/libgpk.so $L/prev/libgpk.so; do
    echo "lib $lib"; GPK_LIB_PATH=$lib timeout -k 10 200 python -u tools/ab_flags.py --config C4 --reps 2 | tail -1 || exit 1
  done
done
GPK_LIB_PATH=$L/libgpk_trace.so timeout -k 10 120 python -u tools/timeline.py --config C4 --steps 5 > gpurun_out/r5/timeline_C4_tail.txt 2>&1 || { cat gpurun_out/r5/timeline_C4_tail.txt; exit 1; }
grep -E "pg |fin|pgrad" gpurun_out/r5/timeline_C4_tail.txt
