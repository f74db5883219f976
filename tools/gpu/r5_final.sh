# round 5, final tree: bench + kernel traces + PMC passes (r5_profile.sh, suite skipped: run
# separately), then the per-config table
set -o pipefail
OUT=${OUT:-gpurun_out/r5p2}
mkdir -p $OUT
SKIP_TESTS=1 OUT=$OUT bash tools/gpu/r5_profile.sh || exit 1
timeout -k 10 600 python -u tools/baseline_table.py --no-cpu > $OUT/baseline_table.json 2> $OUT/baseline_table.err || { tail -20 $OUT/baseline_table.err; exit 1; }
tail -c 2000 $OUT/baseline_table.json
