# round 5: the whole GPU suite (parity log), smoke and the driver-shape bench line
set -o pipefail
OUT=${OUT:-gpurun_out/r5f}
mkdir -p $OUT
export TMPDIR=/tmp GPK_PARITY_LOG=$PWD/$OUT/parity.jsonl
rm -f $GPK_PARITY_LOG
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/pytest.log | head -30; exit 1; }
python3 tools/parity_summary.py $GPK_PARITY_LOG $OUT/parity.json "round 5 $(cat tools/gpu/TREE.txt)" | sort -k4 | tail -14
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['train_regime']['value'], d['large_factors']['step_ms'], d['large_factors']['spd_inverse_ms'], d['roofline']['frac'])"
