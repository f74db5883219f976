#!/bin/bash
# round-end rehearsal: the driver's three GPU steps (pytest -m gpu, smoke, bench)
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/final/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/final/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/final/pytest.log | head -30; exit 1; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { cat gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/final/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['step1_per_call']['value'], d['large_factors']['step_ms'], d['large_factors']['spd_inverse_ms'])"
