# round 5 session 1: GEMM / timeout / checkpoint / shard tests, C4 training-regime dump, bench
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_timeout.py tests/test_gpu_checkpoint.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/s1_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r5/s1_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r5/s1_tests.log | head -30; exit 1; }
timeout -k 10 300 python -u tools/train_regime_parity.py --dump gpurun_out/r5/train_regime.npz > gpurun_out/r5/train_regime_dump.txt 2>&1 || { cat gpurun_out/r5/train_regime_dump.txt; exit 1; }
cat gpurun_out/r5/train_regime_dump.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r5/bench_s1.json 2> gpurun_out/r5/bench_s1.err || { tail -20 gpurun_out/r5/bench_s1.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r5/bench_s1.json').read().splitlines()[-1]);print({k:d[k] for k in ('value','ms_per_step','train_regime','step_graph')});print(d['large_factors'])"
