set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u tools/train_regime_parity.py --dump gpurun_out/r5/train_regime_fwd.npz
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-large --no-cpu-baseline > gpurun_out/r5/bench_fwd$i.json 2> gpurun_out/r5/bench_fwd$i.err || { tail -20 gpurun_out/r5/bench_fwd$i.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r5/bench_fwd$i.json').read().splitlines()[-1]);print({k:d[k] for k in ('value','ms_per_step','train_regime','step1_per_call')})"; done
