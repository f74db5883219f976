# round 5: the C4 bench line's value vs warm-up length (driver shape 20/5, 20/200, 500/20)
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
for rep in 1 2; do
  for a in "--steps 20 --warmup 5" "--steps 20 --warmup 200" "--steps 500 --warmup 20" "--steps 20 --warmup 50"; do
    timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-large --kernel-iters 5 --step1-calls 10 > gpurun_out/r5/warm.json 2>/dev/null || { echo bench failed; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r5/warm.json').read().strip().splitlines()[-1]); print('$a', round(d['value'],1), 'train_regime', round(d['train_regime']['value'],1), d['step_graph'])"
  done
done
