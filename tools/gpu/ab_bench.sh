# A/B on one box: the bench with libgpk.so vs gpk/_lib/libgpk_ab.so (or the libraries in $LIBS), interleaved.
# C4 at the driver's 20-step shape and at 500 steps; C2 (ms/step) when AB_C2=1.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for rep in 1 2 3; do
  for lib in ${LIBS:-libgpk.so libgpk_ab.so}; do
    for a in "--steps 20 --warmup 5" "--steps 500 --warmup 20"; do
      GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-large --kernel-iters 5 > gpurun_out/ab.json 2>/dev/null || { echo bench failed; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('C4', '$lib', '$a', round(d['value'],1), round(d['step1_per_call']['value'],1))"
    done
    if [ "${AB_C2:-0}" = 1 ]; then
      GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python bench.py --config C2 --steps 100 --warmup 10 --no-cpu-baseline --no-large --kernel-iters 5 --step1-calls 5 > gpurun_out/ab.json 2>/dev/null || { echo C2 bench failed; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('C2', '$lib', round(d['ms_per_step'],4))"
    fi
  done
done
