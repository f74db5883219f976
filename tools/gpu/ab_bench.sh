# A/B on one box: the bench with libgpk.so vs gpk/_lib/libgpk_ab.so, interleaved, at the shapes given
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_ab.so; do
    for a in "--steps 20 --warmup 5" "--steps 500 --warmup 20"; do
      GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-large --kernel-iters 5 > gpurun_out/ab.json 2>/dev/null || { echo bench failed; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$lib', '$a', round(d['value'],1), round(d['step1_per_call']['value'],1))"
    done
  done
done
