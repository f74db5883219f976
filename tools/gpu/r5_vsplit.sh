# round 5: C2 chain_multi, V stage in two phases (libgpk.so) vs one (libgpk_old.so): the C2
# GPU tests on the new library, then an interleaved A/B of the C2 step rate
set -o pipefail
mkdir -p gpurun_out/r5
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain_multi.py tests/test_gpu_accuracy.py -k "C2 or chain_multi or multi" -x -q --timeout 200 --timeout-method thread || exit 1
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_old.so; do
    echo -n "$lib: "; GPK_LIB_PATH=$L/$lib timeout -k 10 120 python -u tools/ab_flags.py --config C2 --reps 1 | tail -1 || exit 1
  done
done
