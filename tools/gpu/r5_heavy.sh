# round 5: C2 chain_multi, the heaviest tile workgroups (macro rows 1-2) swapped onto CUs that
# hold one workgroup (libgpk.so) vs not (libgpk_old.so): C2 GPU tests, then interleaved A/B
set -o pipefail
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain_multi.py tests/test_gpu_accuracy.py tests/test_gpu_parity.py -k "C2 or multi" -x -q --timeout 200 --timeout-method thread || exit 1
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_old.so; do
    echo -n "$lib: "; GPK_LIB_PATH=$L/$lib timeout -k 10 120 python -u tools/ab_flags.py --config C2 --reps 1 | tail -1 || exit 1
  done
done
