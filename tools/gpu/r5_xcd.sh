# round 5: small GEMM stages dealt XCD-major (libgpk.so) vs in tile order (libgpk_old.so): GPU
# tests, then C4 / C3 A/B, interleaved
set -o pipefail
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_accuracy.py tests/test_gpu_fastgraph.py tests/test_gpu_gemm.py -k "C3 or C4 or gemm or small or fast" -x -q --timeout 200 --timeout-method thread || exit 1
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_old.so; do
    echo -n "$lib: "; GPK_LIB_PATH=$L/$lib timeout -k 10 120 python -u tools/ab_flags.py --config C4 --reps 1 | tail -1 || exit 1
  done
done
for lib in libgpk.so libgpk_old.so; do
  echo -n "$lib: "; GPK_LIB_PATH=$L/$lib timeout -k 10 120 python -u tools/ab_flags.py --config C3 --reps 1 | tail -1 || exit 1
done
