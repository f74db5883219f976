# round 5: dense GEMV rows in 1024-pair stretches (16 loads per lane in flight; libgpk.so) vs
# 256-pair steps (libgpk_old.so): 1D GPU tests, then C2 / C1 A/B, interleaved
set -o pipefail
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_accuracy.py tests/test_gpu_chain_multi.py tests/test_gpu_gemm.py -k "C1 or C2 or gemv or multi or 1d" -x -q --timeout 200 --timeout-method thread || exit 1
for rep in 1 2; do
  for lib in libgpk.so libgpk_old.so; do
    echo -n "$lib: "; GPK_LIB_PATH=$L/$lib timeout -k 10 120 python -u tools/ab_flags.py --config C2 --reps 1 | tail -1 || exit 1
    echo -n "$lib: "; GPK_LIB_PATH=$L/$lib timeout -k 10 120 python -u tools/ab_flags.py --config C1 --reps 1 | tail -1 || exit 1
  done
done
