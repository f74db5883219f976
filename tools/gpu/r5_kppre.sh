# round 5: the pgrad tail's small-parameter loads prefetched before its last reduction and pg
# taken from LDS (libgpk.so) vs finalize_body's reload (libgpk_old.so): GPU tests, then C4 A/B
set -o pipefail
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_accuracy.py tests/test_gpu_fastgraph.py tests/test_gpu_golden.py tests/test_gpu_checkpoint.py -x -q --timeout 250 --timeout-method thread || exit 1
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_old.so; do
    echo -n "$lib: "; GPK_LIB_PATH=$L/$lib timeout -k 10 120 python -u tools/ab_flags.py --config C4 --reps 1 | tail -1 || exit 1
  done
done
