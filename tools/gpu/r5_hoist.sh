# round 5: class distances loaded ahead of the barriers in class_eval / the pgrad class
# contraction (libgpk.so) vs after them (libgpk_old.so): GPU tests, then C4 and C2 A/B
set -o pipefail
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_accuracy.py tests/test_gpu_dclass.py tests/test_gpu_golden.py -x -q --timeout 250 --timeout-method thread || exit 1
for rep in 1 2 3; do
  for lib in libgpk.so libgpk_old.so; do
    echo -n "$lib: "; GPK_LIB_PATH=$L/$lib timeout -k 10 120 python -u tools/ab_flags.py --config C4 --reps 1 | tail -1 || exit 1
  done
done
for lib in libgpk.so libgpk_old.so; do
  echo -n "$lib: "; GPK_LIB_PATH=$L/$lib timeout -k 10 120 python -u tools/ab_flags.py --config C2 --reps 1 | tail -1 || exit 1
done
