# round 5: C5 inverse, pivot tile brought up to date one launch early (libgpk.so) vs the
# committed schedule (libgpk_old.so), interleaved; then the update-launch timeline (probe build)
set -o pipefail
mkdir -p gpurun_out/r5
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for rep in 1 2; do
  for lib in libgpk.so libgpk_old.so; do
    GPK_LIB_PATH=$L/$lib timeout -k 10 200 python -u tools/c5_inv_time.py || exit 1
  done
done
GPK_LIB_PATH=$L/libgpk_trace.so timeout -k 10 300 python -u tools/big_timeline.py --reps 3
