# round 5: nontemporal stores in the C5 Adam U plane (libgpk.so) vs plain (libgpk_old.so),
# interleaved: C5 step time and the in-step K-assembly / tail stage times
set -o pipefail
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for rep in 1 2; do
  for lib in libgpk.so libgpk_old.so; do
    GPK_LIB_PATH=$L/$lib timeout -k 10 200 python -u tools/c5_stage_time.py || exit 1
  done
done
