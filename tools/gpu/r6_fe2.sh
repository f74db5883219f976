# round 6: a candidate build (libgpk_new.so): the class-pipe tests and the speed A/B at C4 against
# libgpk.so, then the whole GPU suite on the candidate
set -o pipefail
OUT=${OUT:-gpurun_out/r6fe2}
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_libs.py --config C4 --libs $L/libgpk.so $L/libgpk_new.so --reps 3 > $OUT/ab_c4.txt 2>&1 || { tail $OUT/ab_c4.txt; exit 1; }
cat $OUT/ab_c4.txt
GPK_LIB_PATH=$L/libgpk_new.so timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/suite.log 2>&1; rc=$?
tail -2 $OUT/suite.log
[ $rc -eq 0 ] || { grep -E "FAILED|^E " $OUT/suite.log | head -20; exit 1; }
