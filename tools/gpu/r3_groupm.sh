#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
L=$PWD/gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for rep in 1 2; do
  for lib in libgpk.so libgpk_g2.so libgpk_g8.so; do
    GPK_LIB_PATH=$L/$lib timeout -k 10 200 python tools/c5_gemm_ab.py || exit 1
  done
done
