#!/bin/bash
# round 4: C5 inverse pieces, A/B of libgpk.so vs $AB (default libgpk_abbig.so), interleaved
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
L=gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for rep in 1 2; do
  for lib in libgpk.so ${AB:-libgpk_abbig.so}; do
    echo "== $lib"
    GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python -u tools/c5_pieces.py || { echo pieces failed; exit 1; }
  done
done
