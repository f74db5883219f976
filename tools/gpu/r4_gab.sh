#!/bin/bash
# round 4: the gather in its step contexts, libgpk.so vs libgpk_abgat.so, interleaved
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
L=gaussian-process-slover-for-high-freq-pde_amd/gpk/_lib
for rep in 1 2; do
  for lib in libgpk.so libgpk_abgat.so; do
    echo "== $lib"
    GPK_LIB_PATH=$PWD/$L/$lib timeout -k 10 200 python -u tools/gather_context.py 2>&1 | grep -v write_stream || exit 1
  done
done
