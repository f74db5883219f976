set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 tools/probes/bin/gemm_tile_probe 4096 > gpurun_out/r5/tile_probe1.txt 2>&1 || { cat gpurun_out/r5/tile_probe1.txt; exit 1; }
cat gpurun_out/r5/tile_probe1.txt
timeout -k 10 120 python tools/dgemm_library.py > gpurun_out/r5/dgemm_lib1.txt 2>&1; cat gpurun_out/r5/dgemm_lib1.txt
