set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/spd_pieces.py 1024,2048,3072,4096 both > gpurun_out/pieces.txt 2>&1
rc=$?; cat gpurun_out/pieces.txt; exit $rc
