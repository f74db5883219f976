set -o pipefail
export OMP_NUM_THREADS=16
timeout -k 10 1000 python -u tools/c5_kp_split.py C5 --axis 2
