set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u tools/train_regime_parity.py --dump gpurun_out/r5/train_regime_fwd.npz
