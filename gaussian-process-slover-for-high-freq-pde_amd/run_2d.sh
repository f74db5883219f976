#!/bin/bash
# 2D experiments on the MI355X path (same equations / kernels / epochs as the reference's
# code/run_2d.sh).  Kernels: Matern52_Cos_1d (GP-HM-StM), SE_Cos_1d (GP-HM-GM),
# Matern52_1d (GP-Matern), SE_1d (GP-SE).  Set GPUS=N to train num_fold folds on N GPUs.
set -e
cd "$(dirname "$0")"
make -C csrc -j16 >/dev/null
run() {
  if [ "${GPUS:-1}" -gt 1 ]; then
    python -m torch.distributed.run --nnodes=1 --nproc-per-node "$GPUS" --master-addr 127.0.0.1 -m "$@"
  else
    python -m "$@"
  fi
}
run gpk.model_GP_solver_2d -equation='poisson_2d-sin_sin' -kernel='Matern52_Cos_1d' -nepoch=1000000
run gpk.model_GP_solver_2d -equation='poisson_2d-sin_add_cos' -kernel='Matern52_Cos_1d' -nepoch=1000000
run gpk.model_GP_solver_2d -equation='allencahn_2d-mix-sincos' -kernel='Matern52_Cos_1d' -nepoch=3000000
run gpk.model_GP_solver_advection -equation='advection-sin' -kernel='Matern52_Cos_1d' -nepoch=1000000
