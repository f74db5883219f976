#!/bin/bash
# 1D experiments on the MI355X path (equations of the reference's code/run_1d.sh):
# poisson_1d-{single_sin,x_time_sinx,sin_cos,mix_sin,x2_add_sinx}, allencahn_1d-{single_sin,sin_cos}.
set -e
cd "$(dirname "$0")"
make -C csrc -j16 >/dev/null
python -m gpk.model_GP_solver_1d -equation='poisson_1d-single_sin' -kernel='Matern52_Cos_1d' -nepoch=100000
python -m gpk.model_GP_solver_1d -equation='poisson_1d-x_time_sinx' -kernel='Matern52_Cos_1d' -nepoch=100000
python -m gpk.model_GP_solver_1d -equation='poisson_1d-sin_cos' -kernel='Matern52_Cos_1d' -nepoch=100000
python -m gpk.model_GP_solver_1d -equation='allencahn_1d-single_sin' -kernel='Matern52_Cos_1d' -nepoch=100000
python -m gpk.model_GP_solver_1d -equation='allencahn_1d-sin_cos' -kernel='Matern52_Cos_1d' -nepoch=100000
# the two hardest cases use the extra-GP trick (second Matern52 GP after change_point * nepoch)
python -m gpk.model_GP_solver_1d_extra -equation='poisson_1d-mix_sin' -kernel='Matern52_Cos_1d' -nepoch=1000000
python -m gpk.model_GP_solver_1d_extra -equation='poisson_1d-x2_add_sinx' -kernel='Matern52_Cos_1d' -nepoch=1000000
