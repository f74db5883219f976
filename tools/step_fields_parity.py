"""Device accuracy at a BASELINE config with the field-evaluation perturbation removed (test
infrastructure; GPU box -- the yardstick runs on the box's CPU).

tests/test_gpu_accuracy.py measures the device against the long-double yardstick built on the
ORACLE's K and D.  The step evaluates K and D itself (class values, gpk_forward_field Kc / D): the
two fp64 evaluations differ by ~1 ulp per element, and where the gradient is ill-conditioned in
K and D (C5's kernel parameters; C4 after training) that difference alone moves the answer by
more than the solves' rounding.  Here the yardstick and the fp64 LU oracle (the reference's
algorithm) are evaluated on the step's OWN K and D, so device and reference algorithm are
compared on identical inputs: per key, error / max(floor, MULT x LU distance) as in
test_gpu_accuracy.py, plus the LU oracle fed the step's K and D against the oracle-K/D fixture
(how far the field evaluations alone move the reference algorithm).

usage: python tools/step_fields_parity.py C1 C5 [--out gpurun_out/r5/step_fields.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np

from oracle import gp_oracle as O
from tests.helpers import config_problem
import tools.solve_accuracy as SA

from tests.test_gpu_accuracy import FLOOR, MULT  # noqa: E402  (the same bars)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--out")
    a = ap.parse_args()
    from gpk.problems import make_solver
    O.set_backend(True)
    report = {}
    for cid in a.configs:
        prob, params, _, cfg = config_problem(cid)
        s = make_solver(cid, seed=0)
        try:
            loss, g = s.loss_grad()
            names = ("Kc", "D") if cfg["dim"] == 1 else ("Kc1", "D1", "Kc2", "D2")
            fld = {n: s.forward_field(n) for n in names}
        finally:
            s.close()
        if cfg["dim"] == 1:
            kd = {id(params["kernel_paras"]): (fld["Kc"], fld["D"])}
        else:
            kd = {id(params["kernel_paras_1"]): (fld["Kc1"], fld["D1"]),
                  id(params["kernel_paras_2"]): (fld["Kc2"], fld["D2"])}
        saved = O.kernel_kd
        O.kernel_kd = lambda kind, x, kp, jitter, dv: kd[id(kp)]
        t = time.time()
        try:
            ext = SA.run_mode(prob, params, "ext")
            lu = SA.run_mode(prob, params, "lu")
        finally:
            O.kernel_kd = saved
        gd = O.unflatten_params(params, g)
        dev = SA.distances((loss, {k: O.flatten_params(gd[k]) for k in gd}), ext)
        ref = SA.distances(lu, ext)
        bar = {k: max(FLOOR[cid], MULT[cid] * v) for k, v in ref.items()}
        # the reference algorithm on the step's K and D, against the oracle-K/D fixture
        fx = np.load(os.path.join(ROOT, "tests", "golden", f"ext_{cid}.npz"))
        lu_fx = {"loss": abs(lu[0] - float(fx["loss_ext"])) / abs(float(fx["loss_ext"]))}
        for k, v in lu[1].items():
            if f"sample/{k}" in fx.files:
                v = v[fx[f"sample/{k}"]]
            lu_fx[k] = float(np.max(np.abs(v - fx[f"ext/{k}"])) / float(fx[f"maxabs/{k}"]))
        row = {"device": dev, "lu_oracle": ref, "bar": bar, "error_over_bar": {k: dev[k] / bar[k] for k in bar},
               "device_over_lu": {k: (dev[k] / ref[k] if ref[k] > 0 else None) for k in ref},
               "lu_on_step_KD_vs_oracle_KD_fixture": lu_fx, "seconds": time.time() - t}
        report[cid] = row
        print(cid, json.dumps({k: {kk: float("%.3g" % vv) if vv is not None else None for kk, vv in v.items()}
                               for k, v in row.items() if isinstance(v, dict)}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
