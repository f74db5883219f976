"""Bisect the device preds (gpk_predict) against the oracle over grid sizes and paths (GPU box).
usage: python tools/probe_predict.py [n ...]"""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
import numpy as np
from oracle import gp_oracle as O
from gpk.problems import CONFIGS, make_solver
O.set_backend(True)
ns = [int(v) for v in sys.argv[1:]] or [512, 1600, 2048, 3072, 4096]
for base in ("C5", "C4"):
    for n in ns:
        cfg = dict(CONFIGS[base], n=n)
        prob, (xt, yt), _ = O.setup_2d(cfg["equation"], n, cfg["scale"], cfg["kernel"], llk_weight=cfg["llk_weight"],
                                       beta=cfg.get("beta"), m_test=300)
        params = O.init_params_2d(n, n, 30, cfg["freq_scale"])
        params["U"] = 0.1 * np.random.default_rng(0).normal(size=n * n).reshape(n, n)
        s = make_solver(cfg, seed=0)
        try:
            path = s.inverse_path()
            pd = s.predict(xt, yt)
            A = s.forward_field("K1inv_U")
        finally:
            s.close()
        po = O.preds_2d(prob, params, xt, yt)
        K1 = O.kernel_matrix(prob["kind"], prob["x1"], params["kernel_paras_1"], prob["jitter"])
        Ao = np.linalg.solve(K1, params["U"])
        e = float(np.linalg.norm(pd - po) / np.linalg.norm(po))
        ea = float(np.linalg.norm(A - Ao) / np.linalg.norm(Ao))
        print(json.dumps({"base": base, "n": n, "path": path, "preds_rel_l2": e, "A_rel_l2": ea}), flush=True)
