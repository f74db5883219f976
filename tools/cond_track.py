"""Track cond(K1), cond(K2) and the refinement-gate lower bound along a BASELINE config's training."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-process-slover-for-high-freq-pde_amd")]
from gpk import problems

cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
s = problems.make_solver(cfg, seed=0)
done = 0
for target in [0, 20, 100, 300, 520, 1000, 2000]:
    if target > done:
        s.step(target - done)
        done = target
    K = s.forward_field("K1")
    c = np.linalg.cond(K)
    lb = K[0, 0] * np.max(np.diag(np.linalg.inv(K)))
    print(f"{cfg} step {done:5d}: cond(K1) {c:10.3e}  gate LB {lb:10.3e}  -> refine {lb > 8}", flush=True)
