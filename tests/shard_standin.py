"""Host stand-in of the row-sharded 2D step (test infrastructure; never the product).

`HostShardedSolver` runs the step the way a sharded libgpk handle does -- the plan of
gpk/shard.py `shard_plan` (which rows of which product a rank computes, which outputs are
all-gathered after which stage, the one all-reduce, the U gather after Adam), with the row
partition of `shard_rows` -- in NumPy fp64 on this process's share, exchanging over the
torch.distributed (gloo) group of the caller.  Every output row a rank did not compute and did
not receive is NaN, so a plan that omits an all-gather a later product needs poisons the loss.
The stage formulas are those of csrc/gpk_api.cpp build_descs (the 2D step: forward solves,
residual, reverse pass, G_K / G_D); the kernel fields and the parameter
contraction are the oracle's (oracle/gp_oracle.py, itself pinned to the reference).
It has the solver interface bench.py's `sharded_section` drives (prepare / step / sync / close).
"""
import math

import numpy as np

from gpk import shard as SH
from oracle import gp_oracle as O


class GlooExchange:
    """All-gather of row blocks and a sum all-reduce over the default torch.distributed group."""

    def __init__(self, world, rank):
        self.world, self.rank = world, rank
        self.count = 0  # collectives issued (per step: SH.plan_collectives of the plan)

    def gather_rows(self, M, h):
        self.count += 1
        if self.world == 1:
            return M
        import torch
        import torch.distributed as dist
        n = M.shape[0]
        r0 = self.rank * h
        blk = np.zeros((h,) + M.shape[1:])
        m = max(0, min(n, r0 + h) - r0)
        if m:
            blk[:m] = M[r0:r0 + m]
        parts = [torch.zeros(blk.shape, dtype=torch.float64) for _ in range(self.world)]
        dist.all_gather(parts, torch.from_numpy(blk))
        out = np.concatenate([p.numpy() for p in parts], axis=0)[:n]
        return out.copy()

    def allreduce(self, v):
        self.count += 1
        if self.world == 1:
            return v
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64).copy())
        dist.all_reduce(t)
        return t.numpy().copy()


class HostShardedSolver:
    def __init__(self, prob, params, world, rank, aug=True, refine_fwd=True, refine_rev=True,
                 lr=0.01, exchange=None, refine_fwd2=True):
        self.prob = prob
        self.params = {k: (dict(v) if isinstance(v, dict) else np.array(v, dtype=np.float64))
                       for k, v in params.items()}
        self.opt = O.Adam(lr)
        self.state = self.opt.init(self.params)
        self.world, self.rank = world, rank
        self.x = exchange or GlooExchange(world, rank)
        self.plan = SH.shard_plan(aug, refine_fwd, refine_rev, refine_fwd2)
        self.fwd2 = refine_fwd2
        self.steps = SH.parse_plan(self.plan)
        self.aug = aug
        N1 = len(prob["x1"])
        self.r0, self.r1, self.h = SH.shard_rows(N1, world, rank)
        self.losses = []
        self.collectives_per_step = None

    # -- the sharded step ------------------------------------------------------------------
    def _rows(self, M, zero=False):
        """M with only this rank's rows kept (others NaN; zero for G_K1 / G_D1, which the
        library leaves at zero on the rank and contracts as they are)."""
        out = np.zeros_like(M) if zero else np.full_like(M, np.nan)
        out[self.r0:self.r1] = M[self.r0:self.r1]
        return out

    def _loss_grad(self):
        p, prob = self.params, self.prob
        kind, eq = prob["kind"], prob["eq"]
        x1 = np.asarray(prob["x1"], np.float64)
        x2 = np.asarray(prob["x2"], np.float64)
        N1, N2 = x1.size, x2.size
        deriv = 1 if eq == "advection" else 2
        beta = float(prob.get("beta", 1.0)) if eq == "advection" else 1.0
        ac = eq == "allencahn"
        tau, v = math.exp(float(p["log_tau"])), math.exp(float(p["log_v"]))
        wb, c = float(prob["llk_weight"]), float(prob["logdet"])
        F = np.asarray(prob["src"], np.float64).reshape(N1, N2)
        U = np.asarray(p["U"], np.float64).reshape(N1, N2)
        # replicated: fields, inverses, log-dets (every rank inverts both factors)
        K1, D1 = O.kernel_kd(kind, x1, p["kernel_paras_1"], prob["jitter"], deriv)
        K2, D2 = O.kernel_kd(kind, x2, p["kernel_paras_2"], prob["jitter"], deriv)
        K1i, K2i = np.linalg.inv(K1), np.linalg.inv(K2)
        B = {"U": U}
        nan = np.full((N1, N2), np.nan)
        for k in ("A", "Bt", "S", "R", "W1", "W2", "T1", "T2", "X1", "X2", "Y1", "Y2"):
            B[k] = nan.copy()
        if self.aug:  # the augmented inverse launch: A, Bt whole on every rank
            B["A"], B["Bt"] = K1i @ U, U @ K2i
        P1d, P2d = K1i @ D1.T, K2i @ D2.T
        G = {"GK1": np.zeros((N1, N1)), "GD1": np.zeros((N1, N1)),
             "GK2": np.zeros((N2, N2)), "GD2": np.zeros((N2, N2))}
        part = {}
        rs = slice(self.r0, self.r1)

        def y(X):  # the X producers' side output Y = S / 2 + v X
            return 0.5 * B["S"] + v * X

        # stage k: [(output, full formula, 'k'-mode partial formula or None)]
        def products(k):
            if k == 0:
                return [("A", lambda: K1i @ B["U"]), ("Bt", lambda: B["U"] @ K2i)]
            if k == 1:
                return [("W1", lambda: B["U"] - K1 @ B["A"])] + \
                    ([("W2", lambda: B["U"] - B["Bt"] @ K2)] if self.fwd2 else [])
            if k == 2:
                return [("A", lambda: B["A"] + K1i @ B["W1"])] + \
                    ([("Bt", lambda: B["Bt"] + B["W2"] @ K2i)] if self.fwd2 else [])
            if k == 3:
                def resid():
                    R = beta * (D1 @ B["A"]) + B["Bt"] @ D2.T - F
                    if ac:
                        R = R + B["U"] * (B["U"] * B["U"] - 1.0)
                    return R
                return [("S", lambda: B["A"] @ K2i), ("R", resid)]
            if k == 4:
                return [("W1", lambda: B["A"] - B["S"] @ K2)]
            if k == 5:
                return [("S", lambda: B["S"] + B["W1"] @ K2i)]
            if k == 6:
                gd = [("GD1", lambda: v * beta * (B["R"] @ B["A"].T)),
                      ("GD2", lambda: v * (B["R"][rs].T @ B["Bt"][rs]))]
                if self.aug:
                    return [("X1", lambda: beta * (P1d @ B["R"])), ("X2", lambda: B["R"] @ P2d.T)] + gd
                return [("T1", lambda: beta * (D1.T @ B["R"])), ("T2", lambda: B["R"] @ D2)] + gd
            if k == 7:
                return [("X1", lambda: K1i @ B["T1"]), ("X2", lambda: B["T2"] @ K2i)]
            if k == 8:
                if self.aug:
                    return [("W1", lambda: beta * (D1.T @ B["R"]) - K1 @ B["X1"]),
                            ("W2", lambda: B["R"] @ D2 - B["X2"] @ K2)]
                return [("W1", lambda: B["T1"] - K1 @ B["X1"]), ("W2", lambda: B["T2"] - B["X2"] @ K2)]
            if k == 9:
                return [("X1", lambda: B["X1"] + K1i @ B["W1"]), ("X2", lambda: B["X2"] + B["W2"] @ K2i)]
            if k == 10:
                k2 = 0.5 * c * N1 * K2i if self.rank == 0 else 0.0
                return [("GK1", lambda: 0.5 * c * N2 * K1i - B["Y1"] @ B["A"].T),
                        ("GK2", lambda: k2 - B["Y2"][rs].T @ B["Bt"][rs])]
            raise ValueError(k)

        for op in self.steps:
            if op[0] == "stage":
                _, k, modes = op
                prods = products(k)
                assert len(prods) == len(modes), (k, modes)
                new = {}
                for (name, fn), mode in zip(prods, modes):
                    val = fn()  # ('k' formulas already take this rank's contraction rows)
                    if mode == "r":
                        val = self._rows(val, zero=name in ("GK1", "GD1"))
                    new[name] = val
                for name, val in new.items():
                    if name in G:
                        G[name] = val
                    else:
                        B[name] = val
                    if name in ("X1", "X2"):  # (+ Y = S / 2 + v X, same rows)
                        B["Y" + name[1]] = y(val) if modes[[n for n, _ in prods].index(name)] == "f" \
                            else self._rows(y(val))
                if k == 3:  # the residual launch's per-tile partials of ||R||^2 and <A, Bt>
                    part["egap"] = float(np.sum(B["R"][rs] ** 2))
                    part["quad"] = float(np.sum(B["A"][rs] * B["Bt"][rs]))
            elif op[0] == "gather":
                if op[1] == "U":
                    continue  # after Adam (below)
                B[op[1]] = self.x.gather_rows(B[op[1]], self.h)
            else:  # the one all-reduce: contraction partials + loss partials
                g1 = O.param_grad_contract(kind, x1, p["kernel_paras_1"], G["GK1"], G["GD1"], deriv)
                g2 = O.param_grad_contract(kind, x2, p["kernel_paras_2"], G["GK2"], G["GD2"], deriv)
                keys = ("freq", "log-ls", "log-w")
                vec = np.concatenate([g1[q] for q in keys] + [g2[q] for q in keys] +
                                     [[part["egap"], part["quad"]]])
                vec = self.x.allreduce(vec)
                Q = len(g1["freq"])
                g1 = {q: vec[i * Q:(i + 1) * Q] for i, q in enumerate(keys)}
                g2 = {q: vec[(3 + i) * Q:(4 + i) * Q] for i, q in enumerate(keys)}
                egap, quad = float(vec[6 * Q]), float(vec[6 * Q + 1])
        # loss (identical on every rank) and this rank's rows of dL/dU
        bv = np.asarray(prob["bvals"], np.float64).reshape(-1)
        bres = O.boundary_2d(U) - bv
        bgap = float(bres @ bres)
        ld1, ld2 = np.linalg.slogdet(K1)[1], np.linalg.slogdet(K2)[1]
        Nb, Nc = bv.size, N1 * N2
        log_prior = -0.5 * N2 * ld1 * c - 0.5 * N1 * ld2 * c - 0.5 * quad
        loss = -(log_prior + (0.5 * Nb * math.log(tau) - 0.5 * tau * bgap) * wb + 0.5 * Nc * math.log(v) - 0.5 * v * egap)
        gU = B["S"] + v * (B["X1"] + B["X2"])
        if ac:
            gU = gU + v * (3.0 * U * U - 1.0) * B["R"]
        gU = gU + wb * tau * O._boundary_scatter(N1, N2, bres)
        gU = self._rows(gU, zero=True)  # (rows of other ranks: updated there, gathered below)
        grad = {"U": gU, "kernel_paras_1": g1, "kernel_paras_2": g2,
                "log_tau": wb * (-0.5 * Nb + 0.5 * tau * bgap), "log_v": -0.5 * Nc + 0.5 * v * egap}
        return loss, grad

    def _step(self):
        c0 = self.x.count
        loss, grad = self._loss_grad()
        self.params, self.state = self.opt.update(grad, self.state, self.params)
        # Adam updated this rank's rows of U; the other rows come from their owners
        self.params["U"] = self.x.gather_rows(self.params["U"], self.h)
        self.collectives_per_step = self.x.count - c0
        self.losses.append(loss)
        return loss

    # -- the solver interface bench.py's sharded_section drives ----------------------------
    def shard_plan(self):
        return self.plan

    def prepare(self, n):
        pass

    def step(self, n=1):
        return [self._step() for _ in range(n)]

    def sync(self):
        pass

    def graph_mode(self):
        return False, 0

    def inverse_path(self):
        return "host-stand-in"

    def close(self):
        pass


class HostSolver(HostShardedSolver):
    """The same step on one process (no exchange): the single-GPU reference stand-in."""

    def __init__(self, prob, params, **kw):
        super().__init__(prob, params, 1, 0, **kw)
