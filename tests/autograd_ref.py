"""Independent torch-autograd transcription of the reference's loss (test infrastructure).

This mirrors the reference's own computation path rather than the closed forms:
kappa as written in code/kernel_matrix.py:114-193, derivative covariances by nested autograd
(as jax.grad(grad(kappa)) at code/kernel_matrix.py:49-57), jnp.abs with JAX's JVP convention
select(x >= 0, g, -g), LU solve + slogdet, and reverse-mode autodiff for the full gradient
(code/model_GP_solver_2d.py:87-179, code/model_GP_solver_1d.py:80-154).  It checks the
closed-form adjoints of oracle/gp_oracle.py independently.
"""
import math

import numpy as np
import torch

torch.set_default_dtype(torch.float64)


def _jax_abs(x):
    return torch.where(x >= 0, x, -x)  # autograd: select(x >= 0, g, -g), like jax's abs JVP


def kappa(kind, x1, y1, p):
    """Elementwise kappa over flattened pairs; p: dict of [Q] tensors."""
    d = _jax_abs(x1 - y1)[:, None]
    lw, ll, fr = p["log-w"][None, :], p["log-ls"][None, :], p["freq"][None, :]
    if kind == "SE_Cos_1d":       # kernel_matrix.py:114-128
        v = torch.exp(lw) * torch.exp(-d ** 2 * torch.exp(ll)) * torch.cos(2 * math.pi * d * fr)
    elif kind == "Matern52_Cos_1d":  # :138-155
        matern = (1 + math.sqrt(5) * d * torch.exp(ll) + 5 / 3 * d ** 2 * torch.exp(ll) ** 2) * \
            torch.exp(-math.sqrt(5) * d * torch.exp(ll))
        v = torch.exp(lw) * matern * torch.cos(2 * math.pi * d * fr)
    elif kind == "Matern52_1d":   # :163-176
        v = torch.exp(lw) * (1 + math.sqrt(5) * d * torch.exp(ll) + 5 / 3 * d ** 2 * torch.exp(ll) ** 2) * \
            torch.exp(-math.sqrt(5) * d * torch.exp(ll))
    else:                         # SE_1d :184-193
        v = torch.exp(lw) * torch.exp(-d ** 2 * torch.exp(ll))
    return v.sum(1)


def mats(kind, x, p, jitter, deriv):
    n = x.numel()
    X1 = x.reshape(-1, 1).expand(n, n).reshape(-1).clone().requires_grad_(True)
    X2 = x.reshape(1, -1).expand(n, n).reshape(-1)
    k = kappa(kind, X1, X2, p)
    K = k.reshape(n, n) + jitter * torch.eye(n)
    g1, = torch.autograd.grad(k.sum(), X1, create_graph=True)
    if deriv == 1:
        D = g1
    else:
        D, = torch.autograd.grad(g1.sum(), X1, create_graph=True)
    return K, D.reshape(n, n)


def _tp(params):
    out = {}
    for k, v in params.items():
        if isinstance(v, dict):
            out[k] = _tp(v)
        else:
            out[k] = torch.tensor(np.asarray(v, np.float64), requires_grad=True)
    return out


def _grads(tp):
    out = {}
    for k, v in tp.items():
        out[k] = _grads(v) if isinstance(v, dict) else (v.grad.numpy().copy() if v.grad is not None else np.zeros(v.shape))
    return out


def loss_grad_2d(prob, params):
    tp = _tp(params)
    kind, eq = prob["kind"], prob["eq"]
    x1 = torch.tensor(prob["x1"])
    x2 = torch.tensor(prob["x2"])
    U = tp["U"]
    deriv = 1 if eq == "advection" else 2
    K1, D1 = mats(kind, x1, tp["kernel_paras_1"], prob["jitter"], deriv)
    K2, D2 = mats(kind, x2, tp["kernel_paras_2"], prob["jitter"], deriv)
    A = torch.linalg.solve(K1, U)
    Bt_T = torch.linalg.solve(K2, U.T)
    Uxx = D1 @ A
    Uyy = (D2 @ Bt_T).T
    ub = torch.cat((U[0, :], U[-1, :], U[:, 0], U[:, -1]))
    bv = torch.tensor(prob["bvals"])
    bgap = ((ub - bv) ** 2).sum()
    F = torch.tensor(prob["src"])
    if eq == "advection":
        R = prob["beta"] * Uxx + Uyy - F
    elif eq == "allencahn":
        R = Uxx + Uyy + U * (U ** 2 - 1) - F
    else:
        R = Uxx + Uyy - F
    egap = (R ** 2).sum()
    N1, N2 = U.shape
    c = prob["logdet"]
    log_prior = -0.5 * N2 * torch.linalg.slogdet(K1)[1] * c - 0.5 * N1 * torch.linalg.slogdet(K2)[1] * c \
        - 0.5 * (A * Bt_T.T).sum()
    log_b = 0.5 * ub.numel() * tp["log_tau"] - 0.5 * torch.exp(tp["log_tau"]) * bgap
    eq_ll = 0.5 * N1 * N2 * tp["log_v"] - 0.5 * torch.exp(tp["log_v"]) * egap
    loss = -(log_prior + log_b * prob["llk_weight"] + eq_ll)
    loss.backward()
    return float(loss), _grads(tp)


def loss_grad_1d(prob, params):
    tp = _tp(params)
    kind = prob["kind"]
    x = torch.tensor(prob["x"])
    u = tp["u"]
    K, D = mats(kind, x, tp["kernel_paras"], prob["jitter"], 2)
    alpha = torch.linalg.solve(K, u)
    uxx = D @ alpha
    xind = torch.tensor(np.asarray(prob["xind"]))
    bgap = ((u[xind].reshape(-1) - torch.tensor(prob["y"])) ** 2).sum()
    f = torch.tensor(prob["src"])
    if prob["eq"] == "allencahn":
        R = uxx.reshape(-1) + (u * (u ** 2 - 1)).reshape(-1) - f
    else:
        R = uxx.reshape(-1) - f
    egap = (R ** 2).sum()
    log_prior = -0.5 * torch.linalg.slogdet(K)[1] * prob["logdet"] - 0.5 * (u * alpha).sum()
    log_b = 0.5 * xind.numel() * tp["log_tau"] - 0.5 * torch.exp(tp["log_tau"]) * bgap
    eq_ll = 0.5 * x.numel() * tp["log_v"] - 0.5 * torch.exp(tp["log_v"]) * egap
    loss = -(log_prior + log_b * prob["llk_weight"] + eq_ll)
    loss.backward()
    return float(loss), _grads(tp)


def loss_grad_1d_extra(prob, params, params_extra, kind_extra):
    """loss_extra (code/model_GP_solver_1d_extra.py:101-137) transcribed literally, reverse-mode
    gradient w.r.t. params_extra (the first GP is evaluated but not differentiated)."""
    x = torch.tensor(prob["x"])
    with torch.no_grad():
        kp0 = {k: torch.tensor(np.asarray(v, np.float64)) for k, v in params["kernel_paras"].items()}
    u0 = torch.tensor(np.asarray(params["u"], np.float64).reshape(-1, 1))
    K0, D0 = mats(prob["kind"], x, kp0, prob["jitter"], 2)
    u_xx = (D0 @ torch.linalg.solve(K0, u0)).detach()
    tp = _tp(params_extra)
    kpe = dict(tp["kernel_paras"])
    kpe["freq"] = torch.zeros_like(kpe["log-w"])
    u_extra = tp["u"].sum(axis=1).reshape(-1, 1)
    Ke, De = mats(kind_extra, x, kpe, prob["jitter"], 2)
    Kinv_u_extra = torch.linalg.solve(Ke, u_extra)
    u_xx_extra = De @ Kinv_u_extra
    xind = torch.tensor(np.asarray(prob["xind"]))
    y = torch.tensor(prob["y"])
    boundary_gap = ((u0[xind].reshape(-1) + u_extra[xind].reshape(-1) - y.reshape(-1)) ** 2).sum()
    f = torch.tensor(prob["src"]).reshape(-1)
    if prob["eq"] == "allencahn":
        u = u0 + u_extra
        eq_gap = ((u_xx.flatten() + u_xx_extra.flatten() + (u * (u ** 2 - 1)).flatten() - f) ** 2).sum()
    else:
        eq_gap = ((u_xx.flatten() + u_xx_extra.flatten() - f) ** 2).sum()
    log_prior = -0.5 * torch.linalg.slogdet(Ke)[1] * prob["logdet"] - 0.5 * (u_extra * Kinv_u_extra).sum()
    log_boundary_ll = 0.5 * xind.numel() * tp["log_tau"] - 0.5 * torch.exp(tp["log_tau"]) * boundary_gap
    eq_ll = 0.5 * x.numel() * tp["log_v"] - 0.5 * torch.exp(tp["log_v"]) * eq_gap
    loss = -(log_prior + log_boundary_ll * prob["llk_weight"] + eq_ll)
    loss.backward()
    return float(loss), _grads(tp)


def loss_grad_3d(prob, params):
    """The 3-axis Kronecker log joint (oracle/gp_oracle.py loss_grad_3d) written with DENSE
    Kronecker products -- K = K1 (x) K2 (x) K3, U_xx = (D1 (x) K2 (x) K3) K^{-1} vec U, the
    log-det of K itself -- so the oracle's mode products, unfoldings and log-det weights are
    checked against an independent formulation (small grids only)."""
    tp = _tp(params)
    kind, eq = prob["kind"], prob["eq"]
    xs = [torch.tensor(prob[f"x{a}"]) for a in (1, 2, 3)]
    KD = [mats(kind, xs[k], tp[f"kernel_paras_{k + 1}"], prob["jitter"], 2) for k in range(3)]
    (K1, D1), (K2, D2), (K3, D3) = KD
    U = tp["U"]
    u = U.reshape(-1)
    K = torch.kron(K1, torch.kron(K2, K3))
    Kinv_u = torch.linalg.solve(K, u)
    lap = (torch.kron(D1, torch.kron(K2, K3)) + torch.kron(K1, torch.kron(D2, K3))
           + torch.kron(K1, torch.kron(K2, D3))) @ Kinv_u
    F = torch.tensor(prob["src"]).reshape(-1)
    R = lap - F
    if eq == "allencahn":
        R = R + u * (u ** 2 - 1)
    egap = (R ** 2).sum()
    ub = torch.cat((U[0].reshape(-1), U[-1].reshape(-1), U[:, 0].reshape(-1), U[:, -1].reshape(-1),
                    U[:, :, 0].reshape(-1), U[:, :, -1].reshape(-1)))
    bgap = ((ub - torch.tensor(prob["bvals"])) ** 2).sum()
    log_prior = -0.5 * torch.linalg.slogdet(K)[1] * prob["logdet"] - 0.5 * (u * Kinv_u).sum()
    log_b = 0.5 * ub.numel() * tp["log_tau"] - 0.5 * torch.exp(tp["log_tau"]) * bgap
    eq_ll = 0.5 * u.numel() * tp["log_v"] - 0.5 * torch.exp(tp["log_v"]) * egap
    loss = -(log_prior + log_b * prob["llk_weight"] + eq_ll)
    loss.backward()
    return float(loss), _grads(tp)
