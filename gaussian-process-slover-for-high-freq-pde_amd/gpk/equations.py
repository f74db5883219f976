"""The reference's equation_dict entries with their PDE source terms.

The reference builds sources by differentiating the exact solution with jax.grad
(code/model_GP_solver_1d.py:299-307, code/model_GP_solver_2d.py:355-366,
code/model_GP_solver_advection.py:354-362).  Here each exact solution carries its analytic
derivatives (host-side setup, not the hot path); `autodiff_source_*` offers the same
autodiff construction for user-supplied torch-expressible solutions.
"""
import numpy as np

s_, c_ = np.sin, np.cos

# name -> (u, u_x, u_xx) for 1D solutions  (code/model_GP_solver_1d.py:313-332)
_U1D = {
    "mix_sin": (lambda x: s_(x) + 0.1 * s_(20 * x) + 0.05 * s_(100 * x),
                lambda x: c_(x) + 2.0 * c_(20 * x) + 5.0 * c_(100 * x),
                lambda x: -s_(x) - 40.0 * s_(20 * x) - 500.0 * s_(100 * x)),
    "single_sin": (lambda x: s_(100 * x), lambda x: 100.0 * c_(100 * x),
                   lambda x: -1e4 * s_(100 * x)),
    "sin_cos": (lambda x: s_(6 * x) * c_(100 * x),
                lambda x: 6.0 * c_(6 * x) * c_(100 * x) - 100.0 * s_(6 * x) * s_(100 * x),
                lambda x: -10036.0 * s_(6 * x) * c_(100 * x) - 1200.0 * c_(6 * x) * s_(100 * x)),
    "x_time_sinx": (lambda x: x * s_(200 * x), lambda x: s_(200 * x) + 200.0 * x * c_(200 * x),
                    lambda x: 400.0 * c_(200 * x) - 40000.0 * x * s_(200 * x)),
    "x2_add_sinx": (lambda x: s_(500 * x) - 2 * (x - 0.5) ** 2,
                    lambda x: 500.0 * c_(500 * x) - 4.0 * (x - 0.5),
                    lambda x: -250000.0 * s_(500 * x) - 4.0),
    "x_time_sinx_scale": (lambda x: x * s_(200 * x * np.pi),
                          lambda x: s_(200 * np.pi * x) + 200 * np.pi * x * c_(200 * np.pi * x),
                          lambda x: 400 * np.pi * c_(200 * np.pi * x)
                          - (200 * np.pi) ** 2 * x * s_(200 * np.pi * x)),
}

EQUATIONS_1D = [
    "poisson_1d-mix_sin", "poisson_1d-single_sin", "poisson_1d-sin_cos", "poisson_1d-x_time_sinx",
    "poisson_1d-x2_add_sinx", "allencahn_1d-sin_cos", "allencahn_1d-single_sin",
]
EQUATIONS_2D = ["poisson_2d-sin_cos", "poisson_2d-sin_sin", "poisson_2d-sin_add_cos",
                "allencahn_2d-mix-sincos"]
EQUATIONS_ADV = ["advection-sin"]


def solution_1d(equation):
    """(u, src) with src = u'' (Poisson) or u'' + u(u^2-1) (Allen-Cahn)."""
    kind, name = equation.split("-", 1)
    u, _, uxx = _U1D[name]
    if kind == "allencahn_1d":
        return u, (lambda x: uxx(x) + u(x) * (u(x) ** 2 - 1.0))
    if kind == "poisson_1d":
        return u, uxx
    raise KeyError(equation)


def solution_2d(equation, beta=None):
    """(u, src) for the 2D Poisson / Allen-Cahn / advection equations."""
    if equation == "poisson_2d-sin_sin":
        return (lambda x, y: s_(100 * x) * s_(100 * y)), (lambda x, y: -2e4 * s_(100 * x) * s_(100 * y))
    if equation == "poisson_2d-sin_cos":
        return (lambda x, y: s_(100 * x) * c_(100 * y)), (lambda x, y: -2e4 * s_(100 * x) * c_(100 * y))
    if equation == "poisson_2d-sin_add_cos":
        g = lambda t: s_(6 * t) * c_(20 * t)
        g2 = lambda t: -436.0 * s_(6 * t) * c_(20 * t) - 240.0 * c_(6 * t) * s_(20 * t)
        return (lambda x, y: g(x) + g(y)), (lambda x, y: g2(x) + g2(y))
    if equation == "allencahn_2d-mix-sincos":
        g = lambda t: s_(t) + 0.1 * s_(20 * t) + c_(100 * t)
        g2 = lambda t: -s_(t) - 40.0 * s_(20 * t) - 1e4 * c_(100 * t)
        u = lambda x, y: g(x) * g(y)
        return u, (lambda x, y: g2(x) * g(y) + g(x) * g2(y) + u(x, y) * (u(x, y) ** 2 - 1.0))
    if equation == "advection-sin":
        # beta*u_x + u_y of sin(x - beta*y) vanishes identically (advection.py:386-388)
        return (lambda x, y: s_(x - beta * y)), (lambda x, y: 0.0 * x * y)
    if equation == "advection-multiscale":
        # synthetic multi-scale source for config C5
        u = lambda x, y: s_(x - beta * y) + 0.1 * s_(20 * np.pi * x) * s_(2 * np.pi * y)
        f = lambda x, y: (beta * 0.1 * 20 * np.pi * c_(20 * np.pi * x) * s_(2 * np.pi * y)
                          + 0.1 * s_(20 * np.pi * x) * 2 * np.pi * c_(2 * np.pi * y))
        return u, f
    raise KeyError(equation)


def boundary_2d(u_mesh):
    """get_boundary_vals: hstack(U[0,:], U[-1,:], U[:,0], U[:,-1]) (model_GP_solver_2d.py:377-379)."""
    return np.hstack((u_mesh[0, :], u_mesh[-1, :], u_mesh[:, 0], u_mesh[:, -1]))


def autodiff_source_1d(u_torch, x, allen_cahn=False):
    """src = u'' (+u(u^2-1)) by torch autograd, for a torch-expressible u (the reference's
    vmap(grad(grad(u))) construction, model_GP_solver_1d.py:299-307)."""
    import torch
    xt = torch.tensor(np.asarray(x, np.float64).reshape(-1), requires_grad=True)
    u = u_torch(xt)
    g, = torch.autograd.grad(u.sum(), xt, create_graph=True)
    gg, = torch.autograd.grad(g.sum(), xt)
    out = gg.detach().numpy()
    if allen_cahn:
        uv = u.detach().numpy()
        out = out + uv * (uv ** 2 - 1.0)
    return out
