"""Device-resident solver handle: the Python face of libgpk's C ABI.

One `DeviceSolver` = one reference solver object (GP_solver_1d_single /
GP_solver_2d_single / GP_solver_2d_single_advection) whose params and optax Adam state
live in HBM on one MI355X.  Methods map 1:1 onto include/gpk.h.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, dptr, f64


def tree_flatten(t):
    """jax pytree leaf order for nested dicts: keys sorted (code/model_GP_solver_2d.py:245-261)."""
    if isinstance(t, dict):
        parts = [tree_flatten(t[k]) for k in sorted(t)]
        return np.concatenate(parts) if parts else np.zeros(0)
    return np.asarray(t, dtype=np.float64).reshape(-1)


def tree_unflatten(template, flat):
    flat = np.asarray(flat, dtype=np.float64)
    pos = [0]

    def rec(t):
        if isinstance(t, dict):
            return {k: rec(t[k]) for k in sorted(t)}
        a = np.asarray(t)
        n = a.size
        out = flat[pos[0]:pos[0] + n].reshape(a.shape).copy()
        pos[0] += n
        return out if a.shape else float(out)

    out = rec(template)
    if pos[0] != flat.size:
        raise ValueError("flat vector does not match the params template")
    return out


def params_template(dim, n1, n2, Q):
    """Shapes of the reference's params pytree (train(), 1d.py:203-213 / 2d.py:245-261)."""
    kp = {"freq": np.zeros(Q), "log-ls": np.zeros(Q), "log-w": np.zeros(Q)}
    if dim == 1:
        return {"kernel_paras": kp, "log_tau": 0.0, "log_v": 0.0, "u": np.zeros((n1, 1))}
    return {"U": np.zeros((n1, n2)), "kernel_paras_1": dict(kp),
            "kernel_paras_2": {k: v.copy() for k, v in kp.items()}, "log_tau": 0.0, "log_v": 0.0}


def distance_classes(x):
    """(ncls, vmax) of one axis' distance classes (host only; include/gpk.h
    gpk_distance_classes).  ncls = 0: more than 32 distances on one diagonal."""
    x = _lib.f64(x)
    c, v = ctypes.c_int32(), ctypes.c_int32()
    check(_lib.load().gpk_distance_classes(_lib.dptr(x), len(x), ctypes.byref(c), ctypes.byref(v)))
    return int(c.value), int(v.value)


class DeviceSolver:
    def __init__(self, dim, eq, kind, x1, src, bvals, x2=None, bidx=None, Q=30, jitter=1e-6,
                 llk_weight=200.0, logdet=True, beta=1.0, lr=0.01, freq_scale=20.0, device=0,
                 b1=0.9, b2=0.999, eps=1e-8, flags=0, uoff=None, shard=None):
        lib = _lib.load()
        self.dim = int(dim)
        self.eq = eq
        self.kind = kind
        self.Q = int(Q)
        self._x1 = f64(x1).reshape(-1)
        self.n1 = self._x1.size
        self._x2 = f64(x2).reshape(-1) if x2 is not None else np.zeros(1)
        self.n2 = self._x2.size if dim == 2 else 1
        self._src = f64(src).reshape(-1)
        self._bvals = f64(bvals).reshape(-1)
        if self._src.size != self.n1 * self.n2:
            raise ValueError("src must have n1*n2 entries")
        if dim == 1:
            self._bidx = np.ascontiguousarray(np.asarray(bidx, dtype=np.int32).reshape(-1))
            if self._bidx.size != self._bvals.size:
                raise ValueError("Xind and y must have the same length")
        else:
            self._bidx = np.zeros(1, dtype=np.int32)
            if self._bvals.size != 2 * self.n1 + 2 * self.n2:
                raise ValueError("2D bvals must be hstack(U[0,:],U[-1,:],U[:,0],U[:,-1])")
        p = _lib.gpk_problem()
        p.dim = self.dim
        p.eq = _lib.EQ_IDS[eq]
        p.kind = _lib.KIND_IDS[kind] if isinstance(kind, str) else int(kind)
        p.n1, p.n2, p.q = self.n1, self.n2, self.Q
        p.x1, p.x2, p.src, p.bvals = dptr(self._x1), dptr(self._x2), dptr(self._src), dptr(self._bvals)
        p.bidx = self._bidx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        p.nb = self._bvals.size if dim == 1 else 0
        p.jitter, p.llk_weight, p.logdet, p.beta = jitter, llk_weight, float(logdet), beta
        p.lr, p.b1, p.b2, p.eps = lr, b1, b2, eps
        p.device = device
        p.flags = int(flags)
        if uoff is not None:  # 1D Allen-Cahn offset (extra-GP second phase)
            if dim != 1:
                raise ValueError("uoff is a 1D (extra-GP) option")
            self._uoff = f64(uoff).reshape(-1)
            if self._uoff.size != self.n1:
                raise ValueError("uoff must have n1 entries")
            p.uoff = dptr(self._uoff)
        self._prob = p
        self._h = self._create(lib, p, float(freq_scale), shard)
        h = self._h
        n = ctypes.c_int64()
        check(lib.gpk_num_params(h, ctypes.byref(n)))
        self.nparams = n.value
        self.template = params_template(self.dim, self.n1, self.n2, self.Q)

    def _create(self, lib, p, freq_scale, shard):
        h = ctypes.c_void_p()
        if shard is None:
            check(lib.gpk_create(ctypes.byref(p), freq_scale, ctypes.byref(h)))
        else:  # (rank, nranks, 128-byte RCCL id): one rank of a row-sharded group
            rank, nranks, cid = shard
            buf = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(cid))
            check(lib.gpk_create_sharded(ctypes.byref(p), freq_scale, int(rank), int(nranks), buf,
                                         ctypes.byref(h)))
        return h

    def shard_info(self):
        """(rank, nranks, row0, rows): the rows of U this handle owns (all rows unsharded)."""
        v = [ctypes.c_int32() for _ in range(4)]
        check(_lib.load().gpk_shard_info(self._h, *[ctypes.byref(x) for x in v]))
        return tuple(int(x.value) for x in v)

    def shard_plan(self):
        """The row-sharded step's plan (gpk_shard_plan; gpk/shard.py shard_plan restates it)."""
        buf = ctypes.create_string_buffer(4096)
        check(_lib.load().gpk_shard_plan(self._h, buf, len(buf)))
        return buf.value.decode()

    def graph_mode(self):
        """(fast, rollbacks): whether the next step runs the graph without the refinement
        stages, and how many batches were rolled back and rerun with the full graph."""
        f, r = ctypes.c_int32(), ctypes.c_int64()
        check(_lib.load().gpk_graph_mode(self._h, ctypes.byref(f), ctypes.byref(r)))
        return bool(f.value), int(r.value)

    def inverse_path(self):
        """The SPD inverse the step uses: 'sweep' | 'chain' | 'chain_aug' | 'big'."""
        v = ctypes.c_int32()
        check(_lib.load().gpk_inverse_path(self._h, ctypes.byref(v)))
        return _lib.INV_PATH_NAMES[int(v.value)]

    # -- lifecycle ---------------------------------------------------------------------
    def class_counts(self):
        """Distance classes the step evaluates per axis (0: per-pair kernels)."""
        out = []
        for a in range(1 if self.dim == 1 else 2):
            c = ctypes.c_int32()
            check(_lib.load().gpk_class_count(self._h, a, ctypes.byref(c)))
            out.append(int(c.value))
        return out

    def class_sums_in_epilogue(self):
        """True when the G_K / G_D GEMM epilogues write the class partials (gpk_class_sum_path)."""
        v = ctypes.c_int32()
        check(_lib.load().gpk_class_sum_path(self._h, ctypes.byref(v)))
        return bool(v.value)

    def class_pipe(self):
        """True when multi-step batches evaluate the next step's class values inside the
        parameter-gradient launch (gpk_class_pipe)."""
        v = ctypes.c_int32()
        check(_lib.load().gpk_class_pipe(self._h, ctypes.byref(v)))
        return bool(v.value)

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().gpk_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- params / optimizer state --------------------------------------------------------
    def get_flat(self):
        out = np.empty(self.nparams)
        check(_lib.load().gpk_get_params(self._h, dptr(out), self.nparams))
        return out

    def set_flat(self, flat):
        flat = f64(flat).reshape(-1)
        check(_lib.load().gpk_set_params(self._h, dptr(flat), flat.size))

    def get_params(self):
        return tree_unflatten(self.template, self.get_flat())

    def set_params(self, params):
        self.set_flat(tree_flatten(params))

    def get_opt_state(self):
        mu = np.empty(self.nparams)
        nu = np.empty(self.nparams)
        c = ctypes.c_int64()
        check(_lib.load().gpk_get_opt_state(self._h, ctypes.byref(c), dptr(mu), dptr(nu), self.nparams))
        return int(c.value), mu, nu

    def set_opt_state(self, count, mu, nu):
        mu, nu = f64(mu).reshape(-1), f64(nu).reshape(-1)
        check(_lib.load().gpk_set_opt_state(self._h, int(count), dptr(mu), dptr(nu), self.nparams))

    # -- hot path ---------------------------------------------------------------------------
    def loss_grad(self):
        loss = ctypes.c_double()
        g = np.empty(self.nparams)
        check(_lib.load().gpk_loss_grad(self._h, ctypes.byref(loss), dptr(g)))
        return loss.value, g

    def step(self, n=1, losses=True):
        out = np.empty(max(int(n), 1))
        check(_lib.load().gpk_step(self._h, int(n), dptr(out) if losses else None))
        return out[:n] if losses else None

    def prepare(self, n=1):
        """Build every step graph a step(n) call can launch, without stepping (gpk_prepare)."""
        check(_lib.load().gpk_prepare(self._h, int(n)))

    def sync(self):
        """Wait for the handle's device work (gpk_sync); step() returns once its losses are known."""
        check(_lib.load().gpk_sync(self._h))

    def predict(self, xte1, xte2=None):
        x1 = f64(xte1).reshape(-1)
        if self.dim == 1:
            out = np.empty(x1.size)
            check(_lib.load().gpk_predict(self._h, dptr(x1), x1.size, None, 0, dptr(out)))
            return out
        x2 = f64(xte2).reshape(-1)
        out = np.empty(x1.size * x2.size)
        check(_lib.load().gpk_predict(self._h, dptr(x1), x1.size, dptr(x2), x2.size, dptr(out)))
        return out.reshape(x1.size, x2.size)

    def criterion(self):
        c = ctypes.c_double()
        check(_lib.load().gpk_criterion(self._h, ctypes.byref(c)))
        return c.value

    FIELDS_2D = {"K1": 0, "K2": 1, "K1inv_U": 2, "K2inv_Ut": 3, "U_xx": 4, "U_yy": 5,
                 "G_K1": 6, "G_D1": 7, "G_K2": 8, "G_D2": 9, "K1inv": 10, "K2inv": 11,
                 "K1inv_D1t": 12, "K2inv_D2t": 13, "R": 14, "X1": 15, "X2": 16, "S": 17,
                 "Kc1": 18, "Kc2": 19, "D1": 20, "D2": 21,
                 "K1_classes": 22, "K2_classes": 23, "D1_classes": 24, "D2_classes": 25}
    FIELDS_1D = {"K": 0, "Kinv_u": 2, "u_xx": 4, "Kc": 6, "D": 7}

    def forward_field(self, name):
        """value_and_grad_kernel quantities at the current params, computed on the device."""
        if self.dim == 2:
            what = self.FIELDS_2D[name]
            shape = [(self.n1, self.n1), (self.n2, self.n2), (self.n1, self.n2),
                     (self.n2, self.n1), (self.n1, self.n2), (self.n1, self.n2),
                     (self.n1, self.n1), (self.n1, self.n1), (self.n2, self.n2), (self.n2, self.n2),
                     (self.n1, self.n1), (self.n2, self.n2), (self.n1, self.n1), (self.n2, self.n2),
                     (self.n1, self.n2), (self.n1, self.n2), (self.n1, self.n2), (self.n1, self.n2),
                     (self.n1, self.n1), (self.n2, self.n2), (self.n1, self.n1), (self.n2, self.n2),
                     (self.n1, self.n1), (self.n2, self.n2), (self.n1, self.n1), (self.n2, self.n2)][what]
        else:
            what = self.FIELDS_1D[name]
            shape = (self.n1, self.n1) if what in (0, 6, 7) else (self.n1, 1)
        out = np.empty(shape)
        check(_lib.load().gpk_forward_field(self._h, what, dptr(out), out.size))
        return out

    # -- measurement -----------------------------------------------------------------------
    def profile_stages(self, iters=10):
        lib = _lib.load()
        cap = 16
        out = np.zeros(cap)
        n = ctypes.c_int32()
        check(lib.gpk_profile_stages(self._h, int(iters), dptr(out), cap, ctypes.byref(n)))
        return {lib.gpk_stage_name(self._h, k).decode(): float(out[k]) for k in range(n.value)}

    def time_spd_inverse(self, iters=10):
        us = ctypes.c_double()
        check(_lib.load().gpk_time_spd_inverse(self._h, int(iters), ctypes.byref(us)))
        return us.value

    def bench_kernel(self, name, iters=50):
        """(avg_us, algorithmic_flops, algorithmic_bytes) of one kernel launch (HIP events)."""
        us, fl, by = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        check(_lib.load().gpk_bench_kernel(self._h, name.encode(), int(iters), ctypes.byref(us),
                                           ctypes.byref(fl), ctypes.byref(by)))
        return us.value, fl.value, by.value


def kernel_pairs(kind, x1, x2, paras, deriv=0):
    """gpk_kernel_pairs: elementwise kappa / D_x1_kappa / DD_x1_kappa over pairs (vmap)."""
    lib = _lib.load()
    a, b = f64(x1).reshape(-1), f64(x2).reshape(-1)
    if a.size != b.size:
        raise ValueError("x1 and x2 must have the same number of elements")
    lw, ll, fr = (f64(paras[k]).reshape(-1) for k in ("log-w", "log-ls", "freq"))
    out = np.empty(a.size)
    k = _lib.KIND_IDS[kind] if isinstance(kind, str) else int(kind)
    check(lib.gpk_kernel_pairs(k, int(deriv), dptr(a), dptr(b), a.size, dptr(lw), dptr(ll),
                               dptr(fr), lw.size, dptr(out)))
    return out


def kernel_matrices(kind, x1, x2, paras, jitter=0.0, deriv=0):
    """gpk_kernel_matrices: (K, D) with K = kappa(x1_i, x2_j) + jitter*[i==j]."""
    lib = _lib.load()
    x1, x2 = f64(x1).reshape(-1), f64(x2).reshape(-1)
    lw, ll, fr = (f64(paras[k]).reshape(-1) for k in ("log-w", "log-ls", "freq"))
    K = np.empty((x1.size, x2.size))
    D = np.empty_like(K) if deriv else None
    k = _lib.KIND_IDS[kind] if isinstance(kind, str) else int(kind)
    check(lib.gpk_kernel_matrices(k, int(deriv), dptr(x1), x1.size, dptr(x2), x2.size, dptr(lw),
                                  dptr(ll), dptr(fr), lw.size, float(jitter), dptr(K),
                                  dptr(D) if deriv else None))
    return K, D


def set_chain_capacity(workgroups):
    """Override the co-resident workgroup budget gpk_create checks the persistent chain inverse
    against (0: query the device).  Tests use it to force the per-sweep fallback."""
    check(_lib.load().gpk_set_chain_capacity(int(workgroups)))


def set_spd_big_workgroups(workgroups):
    """Tile workgroups per factor of the large-factor inverse's update launch (0: default, two
    per CU).  Tests use a few to give each workgroup long runs of tiles at small sizes."""
    check(_lib.load().gpk_set_spd_big_workgroups(int(workgroups)))


def set_wait_limit(polls):
    """Poll budget of every inter-workgroup wait of later launches (0: the default 2^22).  Tests
    use 1 to force the hand-off-timeout path (GPK_ENOTPD, the failed gpk_step batch undone)."""
    check(_lib.load().gpk_set_wait_limit(int(polls)))


def set_wait_limit_chunk(polls, chunk):
    """Tests: the poll budget of set_wait_limit, applied only while step() runs its 64-step
    chunk number `chunk` (0-based); polls = 0 clears it (include/gpk.h)."""
    check(_lib.load().gpk_set_wait_limit_chunk(int(polls), int(chunk)))


def comm_unique_id():
    """128-byte RCCL id for gpk_create_sharded (rank 0 makes it, every rank uses the same)."""
    buf = (ctypes.c_uint8 * 128)()
    check(_lib.load().gpk_comm_unique_id(buf, 128))
    return bytes(buf)


class DeviceGroup(DeviceSolver):
    """`nranks` row-sharded handles of one 2D problem on ONE GPU, exchanging through device copies
    (gpk_group_create): the multi-GPU sharded step with an in-process stand-in for RCCL, for
    parity tests on a single device.  Same interface as DeviceSolver; set_* go to every rank,
    loss_grad returns the full gradient (U rows collected from their owners)."""

    def __init__(self, nranks, *args, **kw):
        self.nranks = int(nranks)
        super().__init__(*args, **kw)

    def sync(self):
        lib = _lib.load()
        for k in range(self.nranks):
            check(lib.gpk_sync(ctypes.c_void_p(self._hs[k])))

    def _create(self, lib, p, freq_scale, shard):
        arr = (ctypes.c_void_p * self.nranks)()
        check(lib.gpk_group_create(ctypes.byref(p), freq_scale, self.nranks, arr))
        self._hs = arr
        return ctypes.c_void_p(arr[0])

    def close(self):
        if getattr(self, "_hs", None) is not None:
            lib = _lib.load()
            for k in range(self.nranks):
                if self._hs[k]:
                    lib.gpk_destroy(self._hs[k])
            self._hs = None
            self._h = None

    def set_flat(self, flat):
        flat = f64(flat).reshape(-1)
        for k in range(self.nranks):
            check(_lib.load().gpk_set_params(self._hs[k], dptr(flat), flat.size))

    def set_opt_state(self, count, mu, nu):
        mu, nu = f64(mu).reshape(-1), f64(nu).reshape(-1)
        for k in range(self.nranks):
            check(_lib.load().gpk_set_opt_state(self._hs[k], int(count), dptr(mu), dptr(nu), self.nparams))

    def shard_plan(self, k=0):
        """Rank k's sharded-step plan (gpk_shard_plan)."""
        buf = ctypes.create_string_buffer(4096)
        check(_lib.load().gpk_shard_plan(ctypes.c_void_p(self._hs[k]), buf, len(buf)))
        return buf.value.decode()

    def inverse_path(self, k=0):
        v = ctypes.c_int32()
        check(_lib.load().gpk_inverse_path(ctypes.c_void_p(self._hs[k]), ctypes.byref(v)))
        return _lib.INV_PATH_NAMES[int(v.value)]

    def rank_state(self, k):
        """(flat params, Adam count, mu, nu) held by rank k's handle."""
        lib = _lib.load()
        flat, mu, nu = np.empty(self.nparams), np.empty(self.nparams), np.empty(self.nparams)
        cnt = ctypes.c_int64()
        check(lib.gpk_get_params(self._hs[k], dptr(flat), self.nparams))
        check(lib.gpk_get_opt_state(self._hs[k], ctypes.byref(cnt), dptr(mu), dptr(nu), self.nparams))
        return flat, cnt.value, mu, nu

    def loss_grad(self):
        loss = ctypes.c_double()
        g = np.empty(self.nparams)
        check(_lib.load().gpk_group_loss_grad(self._hs, self.nranks, ctypes.byref(loss), dptr(g)))
        return loss.value, g

    def step(self, n=1, losses=True):
        out = np.empty(max(int(n), 1))
        done = 0
        while done < n:
            k = min(4096, n - done)
            check(_lib.load().gpk_group_step(self._hs, self.nranks, k, dptr(out[done:])))
            done += k
        return out[:n] if losses else None
