"""ctypes binding of libgpk.so (include/gpk.h).

The product path has exactly one compute backend: the gfx950 HIP library.  If it is not
built, or no gfx950 device is visible, every call raises — there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPK_LIB_PATH") or os.path.join(_HERE, "_lib", "libgpk.so")

GPK_OK, GPK_EINVAL, GPK_ENOTPD, GPK_EHIP, GPK_ERCCL, GPK_ENOMEM, GPK_ENODEV = range(7)
GPK_FLAG_FORCE_BIG_GEMM = 1  # include/gpk.h
GPK_FLAG_FORCE_BIG_SPD = 2
GPK_FLAG_FORCE_SMALL_SPD = 4
GPK_FLAG_FORCE_HUGE_GEMM = 8
GPK_FLAG_NO_FAST_GRAPH = 16
GPK_FLAG_FAST_FIRST = 32
GPK_FLAG_NO_DCLASS = 64
GPK_FLAG_NO_CHAIN = 128
GPK_FLAG_NO_CHAIN_AUG = 256
GPK_FLAG_FORCE_WIDE_SPD = 512
GPK_FLAG_FORCE_NARROW_SPD = 1024
GPK_FLAG_SPLIT_FACTORS = 2048
GPK_FLAG_FORCE_CHAIN_MULTI = 4096
GPK_FLAG_REFINE_ALL = 8192
GPK_FLAG_NO_REFINE = 16384
GPK_FLAG_MATRIX_GEMV = 32768
GPK_FLAG_NO_QUARTER_TILES = 65536
GPK_FLAG_DD_CONTRACTION = 131072
GPK_FLAG_NO_DD_CONTRACTION = 262144
GPK_FLAG_ONE_SWEEP_UPDATE = 524288
GPK_FLAG_NO_QUARTER_FIRST = 1048576
GPK_FLAG_REFINE_FWD1_ONLY = 2097152
GPK_FLAG_NO_CLASS_BINS = 4194304
GPK_FLAG_NO_CLASS_PIPE = 8388608
GPK_INV_SWEEP, GPK_INV_CHAIN, GPK_INV_CHAIN_AUG, GPK_INV_BIG, GPK_INV_BIG_WIDE, GPK_INV_CHAIN_MULTI = range(6)
INV_PATH_NAMES = {0: "sweep", 1: "chain", 2: "chain_aug", 3: "big", 4: "big_wide", 5: "chain_multi"}
KIND_IDS = {"SE_Cos_1d": 0, "Matern52_Cos_1d": 1, "SE_1d": 2, "Matern52_1d": 3}
EQ_IDS = {"poisson": 0, "allencahn": 1, "advection": 2}

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


class GPKError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libgpk error {code}: {msg}")
        self.code = code


class NotPositiveDefinite(GPKError):
    pass


class gpk_problem(ctypes.Structure):
    _fields_ = [
        ("dim", ctypes.c_int32), ("eq", ctypes.c_int32), ("kind", ctypes.c_int32),
        ("n1", ctypes.c_int32), ("n2", ctypes.c_int32), ("q", ctypes.c_int32),
        ("x1", _dp), ("x2", _dp), ("src", _dp), ("bvals", _dp), ("bidx", _ip),
        ("nb", ctypes.c_int32),
        ("jitter", ctypes.c_double), ("llk_weight", ctypes.c_double),
        ("logdet", ctypes.c_double), ("beta", ctypes.c_double),
        ("lr", ctypes.c_double), ("b1", ctypes.c_double), ("b2", ctypes.c_double),
        ("eps", ctypes.c_double),
        ("device", ctypes.c_int32), ("flags", ctypes.c_int32),
        ("uoff", _dp),
    ]


class gpk_problem3(ctypes.Structure):
    _fields_ = [
        ("eq", ctypes.c_int32), ("kind", ctypes.c_int32),
        ("n1", ctypes.c_int32), ("n2", ctypes.c_int32), ("n3", ctypes.c_int32), ("q", ctypes.c_int32),
        ("x1", _dp), ("x2", _dp), ("x3", _dp), ("src", _dp), ("bvals", _dp),
        ("jitter", ctypes.c_double), ("llk_weight", ctypes.c_double), ("logdet", ctypes.c_double),
        ("lr", ctypes.c_double), ("b1", ctypes.c_double), ("b2", ctypes.c_double),
        ("eps", ctypes.c_double),
        ("device", ctypes.c_int32), ("flags", ctypes.c_int32),
    ]


EXPORTS = {
    "gpk_abi_version": ([], ctypes.c_int),
    "gpk_last_error": ([], ctypes.c_char_p),
    "gpk_device_count": ([_ip], ctypes.c_int),
    "gpk_kernel_matrices": ([ctypes.c_int32, ctypes.c_int32, _dp, ctypes.c_int32, _dp,
                             ctypes.c_int32, _dp, _dp, _dp, ctypes.c_int32, ctypes.c_double,
                             _dp, _dp], ctypes.c_int),
    "gpk_create": ([ctypes.POINTER(gpk_problem), ctypes.c_double,
                    ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "gpk_destroy": ([ctypes.c_void_p], ctypes.c_int),
    "gpk_num_params": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)], ctypes.c_int),
    "gpk_set_params": ([ctypes.c_void_p, _dp, ctypes.c_int64], ctypes.c_int),
    "gpk_get_params": ([ctypes.c_void_p, _dp, ctypes.c_int64], ctypes.c_int),
    "gpk_set_opt_state": ([ctypes.c_void_p, ctypes.c_int64, _dp, _dp, ctypes.c_int64], ctypes.c_int),
    "gpk_get_opt_state": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), _dp, _dp,
                           ctypes.c_int64], ctypes.c_int),
    "gpk_loss_grad": ([ctypes.c_void_p, _dp, _dp], ctypes.c_int),
    "gpk_step": ([ctypes.c_void_p, ctypes.c_int32, _dp], ctypes.c_int),
    "gpk_prepare": ([ctypes.c_void_p, ctypes.c_int32], ctypes.c_int),
    "gpk_sync": ([ctypes.c_void_p], ctypes.c_int),
    "gpk_predict": ([ctypes.c_void_p, _dp, ctypes.c_int32, _dp, ctypes.c_int32, _dp], ctypes.c_int),
    "gpk_criterion": ([ctypes.c_void_p, _dp], ctypes.c_int),
    "gpk_profile_stages": ([ctypes.c_void_p, ctypes.c_int32, _dp, ctypes.c_int32, _ip], ctypes.c_int),
    "gpk_stage_name": ([ctypes.c_void_p, ctypes.c_int32], ctypes.c_char_p),
    "gpk_time_spd_inverse": ([ctypes.c_void_p, ctypes.c_int32, _dp], ctypes.c_int),
    "gpk_bench_kernel": ([ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32, _dp, _dp, _dp], ctypes.c_int),
    "gpk_kernel_pairs": ([ctypes.c_int32, ctypes.c_int32, _dp, _dp, ctypes.c_int64, _dp, _dp, _dp,
                          ctypes.c_int32, _dp], ctypes.c_int),
    "gpk_forward_field": ([ctypes.c_void_p, ctypes.c_int32, _dp, ctypes.c_int64], ctypes.c_int),
    "gpk_comm_unique_id": ([ctypes.POINTER(ctypes.c_uint8), ctypes.c_int32], ctypes.c_int),
    "gpk_create_sharded": ([ctypes.POINTER(gpk_problem), ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                            ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "gpk_group_create": ([ctypes.POINTER(gpk_problem), ctypes.c_double, ctypes.c_int32,
                          ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "gpk_group_step": ([ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32, ctypes.c_int32, _dp], ctypes.c_int),
    "gpk_group_loss_grad": ([ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32, _dp, _dp], ctypes.c_int),
    "gpk_shard_info": ([ctypes.c_void_p, _ip, _ip, _ip, _ip], ctypes.c_int),
    "gpk_shard_plan": ([ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64], ctypes.c_int),
    "gpk_inverse_path": ([ctypes.c_void_p, _ip], ctypes.c_int),
    "gpk_set_chain_capacity": ([ctypes.c_int32], ctypes.c_int),
    "gpk_set_spd_big_workgroups": ([ctypes.c_int32], ctypes.c_int),
    "gpk_set_wait_limit": ([ctypes.c_int32], ctypes.c_int),
    "gpk_set_wait_limit_chunk": ([ctypes.c_int32, ctypes.c_int32], ctypes.c_int),
    "gpk_graph_mode": ([ctypes.c_void_p, _ip, ctypes.POINTER(ctypes.c_int64)], ctypes.c_int),
    "gpk_distance_classes": ([_dp, ctypes.c_int32, _ip, _ip], ctypes.c_int),
    "gpk_class_count": ([ctypes.c_void_p, ctypes.c_int32, _ip], ctypes.c_int),
    "gpk_class_sum_path": ([ctypes.c_void_p, _ip], ctypes.c_int),
    "gpk_class_pipe": ([ctypes.c_void_p, _ip], ctypes.c_int),
    "gpk_create3": ([ctypes.POINTER(gpk_problem3), ctypes.c_double,
                     ctypes.POINTER(ctypes.c_void_p)], ctypes.c_int),
    "gpk_destroy3": ([ctypes.c_void_p], ctypes.c_int),
    "gpk_num_params3": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)], ctypes.c_int),
    "gpk_set_params3": ([ctypes.c_void_p, _dp, ctypes.c_int64], ctypes.c_int),
    "gpk_get_params3": ([ctypes.c_void_p, _dp, ctypes.c_int64], ctypes.c_int),
    "gpk_loss_grad3": ([ctypes.c_void_p, _dp, _dp], ctypes.c_int),
    "gpk_step3": ([ctypes.c_void_p, ctypes.c_int32, _dp], ctypes.c_int),
    "gpk_dgemm": ([ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_double, _dp,
                   ctypes.c_int32, ctypes.c_int32, _dp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                   ctypes.c_double, _dp, ctypes.c_int32, ctypes.c_int32, _dp, ctypes.c_int32, ctypes.c_int32,
                   ctypes.c_double, _dp, _dp, ctypes.c_int32, ctypes.c_int32, _dp], ctypes.c_int),
    "gpk_wide_schedule": ([ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int64],
                          ctypes.c_int),
    "gpk_trace_reset": ([], ctypes.c_int),
    "gpk_trace_read": ([ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                        ctypes.c_int32], ctypes.c_int),
}

_LIB = None


def load():
    """Load libgpk.so (raises if it has not been built — no fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise GPKError(GPK_ENODEV, f"{LIB_PATH} not built; run __graft_entry__.build() "
                                       "or `make -C gaussian-process-slover-for-high-freq-pde_amd/csrc`")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (argtypes, restype) in EXPORTS.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = restype
        _LIB = lib
    return _LIB


def check(rc):
    if rc != GPK_OK:
        msg = load().gpk_last_error().decode(errors="replace")
        if rc == GPK_ENOTPD:
            raise NotPositiveDefinite(rc, msg)
        raise GPKError(rc, msg)


def dptr(a):
    return a.ctypes.data_as(_dp)


def f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


GEMM_AUTO, GEMM_SMALL, GEMM_BIG, GEMM_TILE128 = 0, 1, 2, 3


def dgemm(A, B, ta=False, tb=False, alpha=1.0, A2=None, B2=None, ta2=False, tb2=False, alpha2=1.0,
          beta=0.0, C0=None, variant=GEMM_AUTO, iters=0):
    """The step's fp64 MFMA GEMM kernels (gpk_dgemm) on host arrays: returns (C, avg_us) with
    C = alpha op(A) op(B) [+ alpha2 op(A2) op(B2)] [+ beta C0]; avg_us is the average device time
    of `iters` back-to-back launches (None when iters = 0).  Dimensions must be multiples of 32."""
    A, B = f64(A), f64(B)
    M, K = (A.shape[1], A.shape[0]) if ta else A.shape
    N = B.shape[0] if tb else B.shape[1]
    C = np.zeros((M, N)) if C0 is None else f64(C0).copy()
    K2, pa2, pb2, lda2, ldb2 = 0, None, None, 1, 1
    if A2 is not None:
        A2, B2 = f64(A2), f64(B2)
        K2 = A2.shape[0] if ta2 else A2.shape[1]
        pa2, pb2, lda2, ldb2 = dptr(A2), dptr(B2), A2.shape[1], B2.shape[1]
    us = ctypes.c_double(0.0)
    check(load().gpk_dgemm(variant, M, N, K, alpha, dptr(A), A.shape[1], int(ta), dptr(B), B.shape[1],
                           int(tb), K2, alpha2, pa2, lda2, int(ta2), pb2, ldb2, int(tb2), beta,
                           dptr(C) if C0 is not None else None, dptr(C), N, iters,
                           ctypes.byref(us) if iters else None))
    return C, (us.value if iters else None)
