"""The step's fp64 MFMA GEMM kernels through the C ABI (gpk_dgemm) against NumPy fp64 products.

Every product of the log-joint step (code/model_GP_solver_2d.py:104-119 and
code/model_GP_solver_advection.py:104-119: the K^{-1}-applications, the D-products of the
residual and the gradient products of the reverse pass) is one of these GEMMs.  Checked here
for each kernel (16x16 latency tiles, 64x64 tiles, the pipelined 128x128 tile of
gemm_tile_dev.h), every transpose signature, edge tiles (M, N multiples of 32 but not of 128),
the dual product (two passes on the 128x128 tile, in mixed signatures, alpha = 0 included),
beta C0 and the in-place update C += op(A) op(B).

Bar: max |C - C_ref| <= 64 K eps max(|A|)max(|B|) -- fp64 summation of K products of bounded
operands in any order (the kernels sum in MFMA k-slot order).
"""
import numpy as np
import pytest

from gpk._lib import GEMM_BIG, GEMM_SMALL, GEMM_TILE128, dgemm

pytestmark = pytest.mark.gpu
EPS = np.finfo(np.float64).eps


def _op(X, t):
    return X.T if t else X


def _mat(rng, rows, cols):
    return rng.uniform(-1.0, 1.0, size=(rows, cols))


def _bar(K, *mats):
    m = 1.0
    for X in mats:
        m *= np.abs(X).max()
    return 64 * K * EPS * m


@pytest.mark.parametrize("variant", [GEMM_SMALL, GEMM_BIG, GEMM_TILE128])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (288, 160, 96), (160, 416, 544)])
def test_single_product(variant, ta, tb, M, N, K):
    rng = np.random.default_rng(M * 7 + N * 3 + K + 11 * ta + 5 * tb)
    A = _mat(rng, *((K, M) if ta else (M, K)))
    B = _mat(rng, *((N, K) if tb else (K, N)))
    C, _ = dgemm(A, B, ta=ta, tb=tb, alpha=0.75, variant=variant)
    ref = 0.75 * (_op(A, ta) @ _op(B, tb))
    assert np.abs(C - ref).max() <= _bar(K, A, B)


@pytest.mark.parametrize("sig", [(0, 0, 0, 1), (1, 0, 0, 0), (0, 1, 1, 1), (1, 1, 0, 0)])
@pytest.mark.parametrize("alpha", [1.5, 0.0])
def test_dual_product_tile128(sig, alpha):
    """C = alpha op(A) op(B) + alpha2 op(A2) op(B2) + beta C0 on the 128x128 tile (two passes)
    and on the 64x64 kernel (one pass), both against NumPy."""
    ta, tb, ta2, tb2 = sig
    M, N, K, K2 = 288, 416, 160, 224
    rng = np.random.default_rng(sum(sig) + int(alpha * 4))
    A = _mat(rng, *((K, M) if ta else (M, K)))
    B = _mat(rng, *((N, K) if tb else (K, N)))
    A2 = _mat(rng, *((K2, M) if ta2 else (M, K2)))
    B2 = _mat(rng, *((N, K2) if tb2 else (K2, N)))
    C0 = _mat(rng, M, N)
    ref = alpha * (_op(A, ta) @ _op(B, tb)) - 0.5 * (_op(A2, ta2) @ _op(B2, tb2)) + 0.25 * C0
    for variant in (GEMM_TILE128, GEMM_BIG):
        C, _ = dgemm(A, B, ta=ta, tb=tb, alpha=alpha, A2=A2, B2=B2, ta2=ta2, tb2=tb2, alpha2=-0.5,
                     beta=0.25, C0=C0, variant=variant)
        assert np.abs(C - ref).max() <= _bar(K + K2, A, B) + _bar(K2, A2, B2)


@pytest.mark.parametrize("variant", [GEMM_BIG, GEMM_TILE128])
def test_in_place_update(variant):
    """C += -op(A) op(B) with C0 = C (the refinement fix-ups x += K^{-1} r)."""
    rng = np.random.default_rng(3)
    M, N, K = 256, 384, 320
    A, B, C0 = _mat(rng, M, K), _mat(rng, K, N), _mat(rng, M, N)
    C, _ = dgemm(A, B, alpha=-1.0, beta=1.0, C0=C0, variant=variant)
    assert np.abs(C - (C0 - A @ B)).max() <= _bar(K, A, B) + 4 * EPS


def test_tile128_rate_at_c5_size():
    """The 128x128 tile at the C5 stage shape (4096^3, each signature): correct against a
    column sample of the NumPy product, and its average device time reported (the bench's
    large_factors line carries the rate; no speed assertion here)."""
    n = 4096
    rng = np.random.default_rng(5)
    A, B = _mat(rng, n, n), _mat(rng, n, n)
    cols = rng.choice(n, size=16, replace=False)
    for ta, tb in ((0, 0), (0, 1), (1, 0), (1, 1)):
        C, us = dgemm(A, B, ta=ta, tb=tb, variant=GEMM_TILE128, iters=3)
        ref = _op(A, ta) @ _op(B, tb)[:, cols]
        assert np.abs(C[:, cols] - ref).max() <= _bar(n, A, B)
        assert us > 0.0
        print(f"tile128 ta={ta} tb={tb}: {us:.0f} us = {2 * n ** 3 / us / 1e6:.1f} TF/s")
