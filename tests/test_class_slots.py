"""CPU: the class tile partials of the 2D class path (csrc/gpk_internal.h class_slots,
csrc/gemm.hip gemm_small_kernel's class epilogue, csrc/pgrad.hip's class staging).

A restatement of the device's index arithmetic in numpy: every 16x16 tile of a P x P matrix G
sums its elements per (signed diagonal offset, distance variant) and stores each sum into the
slot (class, sign, band group, tile row) -- the contraction then adds each class's row of slots.
Checked here: no slot is written twice, every in-range element lands in exactly one slot of its
own class, and the per-class row sums equal the direct class sums (what the class-sum launch
computes, csrc/pgrad.hip class_sum_kernel)."""
import numpy as np
import pytest


def classes(x):
    """cid [n, n], cbase [n + 1]: per diagonal k the distinct exact |x_{j+k} - x_j| in order of
    first appearance (gpk_api.cpp build_classes)."""
    n = len(x)
    cid = -np.ones((n, n), dtype=np.int64)
    cbase = np.zeros(n + 1, dtype=np.int64)
    u = 0
    for k in range(n):
        cbase[k] = u
        vals = []
        for j in range(n - k):
            d = abs(x[j + k] - x[j])
            if d not in vals:
                vals.append(d)
            c = u + vals.index(d)
            cid[j + k, j] = c
            cid[j, j + k] = c
        u += len(vals)
    cbase[n] = u
    return cid, cbase


def fdiv16(s):
    return s // 16  # floor, as the kernel's s >= 0 ? s / 16 : -((15 - s) / 16)


def epilogue_slots(G, cid, cbase, n, P):
    """The G_K / G_D epilogue of every 16x16 tile: returns the partials per (class, slot) [ncls, 4T] (the device stores them [4T][ncls])
    and the write count per slot."""
    T = P // 16
    ncls = int(cbase[n])
    cp = np.zeros((ncls, 4 * T))
    writes = np.zeros((ncls, 4 * T), dtype=np.int64)
    cidP = -np.ones((P, P), dtype=np.int64)
    cidP[:n, :n] = cid
    for I in range(T):
        for J in range(T):
            b = I - J
            tile = G[16 * I:16 * I + 16, 16 * J:16 * J + 16]
            tc = cidP[16 * I:16 * I + 16, 16 * J:16 * J + 16]
            for t, v2 in [(t, v2) for t in range(31 * 8) for v2 in (t & 7, (t & 7) + 8)]:
                dl, v = (t >> 3) - 15, v2
                s = 16 * b + dl
                k = abs(s)
                if k >= n or v >= cbase[k + 1] - cbase[k]:
                    continue
                e = ((2 if s < 0 else 0) + (0 if b == fdiv16(s) else 1)) * T + I - max(0, b)
                acc = 0.0
                for r in range(16):  # rows in order, as the kernel
                    c = r - dl
                    if 0 <= c < 16 and tc[r, c] >= 0 and tc[r, c] - cbase[abs(16 * I + r - 16 * J - c)] == v:
                        acc += tile[r, c]
                cp[cbase[k] + v, e] = acc
                writes[cbase[k] + v, e] += 1
    return cp, writes


@pytest.mark.parametrize("n,scale", [(40, 1.0), (64, 2 * np.pi), (72, 1.0), (96, 2 * np.pi), (130, 2 * np.pi)])
def test_class_slots_cover_every_pair_once(n, scale):
    x = np.linspace(0, scale, n)
    P = (n + 31) // 32 * 32
    cid, cbase = classes(x)
    vmax = int(np.max(np.diff(cbase)))
    assert vmax <= 16  # the epilogue's variant range (gpk_api.cpp enables it for vmax <= CB_VMAX)
    rng = np.random.default_rng(n)
    G = np.zeros((P, P))
    G[:n, :n] = rng.normal(size=(n, n))
    cp, writes = epilogue_slots(G, cid, cbase, n, P)
    assert writes.max() <= 1  # no slot written twice (the slot map is injective)
    direct = np.zeros(int(cbase[n]))
    np.add.at(direct, cid.ravel(), G[:n, :n].ravel())
    np.testing.assert_allclose(cp.sum(axis=1), direct, rtol=1e-12, atol=1e-12)
    # every pair counted exactly once: the same map on an all-ones G counts each class's pairs
    cnt, _ = epilogue_slots(np.pad(np.ones((n, n)), ((0, P - n), (0, P - n))), cid, cbase, n, P)
    np.testing.assert_array_equal(cnt.sum(axis=1), np.bincount(cid.ravel(), minlength=int(cbase[n])))


def test_class_slots_row_length_bounds_the_contributions():
    # a class on diagonal k: signs {+k, -k} x up to two bands x up to T tiles = 4T slots
    n, P = 64, 64
    T = P // 16
    x = np.linspace(0, 1, n)
    cid, cbase = classes(x)
    _, writes = epilogue_slots(np.zeros((P, P)), cid, cbase, n, P)
    assert writes.shape[1] == 4 * T
    # diagonal 0: one sign, one band -> T slots written; others at most 4T
    assert writes[cbase[0]:cbase[1]].sum(axis=1).max() == T
    assert writes.sum(axis=1).max() <= 4 * T
