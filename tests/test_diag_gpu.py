"""The 32x32 diagonal-block factorisations of the blocked Cholesky
(chol.h): the lane recurrence (diag_factor_inv_lds) and the MFMA-blocked
factor (diag_factor_inv_blk, used by the d-space and TH >= 6 history-space
kernels).  Every pivot block of every solve goes through one of them, so
they are checked directly on random SPD tiles, ill-conditioned ones
included: L^-1 A L^-T = I within a bound that grows with cond(A), the upper
triangle exactly zero, and both routines agreeing.  (Replaces the
non-failing scripts/micro/diag_check.hip.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")


def _tiles(n, cond, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        q, _ = np.linalg.qr(rng.standard_normal((32, 32)))
        ev = np.geomspace(1.0, 1.0 / cond, 32) * rng.uniform(0.5, 50.0)
        out.append((q * ev) @ q.T)
    a = np.array(out)
    return ((a + a.transpose(0, 2, 1)) / 2).astype(np.float32)


@pytest.mark.parametrize("cond", [1e1, 1e3, 1e5])
@pytest.mark.parametrize("blocked", [False, True])
def test_diag_factor_inverse(cond, blocked):
    ctx = fh.Context(64, 1, 1)
    A = _tiles(64, cond, int(cond) + blocked)
    L, ok = ctx.debug_diag_factor(A, blocked)
    assert ok.all()
    assert np.all(np.triu(L, 1) == 0.0)
    A64, L64 = A.astype(np.float64), L.astype(np.float64)
    I = np.eye(32)
    err = np.abs(L64 @ A64 @ L64.transpose(0, 2, 1) - I).max(axis=(1, 2))
    assert err.max() < 4e-6 * cond, (err.max(), cond)
    ctx.close()


def test_diag_factor_variants_agree():
    ctx = fh.Context(64, 1, 1)
    A = _tiles(128, 1e3, 9)
    L0, ok0 = ctx.debug_diag_factor(A, False)
    L1, ok1 = ctx.debug_diag_factor(A, True)
    assert ok0.all() and ok1.all()
    scale = np.abs(L0).max(axis=(1, 2), keepdims=True)
    assert (np.abs(L1 - L0) / scale).max() < 1e-4
    ctx.close()


@pytest.mark.parametrize("blocked", [False, True])
def test_diag_factor_reports_non_spd(blocked):
    ctx = fh.Context(64, 1, 1)
    A = _tiles(8, 1e2, 3)
    A[2, 17, 17] = -1.0  # indefinite
    A[5] = -A[5]
    _, ok = ctx.debug_diag_factor(A, blocked)
    assert ok[2] == 0 and ok[5] == 0
    assert ok[[0, 1, 3, 4, 6, 7]].all()
    ctx.close()
