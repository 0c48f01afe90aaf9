"""Basis versioning and early basis builds (capi.hip): a Gramian recomputed
from unchanged embeddings is reused, a basis / rotated copy is rebuilt only
when its inputs changed, and a Gramian whose consumer took the history-space
path last time gets its basis built on a side stream right away.  None of it
may change a result: every check is bitwise against the same calls with
FRECSYS_EAGER=0 (no early builds) or against a freshly formed Gramian.
"""
import numpy as np
import pytest

import oracle as O
from test_parity_gpu import _ctx

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")


def _epoch(ctx, reg=0.003, w=0.1):
    """The iALS Train() sequence (ials.h:187-206 / include/frecsys/ials.h)."""
    ctx.gramian(fh.SIDE_ITEM, fetch=False)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, reg, w)
    ctx.gramian(fh.SIDE_USER, fetch=False)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, reg, w)
    ctx.gramian(fh.SIDE_ITEM, fetch=False)
    return ctx.user_loss(fh.SIDE_USER, w, False)


@pytest.mark.parametrize("dim", [64, 128, 256, 512, 1000])
def test_eager_epochs_bitwise(quirk_data, monkeypatch, dim):
    nu, ni, up, uc, ip, ic = quirk_data
    out = []
    for eager in ("0", "1"):
        monkeypatch.setenv("FRECSYS_EAGER", eager)
        ctx, _, _ = _ctx(dim, nu, ni, up, uc, ip, ic)
        losses = [_epoch(ctx) for _ in range(3)]
        out.append((ctx.get_embeddings(fh.SIDE_USER), ctx.get_embeddings(fh.SIDE_ITEM), losses))
        ctx.close()
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    for a, b in zip(out[0][2], out[1][2]):
        np.testing.assert_array_equal(a, b)


def test_gramian_follows_embeddings(quirk_data):
    """Reuse only while the rows are unchanged: after set_embeddings and
    after a solve the Gramian is formed anew."""
    nu, ni, up, uc, ip, ic = quirk_data
    dim = 64
    ctx, _, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    G1 = ctx.gramian(fh.SIDE_ITEM)
    np.testing.assert_array_equal(G1, ctx.gramian(fh.SIDE_ITEM))  # reused
    V2 = (V * 1.5).astype(np.float32)
    ctx.set_embeddings(fh.SIDE_ITEM, V2)
    G2 = ctx.gramian(fh.SIDE_ITEM)
    ref = V2.astype(np.float64).T @ V2.astype(np.float64)
    assert np.abs(G2 - ref).max() / np.abs(ref).max() < 1e-5
    _epoch(ctx)
    V3 = ctx.get_embeddings(fh.SIDE_ITEM).astype(np.float64)
    G3 = ctx.gramian(fh.SIDE_ITEM)
    ref3 = V3.T @ V3
    assert np.abs(G3 - ref3).max() / np.abs(ref3).max() < 1e-5
    # a weighted Gramian of the same side is never served from the plain one
    wts = np.linspace(0.5, 1.5, ni).astype(np.float32)
    Gw = ctx.gramian(fh.SIDE_ITEM, weights=wts)
    refw = (V3 * wts[:, None]).T @ V3
    assert np.abs(Gw - refw).max() / np.abs(refw).max() < 1e-5
    np.testing.assert_array_equal(ctx.gramian(fh.SIDE_ITEM), G3)
    ctx.close()


def test_basis_rebuilt_after_set_gramian(quirk_data, monkeypatch):
    """set_gramian invalidates the basis built from the previous Gramian:
    the solve with the new G equals a fresh context's."""
    nu, ni, up, uc, ip, ic = quirk_data
    dim = 64
    rng = np.random.default_rng(3)
    B = rng.standard_normal((dim, dim)).astype(np.float64)
    Gx = (B @ B.T / dim).astype(np.float32)
    res = []
    for warm in (True, False):
        ctx, _, _ = _ctx(dim, nu, ni, up, uc, ip, ic)
        if warm:  # a basis of the item Gramian exists (and an early build ran)
            _epoch(ctx)
            _epoch(ctx)
            U0, V0 = O.init_embeddings(1, 0.1, dim, nu, ni)  # back to _ctx's start
            ctx.set_embeddings(fh.SIDE_USER, U0)
            ctx.set_embeddings(fh.SIDE_ITEM, V0)
        ctx.set_gramian(fh.SIDE_ITEM, Gx)
        ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, 0.003, 0.1)
        res.append(ctx.get_embeddings(fh.SIDE_USER))
        ctx.close()
    np.testing.assert_array_equal(res[0], res[1])
