"""The register-resident d-space kernel at Dp = 256 (csrc/solve_rr.hip,
opt-in with FRECSYS_RR=1, read at every launch) against the CPU oracle.

Every entity goes through the d-space path (FRECSYS_DUAL=0), long histories
through the split kernel's slabs (FRECSYS_SPLIT_ROWS=64: the kernel reads
them transposed), for the three solve kinds it serves -- iALS, ProjectU,
ProjectV with and without the tail quirk -- at the north-star bar of 1e-4
per row, plus the NOT_SPD report.  The CVaR-MF gradient kinds keep the tiled
kernel.
"""
import numpy as np
import pytest

import oracle as O
from conftest import rel_rows

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")

TOL_ROW = 1e-4
DIM = 256


@pytest.fixture
def rr_env(monkeypatch):
    monkeypatch.setenv("FRECSYS_RR", "1")
    monkeypatch.setenv("FRECSYS_DUAL", "0")
    monkeypatch.setenv("FRECSYS_SPLIT_ROWS", "64")


def _ctx(nu, ni, up, uc, ip, ic, quirks=True):
    ctx = fh.Context(DIM, nu, ni, parity_quirks=quirks)
    ctx.load_csr(fh.SIDE_USER, up, uc)
    ctx.load_csr(fh.SIDE_ITEM, ip, ic)
    U, V = O.init_embeddings(1, 0.1, DIM, nu, ni)
    ctx.set_embeddings(fh.SIDE_USER, U)
    ctx.set_embeddings(fh.SIDE_ITEM, V)
    return ctx, U, V


def test_rr_ials(rr_env, quirk_data):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(nu, ni, up, uc, ip, ic)
    ctx.gramian(fh.SIDE_ITEM)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, 0.003, 0.1)
    Uo, rc = O.step(up, uc, V, O.gramian(V), 0, 0.003, 0.1, out=U.copy())
    assert rc == 0
    assert rel_rows(ctx.get_embeddings(fh.SIDE_USER), Uo).max() < TOL_ROW
    ctx.set_embeddings(fh.SIDE_USER, Uo)
    ctx.gramian(fh.SIDE_USER)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, 0.003, 0.1)
    Vo, rc = O.step(ip, ic, Uo, O.gramian(Uo), 0, 0.003, 0.1, out=V.copy())
    assert rc == 0
    Vg = ctx.get_embeddings(fh.SIDE_ITEM)
    assert rel_rows(Vg, Vo).max() < TOL_ROW
    np.testing.assert_array_equal(Vg[9], V[9])  # idle item untouched


def test_rr_weighted(rr_env, quirk_data):
    nu, ni, up, uc, ip, ic = quirk_data
    om = (0.05 + 0.95 * np.random.default_rng(5).random(nu)).astype(np.float32)
    ctx, U, V = _ctx(nu, ni, up, uc, ip, ic)
    ctx.gramian(fh.SIDE_ITEM)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_WEIGHTED_U, 0.004, 0.004, entity_weight=om)
    Uo, rc = O.step(up, uc, V, O.gramian(V), 1, 0.004, 0.004, entity_weight=om, out=U.copy())
    assert rc == 0
    assert rel_rows(ctx.get_embeddings(fh.SIDE_USER), Uo).max() < TOL_ROW
    h = np.diff(up).astype(np.float32)
    nu_w = np.where(h > 0, om / np.maximum(h, 1), 0).astype(np.float32)
    item_reg = (0.5 + np.random.default_rng(6).random(ni)).astype(np.float32)
    for quirk in (True, False):
        ctx, U, V = _ctx(nu, ni, up, uc, ip, ic, quirks=quirk)
        ctx.gramian(fh.SIDE_USER, weights=om)
        ctx.solve_side(fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, 0.004, 0.004, alpha=0.3,
                       entity_reg=item_reg, other_weight=nu_w)
        Vo, rc = O.step(ip, ic, U, O.gramian(U, om), 2, 0.004, 0.004, alpha=0.3,
                        quirk=int(quirk), entity_reg=item_reg, other_weight=nu_w, out=V.copy())
        assert rc == 0
        assert rel_rows(ctx.get_embeddings(fh.SIDE_ITEM), Vo).max() < TOL_ROW


def test_rr_not_spd(rr_env, quirk_data):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(nu, ni, up, uc, ip, ic)
    ctx.gramian(fh.SIDE_ITEM)
    with pytest.raises(fh.FrecsysError) as ei:
        ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, -50.0, 0.1)
    assert ei.value.code == fh.ERR_NOT_SPD
    assert 0 <= ei.value.entity < nu
