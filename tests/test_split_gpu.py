"""Long-history split of the d-space solve: the SYRK of an entity with more
than 2*FRECSYS_SPLIT_ROWS assembly rows is cut into slabs computed by
separate workgroups and summed by the entity's own workgroup.  Forced here
with tiny slabs (32 / 64 rows) so the small fixture exercises it, for every
kind, with and without the ProjectV tail quirk (whose extra rows straddle
slab boundaries).  FRECSYS_DUAL=0 keeps every entity on the d-space path.
"""
import numpy as np
import pytest

import oracle as O
from conftest import rel_rows
from test_parity_gpu import _ctx, _v_inputs, _weights

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")

TOL_ROW = 1e-4


@pytest.fixture(autouse=True)
def _dspace_only(monkeypatch):
    monkeypatch.setenv("FRECSYS_DUAL", "0")


@pytest.mark.parametrize("dim", [32, 64, 256])
@pytest.mark.parametrize("rows", ["32", "64", "0"])
def test_ials_split(monkeypatch, quirk_data, dim, rows):
    monkeypatch.setenv("FRECSYS_SPLIT_ROWS", rows)
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    ctx.gramian(fh.SIDE_USER)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, 0.003, 0.1)
    Vo, rc = O.step(ip, ic, U, O.gramian(U), 0, 0.003, 0.1, out=V.copy())
    assert rc == 0
    assert rel_rows(ctx.get_embeddings(fh.SIDE_ITEM), Vo).max() < TOL_ROW


@pytest.mark.parametrize("dim", [32, 128])
@pytest.mark.parametrize("quirk", [True, False])
def test_weighted_v_split(monkeypatch, quirk_data, dim, quirk):
    monkeypatch.setenv("FRECSYS_SPLIT_ROWS", "48")
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic, quirks=quirk)
    om = _weights(nu)
    nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
    ctx.gramian(fh.SIDE_USER, weights=om)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, 0.004, 0.004, alpha=0.3,
                   entity_reg=item_reg, other_weight=nu_w)
    Vo, rc = O.step(ip, ic, U, O.gramian(U, om), 2, 0.004, 0.004, alpha=0.3, quirk=int(quirk),
                    entity_reg=item_reg, other_weight=nu_w, out=V.copy())
    assert rc == 0
    assert rel_rows(ctx.get_embeddings(fh.SIDE_ITEM), Vo).max() < TOL_ROW


@pytest.mark.parametrize("dim", [64])
def test_weighted_u_and_cvar_split(monkeypatch, quirk_data, dim):
    monkeypatch.setenv("FRECSYS_SPLIT_ROWS", "32")
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    om = _weights(nu)
    ctx.gramian(fh.SIDE_ITEM)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_WEIGHTED_U, 0.004, 0.004, entity_weight=om)
    Uo, rc = O.step(up, uc, V, O.gramian(V), 1, 0.004, 0.004, entity_weight=om, out=U.copy())
    assert rel_rows(ctx.get_embeddings(fh.SIDE_USER), Uo).max() < TOL_ROW
    # CVaR gradient step on the split path (acc starts at 0, stale upper part)
    ctx.set_embeddings(fh.SIDE_USER, U)
    om2 = (np.random.default_rng(9).random(nu) < 0.4).astype(np.float32)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_CVAR_GRAD_U, 0.002, 0.008, stepsize=0.4,
                   entity_weight=om2)
    Ug, _ = O.step(up, uc, V, O.gramian(V), 3, 0.002, 0.008, stepsize=0.4, entity_weight=om2,
                   E=U)
    assert rel_rows(ctx.get_embeddings(fh.SIDE_USER), Ug).max() < TOL_ROW


def test_split_deterministic(monkeypatch, quirk_data):
    monkeypatch.setenv("FRECSYS_SPLIT_ROWS", "32")
    nu, ni, up, uc, ip, ic = quirk_data
    outs = []
    for _ in range(2):
        ctx, U, V = _ctx(128, nu, ni, up, uc, ip, ic)
        ctx.gramian(fh.SIDE_USER)
        ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, 0.003, 0.1)
        outs.append(ctx.get_embeddings(fh.SIDE_ITEM))
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("dim", [64, 256])
def test_split_side_stream_bitwise(monkeypatch, quirk_data, dim):
    """With every entity in d space, the slabs of the long histories and then
    their entities' solves run on a second stream beside the other entities'
    solve; the result is bitwise the single-stream one (FRECSYS_DUAL_SERIAL=1,
    read when the context is created)."""
    monkeypatch.setenv("FRECSYS_SPLIT_ROWS", "32")
    nu, ni, up, uc, ip, ic = quirk_data
    outs = []
    for serial in ("1", "0"):
        monkeypatch.setenv("FRECSYS_DUAL_SERIAL", serial)
        ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
        ctx.gramian(fh.SIDE_USER)
        ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, 0.003, 0.1)
        assert ctx.timing("solve_item.split")[1] == 1
        outs.append(ctx.get_embeddings(fh.SIDE_ITEM))
    np.testing.assert_array_equal(outs[0], outs[1])
