"""The wide d-space SYRK from the pre-split table (csrc/wide_syrk.hip) against
the register-staged kernel it replaces (wide.hip wide_syrk2_kernel,
FRECSYS_WIDE_PRESPLIT=0): the same products in the same order, so every
solved row must be BIT-identical -- per kind (iALS, ProjectU, ProjectV with
and without the tail quirk, CVaR-MF's gradient step), at Dp = 512 and 1024,
through every SYRK mode (short entities, 2048-row flushes of unsplit long
histories, long-history slabs folded by their entity).  The results are also
held to the oracle at the 1e-4 row bar (the same bar as test_wide_gpu.py).
"""
import numpy as np
import pytest

import oracle as O
from conftest import make_quirk_data, rel_rows
from test_parity_gpu import _ctx, _v_inputs, _weights
from test_wide_split_gpu import long_items  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")

TOL_ROW = 1e-4


@pytest.fixture(scope="module")
def wide_data():
    return make_quirk_data(n_users=400, n_items=300, hot_frac=(0.40, 0.19, 0.29, 0.186, 0.7))


def _solve(monkeypatch, data, dim, side, kind, presplit, quirk=True, split=True):
    monkeypatch.setenv("FRECSYS_WIDE_PRESPLIT", "1" if presplit else "0")
    monkeypatch.setenv("FRECSYS_DUAL", "0")  # every entity through the wide d-space
    monkeypatch.setenv("FRECSYS_SPLIT_ROWS", "4096" if split else "0")
    nu, ni, up, uc, ip, ic = data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic, quirks=quirk)
    om = _weights(nu)
    kw = {}
    if side == fh.SIDE_USER:
        if kind == fh.KIND_IALS:
            ctx.gramian(fh.SIDE_ITEM)
            args = (0.003, 0.1)
        else:
            ctx.gramian(fh.SIDE_ITEM)
            args = (0.004, 0.004)
            kw = dict(entity_weight=om)
    else:
        if kind == fh.KIND_IALS:
            ctx.gramian(fh.SIDE_USER)
            args = (0.003, 0.1)
        else:
            nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
            ctx.gramian(fh.SIDE_USER, weights=om)
            args = (0.004, 0.004)
            kw = dict(alpha=0.3, entity_reg=item_reg, other_weight=nu_w)
            if kind == fh.KIND_CVAR_GRAD_V:
                kw["stepsize"] = 0.4
    ctx.solve_side(side, kind, *args, **kw)
    out = ctx.get_embeddings(side)
    ctx.close()
    return out, (U, V, om, args, kw)


def _ab(monkeypatch, data, dim, side, kind, **kw):
    new, inp = _solve(monkeypatch, data, dim, side, kind, True, **kw)
    old, _ = _solve(monkeypatch, data, dim, side, kind, False, **kw)
    np.testing.assert_array_equal(new, old)
    return new, inp


@pytest.mark.parametrize("dim", [512, 1000])
def test_syrk3_ials_both_sides(monkeypatch, wide_data, dim):
    nu, ni, up, uc, ip, ic = wide_data
    Un, (U, V, _, args, _) = _ab(monkeypatch, wide_data, dim, fh.SIDE_USER, fh.KIND_IALS)
    Uo, rc = O.step(up, uc, V, O.gramian(V), 0, *args, out=U.copy())
    assert rc == 0 and rel_rows(Un, Uo).max() < TOL_ROW
    Vn, (U, V, _, args, _) = _ab(monkeypatch, wide_data, dim, fh.SIDE_ITEM, fh.KIND_IALS)
    Vo, rc = O.step(ip, ic, U, O.gramian(U), 0, *args, out=V.copy())
    assert rc == 0 and rel_rows(Vn, Vo).max() < TOL_ROW


def test_syrk3_weighted_u(monkeypatch, wide_data):
    nu, ni, up, uc, ip, ic = wide_data
    Un, (U, V, om, args, kw) = _ab(monkeypatch, wide_data, 512, fh.SIDE_USER, fh.KIND_WEIGHTED_U)
    Uo, rc = O.step(up, uc, V, O.gramian(V), 1, *args, out=U.copy(), **kw)
    assert rc == 0 and rel_rows(Un, Uo).max() < TOL_ROW


@pytest.mark.parametrize("quirk", [True, False])
def test_syrk3_weighted_v(monkeypatch, wide_data, quirk):
    nu, ni, up, uc, ip, ic = wide_data
    Vn, (U, V, om, args, kw) = _ab(monkeypatch, wide_data, 512, fh.SIDE_ITEM,
                                    fh.KIND_WEIGHTED_V, quirk=quirk)
    Vo, rc = O.step(ip, ic, U, O.gramian(U, om), 2, *args, quirk=int(quirk), out=V.copy(), **kw)
    assert rc == 0 and rel_rows(Vn, Vo).max() < TOL_ROW


def test_syrk3_cvar_grad_v(monkeypatch, wide_data):
    _ab(monkeypatch, wide_data, 512, fh.SIDE_ITEM, fh.KIND_CVAR_GRAD_V)


@pytest.mark.parametrize("split", [True, False], ids=["slabs", "flushes"])
@pytest.mark.parametrize("dim", [512, 1000])
def test_syrk3_long_histories(monkeypatch, long_items, dim, split):  # noqa: F811
    # slabs: items > 4096 rows as 2048-row slabs folded by their entity;
    # flushes: the same items unsplit, two-level sums every 2048 rows
    Vn, (U, V, _, args, _) = _ab(monkeypatch, long_items, dim, fh.SIDE_ITEM, fh.KIND_IALS,
                                  split=split)
    nu, ni, up, uc, ip, ic = long_items
    Vo, rc = O.step(ip, ic, U, O.gramian(U), 0, *args, out=V.copy())
    assert rc == 0 and rel_rows(Vn, Vo).max() < TOL_ROW


@pytest.mark.parametrize("quirk", [True, False])
def test_syrk3_long_weighted_v(monkeypatch, long_items, quirk):  # noqa: F811
    _ab(monkeypatch, long_items, 512, fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, quirk=quirk)
