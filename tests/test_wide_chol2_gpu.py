"""Two-panel wide Cholesky (csrc/wide.hip wide_chol2_kernel, Dp = 512,
opt-in with FRECSYS_WIDE_CHOL2=1, read at every call) against the default
one-panel wide_chol_kernel<16>.  It runs every sum of the one-panel kernel in the same
order, only sharing each streamed L tile between two panels, so the
solutions must be bit-identical -- for iALS, ProjectU and ProjectV with and
without the tail quirk, every entity through the d-space path
(FRECSYS_DUAL=0), odd-width dims included -- and the NOT_SPD report the
same entity.
"""
import numpy as np
import pytest

from test_parity_gpu import _ctx, _v_inputs, _weights
from test_wide_split_gpu import long_items  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")


def _run(monkeypatch, data, dim, side, kind, two, quirk=True, reg=None):
    monkeypatch.setenv("FRECSYS_WIDE_CHOL2", "1" if two else "0")
    monkeypatch.setenv("FRECSYS_DUAL", "0")
    nu, ni, up, uc, ip, ic = data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic, quirks=quirk)
    om = _weights(nu)
    kw = {}
    if kind == fh.KIND_IALS:
        ctx.gramian(fh.SIDE_ITEM if side == fh.SIDE_USER else fh.SIDE_USER)
        args = (0.003 if reg is None else reg, 0.1)
    elif kind == fh.KIND_WEIGHTED_U:
        ctx.gramian(fh.SIDE_ITEM)
        args = (0.004, 0.004)
        kw = dict(entity_weight=om)
    else:
        nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
        ctx.gramian(fh.SIDE_USER, weights=om)
        args = (0.004, 0.004)
        kw = dict(alpha=0.3, entity_reg=item_reg, other_weight=nu_w)
    ctx.solve_side(side, kind, *args, **kw)
    return ctx.get_embeddings(side)


@pytest.mark.parametrize("dim", [512, 300])
def test_chol2_ials_items_bit_identical(monkeypatch, long_items, dim):
    a = _run(monkeypatch, long_items, dim, fh.SIDE_ITEM, fh.KIND_IALS, True)
    b = _run(monkeypatch, long_items, dim, fh.SIDE_ITEM, fh.KIND_IALS, False)
    np.testing.assert_array_equal(a, b)


def test_chol2_weighted_u_bit_identical(monkeypatch, long_items):
    a = _run(monkeypatch, long_items, 512, fh.SIDE_USER, fh.KIND_WEIGHTED_U, True)
    b = _run(monkeypatch, long_items, 512, fh.SIDE_USER, fh.KIND_WEIGHTED_U, False)
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("quirk", [True, False])
def test_chol2_weighted_v_bit_identical(monkeypatch, long_items, quirk):
    a = _run(monkeypatch, long_items, 512, fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, True, quirk)
    b = _run(monkeypatch, long_items, 512, fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, False, quirk)
    np.testing.assert_array_equal(a, b)


def test_chol2_not_spd_same_entity(monkeypatch, long_items):
    codes = []
    for two in (True, False):
        with pytest.raises(fh.FrecsysError) as ei:
            _run(monkeypatch, long_items, 512, fh.SIDE_ITEM, fh.KIND_IALS, two, reg=-50.0)
        codes.append((ei.value.code, ei.value.entity))
    assert codes[0] == codes[1]
    assert codes[0][0] == fh.ERR_NOT_SPD
