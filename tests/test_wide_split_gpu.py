"""Long-history split of the wide d-space SYRK (csrc/wide.hip
wide_syrk2_kernel<2>): at Dp = 512 / 1024 the SYRK of an entity with more
than 2 * 2048 assembly rows is cut into 2048-row slabs (the two-level
accumulation block), computed by their own workgroups, and folded left to
right by the entity's workgroup -- the same additions in the same order as the
unsplit kernel, so the result must be bit-identical to FRECSYS_SPLIT_ROWS=0
(split off) and within 1e-4 per row of the oracle.

Fixture: 12,000 users x 40 items; items 0..5 have 9,000 / 6,150 / 4,097 /
8,192 / 4,100 / 2,500 histories (non-multiples of 128 for the ProjectV
tail-quirk rows that straddle slab boundaries, one exact multiple of the
slab, one just past the split threshold, one below it), the rest 40..600.
"""
import numpy as np
import pytest

import oracle as O
from conftest import rel_rows
from test_parity_gpu import _ctx, _v_inputs, _weights

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")

TOL_ROW = 1e-4


@pytest.fixture(scope="module")
def long_items():
    rng = np.random.default_rng(21)
    n_users, n_items = 12000, 40
    hs = [9000, 6150, 4097, 8192, 4100, 2500] + list(rng.integers(40, 600, n_items - 6))
    users, items = [], []
    for it, h in enumerate(hs):
        us = rng.choice(n_users, int(h), replace=False)
        users.append(us)
        items.append(np.full(len(us), it))
    users = np.concatenate(users).astype(np.int64)
    items = np.concatenate(items).astype(np.int64)
    perm = rng.permutation(len(users))  # file order: interleaved
    users, items = users[perm], items[perm]
    from frecsys_hip.data import _csr_from_pairs
    up, uc = _csr_from_pairs(users, items, n_users)
    ip, ic = _csr_from_pairs(items, users, n_items)
    return n_users, n_items, up, uc, ip, ic


def _solve_items(monkeypatch, data, dim, kind, split, quirk=True):
    monkeypatch.setenv("FRECSYS_SPLIT_ROWS", "1024" if split else "0")
    nu, ni, up, uc, ip, ic = data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic, quirks=quirk)
    kw = {}
    om = _weights(nu)
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
    ctx.solve_side(fh.SIDE_ITEM, kind, *args, **kw)
    return ctx.get_embeddings(fh.SIDE_ITEM), (U, V, om, args, kw)


@pytest.mark.parametrize("dim", [512, 1000])
def test_wide_split_ials_bit_identical_and_parity(monkeypatch, long_items, dim):
    Vs, (U, V, _, args, _) = _solve_items(monkeypatch, long_items, dim, fh.KIND_IALS, True)
    Vn, _ = _solve_items(monkeypatch, long_items, dim, fh.KIND_IALS, False)
    np.testing.assert_array_equal(Vs, Vn)
    nu, ni, up, uc, ip, ic = long_items
    Vo, rc = O.step(ip, ic, U, O.gramian(U), 0, *args, out=V.copy())
    assert rc == 0
    err = rel_rows(Vs, Vo)
    print(f"wide split iALS d={dim}: max row error {err.max():.2e} (items 0..5 {err[:6]})")
    assert err.max() < TOL_ROW


@pytest.mark.parametrize("quirk", [True, False])
def test_wide_split_weighted_v(monkeypatch, long_items, quirk):
    Vs, (U, V, om, args, kw) = _solve_items(monkeypatch, long_items, 512, fh.KIND_WEIGHTED_V,
                                             True, quirk)
    Vn, _ = _solve_items(monkeypatch, long_items, 512, fh.KIND_WEIGHTED_V, False, quirk)
    np.testing.assert_array_equal(Vs, Vn)
    nu, ni, up, uc, ip, ic = long_items
    Vo, rc = O.step(ip, ic, U, O.gramian(U, om), 2, *args, quirk=int(quirk), out=V.copy(), **kw)
    assert rc == 0
    assert rel_rows(Vs, Vo).max() < TOL_ROW


def test_wide_split_cvar_grad_v(monkeypatch, long_items):
    Vs, _ = _solve_items(monkeypatch, long_items, 512, fh.KIND_CVAR_GRAD_V, True)
    Vn, _ = _solve_items(monkeypatch, long_items, 512, fh.KIND_CVAR_GRAD_V, False)
    np.testing.assert_array_equal(Vs, Vn)


def test_wide_split_small_budget(monkeypatch, long_items):
    # a slab budget below the longest entity's slab count: the plan stops at
    # the budget (longest first); the rest run unsplit, results unchanged
    # 8 MB: batches of 14 entities, at most 14 slabs of 561 KB -- items 0, 3
    # and 1 (5 + 4 + 4 slabs) split, item 4 (3 more) not
    monkeypatch.setenv("FRECSYS_WIDE_WS_MB", "8")
    Vs, _ = _solve_items(monkeypatch, long_items, 512, fh.KIND_IALS, True)
    monkeypatch.delenv("FRECSYS_WIDE_WS_MB")
    Vn, _ = _solve_items(monkeypatch, long_items, 512, fh.KIND_IALS, False)
    np.testing.assert_array_equal(Vs, Vn)
