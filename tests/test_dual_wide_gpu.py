"""The history-space wide bucket (dual.hip dual_wide_*: 256 < h_eff <= 512 at
Dp = 512 / 1024, S = I + Z D^-1 Z^T through HBM workspaces and the wide
Cholesky) against the d-space solve of the same entities (FRECSYS_DUAL=0)
and the oracle, every row at the 1e-4 bar (the same bar as test_dual_gpu.py):
iALS on both sides (tridiagonal basis, and the Cholesky basis of
l2_reg_exp = 0), ProjectU with entity weights, ProjectV with and without
the tail quirk (h_eff up to 512 includes the quirk rows).  At Dp = 1024
(d = 1000, 1024: config 5's dims, SAFER2 = the weighted kinds) the bucket is on
by default, so those cases run with no FRECSYS_* override at all; at Dp = 512
the threshold is raised to 512 to reach it.  Margins go to parity_report.jsonl.
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
def mid_data():
    """Users with 1..600 rows, items with ~250..500: both sides fill the
    wide bucket, the tridiagonal buckets below it and the d-space above."""
    rng = np.random.default_rng(5)
    n_users, n_items = 1500, 1200
    hs = rng.integers(1, 600, n_users)
    users, items = [], []
    for u, h in enumerate(hs):
        its = rng.choice(n_items, int(h), replace=False)
        users.append(np.full(len(its), u))
        items.append(its)
    users = np.concatenate(users).astype(np.int64)
    items = np.concatenate(items).astype(np.int64)
    from frecsys_hip.data import _csr_from_pairs
    up, uc = _csr_from_pairs(users, items, n_users)
    ip, ic = _csr_from_pairs(items, users, n_items)
    return n_users, n_items, up, uc, ip, ic


def _heff(h, quirk):
    return np.where(quirk & (h > 128) & (h % 128 != 0), h + 128 - h % 128, h)


def _run(monkeypatch, data, dim, side, kind, wide, quirk=True, reg_exp=1.0):
    monkeypatch.delenv("FRECSYS_DUAL", raising=False)
    monkeypatch.delenv("FRECSYS_DUAL_MAX_H", raising=False)
    if not wide:
        monkeypatch.setenv("FRECSYS_DUAL", "0")  # the d-space reference run
    elif fh.padded_dim(dim) < 1024:
        monkeypatch.setenv("FRECSYS_DUAL_MAX_H", "512")  # default 256 at Dp = 512
    nu, ni, up, uc, ip, ic = data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic, quirks=quirk)
    om = _weights(nu)
    kw = {}
    if side == fh.SIDE_USER:
        ctx.gramian(fh.SIDE_ITEM)
        args = (0.003, 0.1) if kind == fh.KIND_IALS else (0.004, 0.004)
        if kind == fh.KIND_WEIGHTED_U:
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
    if kind == fh.KIND_IALS:
        kw["reg_exp"] = reg_exp
    tag = "solve_user" if side == fh.SIDE_USER else "solve_item"
    ctx.timing_reset()
    ctx.solve_side(side, kind, *args, **kw)
    n_hs = ctx.work(tag + ".hspace")[2]
    assert ctx.counter("hspace_reruns") == 0
    out = ctx.get_embeddings(side)
    ctx.close()
    return out, (U, V, om, args, kw), n_hs


def _check(monkeypatch, data, dim, side, kind, okind, quirk=True, reg_exp=1.0):
    nu, ni, up, uc, ip, ic = data
    Xw, (U, V, om, args, kw), n_hs = _run(monkeypatch, data, dim, side, kind, True, quirk, reg_exp)
    Xd, _, n0 = _run(monkeypatch, data, dim, side, kind, False, quirk, reg_exp)
    ptr = up if side == fh.SIDE_USER else ip
    h = np.diff(ptr)
    he = _heff(h, quirk and kind == fh.KIND_WEIGHTED_V)
    wide = (he > 256) & (he <= 512)
    assert n0 == 0 and n_hs == int(((he > 0) & (he <= 512)).sum()) and wide.sum() >= 50
    if side == fh.SIDE_USER:
        G = O.gramian(V) if kind == fh.KIND_IALS else O.gramian(V)
        okw = dict(kw)
        Xo, rc = O.step(up, uc, V, G, okind, *args, out=U.copy(), **okw)
    else:
        G = O.gramian(U) if kind == fh.KIND_IALS else O.gramian(U, om)
        Xo, rc = O.step(ip, ic, U, G, okind, *args, quirk=int(quirk), out=V.copy(), **kw)
    assert rc == 0
    ew, ed = rel_rows(Xw, Xo), rel_rows(Xd, Xo)
    print(f"side {side} dim {dim} kind {kind}: wide bucket {ew[wide].max():.2e} "
          f"(all rows {ew.max():.2e}), d-space {ed[wide].max():.2e}")
    from test_models_gpu import report
    report(test="wide_bucket", side=int(side), dim=dim, kind=kind, quirk=bool(quirk),
           reg_exp=reg_exp, wide_rows=int(wide.sum()), max_wide_bucket=float(ew[wide].max()),
           max_all=float(ew.max()), max_dspace=float(ed.max()), margin=TOL_ROW / float(ew.max()))
    assert ew.max() < TOL_ROW, (ew[wide].max(), ew.max())
    assert ed.max() < TOL_ROW


@pytest.mark.parametrize("side", ["user", "item"])
@pytest.mark.parametrize("dim", [512, 1000])
def test_wide_bucket_ials(monkeypatch, mid_data, dim, side):
    s = fh.SIDE_USER if side == "user" else fh.SIDE_ITEM
    _check(monkeypatch, mid_data, dim, s, fh.KIND_IALS, 0)


def test_wide_bucket_ials_chol_basis(monkeypatch, mid_data):
    # l2_reg_exp = 0: one M for every entity, the Cholesky basis (unit table)
    _check(monkeypatch, mid_data, 512, fh.SIDE_USER, fh.KIND_IALS, 0, reg_exp=0.0)


@pytest.mark.parametrize("dim", [512, 1000, 1024])
def test_wide_bucket_weighted_u(monkeypatch, mid_data, dim):
    # ProjectU (omega) -- config 5's user side at d = 1024
    _check(monkeypatch, mid_data, dim, fh.SIDE_USER, fh.KIND_WEIGHTED_U, 1)


@pytest.mark.parametrize("dim", [512, 1000, 1024])
@pytest.mark.parametrize("quirk", [True, False])
def test_wide_bucket_weighted_v(monkeypatch, mid_data, quirk, dim):
    # ProjectV (nu, item_reg), with and without the tail quirk -- config 5's
    # item side at d = 1024
    _check(monkeypatch, mid_data, dim, fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, 2, quirk=quirk)
