"""Wide dims, d = 512 / 1024 (Dp > 256, csrc/wide.hip): the Gramian by block
pairs, the per-step tridiagonalisation of the basis, the d-space solve with
A in an HBM workspace, the history-space solve at these widths, the CVaR-MF
gradient step and the user loss -- each against the CPU oracle with the
same bars as test_parity_gpu.py (1e-4 relative per row for embeddings).

The fixture is a smaller cut of conftest.make_quirk_data (400 x 300) so the
oracle's d^3/3 per entity stays cheap; it still has item histories above 256
(d-space even with the history-space path on), ProjectV tail-quirk items,
a 128-exact history and idle rows.  FRECSYS_DUAL=0 runs every entity
through the wide d-space kernels.
"""
import numpy as np
import pytest

import oracle as O
from conftest import make_quirk_data, rel_rows
from test_parity_gpu import _ctx, _v_inputs, _weights

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")

TOL_ROW = 1e-4


@pytest.fixture(scope="module")
def wide_data():
    return make_quirk_data(n_users=400, n_items=300, hot_frac=(0.40, 0.19, 0.29, 0.186, 0.7))


@pytest.fixture(params=["1", "0"], ids=["hspace", "dspace"])
def dual_mode(request, monkeypatch):
    monkeypatch.setenv("FRECSYS_DUAL", request.param)
    return request.param


def test_fixture_shape(wide_data):
    nu, ni, up, uc, ip, ic = wide_data
    h = np.diff(ip)
    assert h.max() > 256 and ((h > 128) & (h % 128 != 0)).sum() >= 2 and (h == 0).any()


@pytest.mark.parametrize("dim", [512, 1000])
@pytest.mark.parametrize("weighted", [False, True])
def test_wide_gramian(wide_data, dim, weighted):
    nu, ni, up, uc, ip, ic = wide_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    w = np.random.default_rng(3).random(nu).astype(np.float32) if weighted else None
    G = ctx.gramian(fh.SIDE_USER, weights=w)
    Gref = U.astype(np.float64).T @ (U.astype(np.float64) * (1 if w is None else w[:, None]))
    err = np.abs(G - Gref).max() / np.abs(Gref).max()
    assert err < 2e-6, err


@pytest.mark.parametrize("dim", [512, 700, 1024])
def test_wide_basis(wide_data, dim):
    nu, ni, up, uc, ip, ic = wide_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    rng = np.random.default_rng(4)
    X = (rng.standard_normal((nu, dim)) * np.geomspace(1.0, 0.03, dim)).astype(np.float32)
    ctx.set_embeddings(fh.SIDE_USER, X)
    G = ctx.gramian(fh.SIDE_USER).astype(np.float64)
    Q, dg, sb = ctx.debug_basis(fh.SIDE_USER)
    Dp = fh.padded_dim(dim)
    Q = Q.astype(np.float64)
    assert np.abs(Q.T @ Q - np.eye(Dp)).max() < 1e-5
    T = np.diag(dg.astype(np.float64)) + np.diag(sb[:-1].astype(np.float64), -1) \
        + np.diag(sb[:-1].astype(np.float64), 1)
    Gp = np.zeros((Dp, Dp))
    Gp[:dim, :dim] = G
    err = np.abs(Q @ T @ Q.T - Gp).max() / np.abs(Gp).max()
    assert err < 2e-5, err
    assert sb[-1] == 0.0


@pytest.mark.parametrize("dim", [500, 1024])
def test_wide_ials(wide_data, dual_mode, dim):
    nu, ni, up, uc, ip, ic = wide_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    reg, w = 0.003, 0.1
    ctx.gramian(fh.SIDE_ITEM)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, reg, w)
    Ug = ctx.get_embeddings(fh.SIDE_USER)
    Uo, rc = O.step(up, uc, V, O.gramian(V), 0, reg, w, out=U.copy())
    assert rc == 0
    assert rel_rows(Ug, Uo).max() < TOL_ROW
    np.testing.assert_array_equal(Ug[5], U[5])  # idle user untouched
    ctx.set_embeddings(fh.SIDE_USER, Uo)
    ctx.gramian(fh.SIDE_USER)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, reg, w)
    Vg = ctx.get_embeddings(fh.SIDE_ITEM)
    Vo, rc = O.step(ip, ic, Uo, O.gramian(Uo), 0, reg, w, out=V.copy())
    assert rc == 0
    assert rel_rows(Vg, Vo).max() < TOL_ROW
    np.testing.assert_array_equal(Vg[9], V[9])


@pytest.mark.parametrize("quirk", [True, False])
def test_wide_weighted_u_v(wide_data, dual_mode, quirk):
    nu, ni, up, uc, ip, ic = wide_data
    dim = 512
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic, quirks=quirk)
    om = _weights(nu)
    reg, w = 0.004, 0.004
    ctx.gramian(fh.SIDE_ITEM)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_WEIGHTED_U, reg, w, entity_weight=om)
    Uo, rc = O.step(up, uc, V, O.gramian(V), 1, reg, w, entity_weight=om, out=U.copy())
    assert rc == 0
    assert rel_rows(ctx.get_embeddings(fh.SIDE_USER), Uo).max() < TOL_ROW
    ctx.set_embeddings(fh.SIDE_USER, U)
    nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
    ctx.gramian(fh.SIDE_USER, weights=om)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, reg, w, alpha=0.3, entity_reg=item_reg,
                   other_weight=nu_w)
    Vo, rc = O.step(ip, ic, U, O.gramian(U, om), 2, reg, w, alpha=0.3, quirk=int(quirk),
                    entity_reg=item_reg, other_weight=nu_w, out=V.copy())
    assert rc == 0
    assert rel_rows(ctx.get_embeddings(fh.SIDE_ITEM), Vo).max() < TOL_ROW


def test_wide_cvar_grad(wide_data):
    nu, ni, up, uc, ip, ic = wide_data
    dim = 512
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    om = (np.random.default_rng(9).random(nu) < 0.4).astype(np.float32)
    reg, w, eta = 0.002, 0.008, 0.4
    ctx.gramian(fh.SIDE_ITEM)
    ctx.snapshot(fh.SIDE_USER)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_CVAR_GRAD_U, reg, w, stepsize=eta, entity_weight=om)
    Uo, _ = O.step(up, uc, V, O.gramian(V), 3, reg, w, stepsize=eta, entity_weight=om, E=U)
    assert rel_rows(ctx.get_embeddings(fh.SIDE_USER), Uo).max() < TOL_ROW
    nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
    ctx.gramian(fh.SIDE_USER, weights=om, from_snapshot=True)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_CVAR_GRAD_V, reg, w, alpha=0.3, stepsize=eta,
                   from_snapshot=True, entity_reg=item_reg, other_weight=nu_w)
    Vo, _ = O.step(ip, ic, U, O.gramian(U, om), 4, reg, w, alpha=0.3, stepsize=eta,
                   entity_reg=item_reg, other_weight=nu_w, E=V)
    assert rel_rows(ctx.get_embeddings(fh.SIDE_ITEM), Vo).max() < TOL_ROW


@pytest.mark.parametrize("dim", [512, 1024])
@pytest.mark.parametrize("half", [False, True])
def test_wide_user_loss(wide_data, dim, half):
    nu, ni, up, uc, ip, ic = wide_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    ctx.gramian(fh.SIDE_ITEM)
    lg = ctx.user_loss(fh.SIDE_USER, 0.1, half)
    lo = O.user_loss(up, uc, U, V, O.gramian(V), 0.1, half)
    np.testing.assert_allclose(lg, lo, rtol=2e-5, atol=1e-7)
    assert lg[5] == 0.0


@pytest.mark.parametrize("dim", [512, 1024])
def test_wide_not_spd_reported(wide_data, dim, monkeypatch):
    # every entity in d space: the wide Cholesky kernels themselves (at 1024
    # the two-panel one) must flag the failed pivot
    monkeypatch.setenv("FRECSYS_DUAL", "0")
    nu, ni, up, uc, ip, ic = wide_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    ctx.gramian(fh.SIDE_ITEM)
    with pytest.raises(fh.FrecsysError) as ei:
        ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, -50.0, 0.1)
    assert ei.value.code == fh.ERR_NOT_SPD


def test_wide_deterministic(wide_data):
    nu, ni, up, uc, ip, ic = wide_data
    outs = []
    for _ in range(2):
        ctx, U, V = _ctx(512, nu, ni, up, uc, ip, ic)
        ctx.gramian(fh.SIDE_USER)
        ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, 0.003, 0.1)
        outs.append(ctx.get_embeddings(fh.SIDE_ITEM))
    np.testing.assert_array_equal(outs[0], outs[1])
