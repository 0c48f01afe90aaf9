"""HIP path vs the CPU oracle (oracle/frecsys_oracle.c) on identical seeded
inputs.  Bar: fp32 embeddings within 1e-4 relative (per row), as north_star
states; Gramians / losses within fp32 summation-order noise.

All calls go through the C-ABI (libfrecsys_hip.so) via frecsys_hip.
"""
import numpy as np
import pytest

import oracle as O
from conftest import rel_rows

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")

TOL_ROW = 1e-4

DIMS = [8, 16, 5, 20, 32, 50, 64, 96, 128, 160, 192, 224, 256]


def _ctx(dim, nu, ni, up, uc, ip, ic, seed=1, quirks=True):
    ctx = fh.Context(dim, nu, ni, parity_quirks=quirks)
    ctx.load_csr(fh.SIDE_USER, up, uc)
    ctx.load_csr(fh.SIDE_ITEM, ip, ic)
    U, V = O.init_embeddings(seed, 0.1, dim, nu, ni)
    ctx.set_embeddings(fh.SIDE_USER, U)
    ctx.set_embeddings(fh.SIDE_ITEM, V)
    return ctx, U, V


def test_device_visible():
    assert fh.device_count() >= 1


@pytest.mark.parametrize("dim", [8, 20, 64, 256])
def test_init_embeddings_match_oracle(quirk_data, dim):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx = fh.Context(dim, nu, ni)
    ctx.init_embeddings(1234, 0.1)
    U0, V0 = O.init_embeddings(1234, 0.1, dim, nu, ni)
    np.testing.assert_array_equal(ctx.get_embeddings(fh.SIDE_USER), U0)
    np.testing.assert_array_equal(ctx.get_embeddings(fh.SIDE_ITEM), V0)


@pytest.mark.parametrize("dim", DIMS)
@pytest.mark.parametrize("weighted", [False, True])
def test_gramian(quirk_data, dim, weighted):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    w = np.random.default_rng(3).random(nu).astype(np.float32) if weighted else None
    G = ctx.gramian(fh.SIDE_USER, weights=w)
    Gref = U.astype(np.float64).T @ (U.astype(np.float64) * (1 if w is None else w[:, None]))
    err = np.abs(G - Gref).max() / np.abs(Gref).max()
    assert err < 2e-6, err
    np.testing.assert_allclose(G, O.gramian(U, w), rtol=2e-5, atol=2e-7 * np.abs(Gref).max())


@pytest.mark.parametrize("dim", DIMS)
def test_ials_half_steps(quirk_data, dim):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    reg, w = 0.003, 0.1
    Gv = ctx.gramian(fh.SIDE_ITEM)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, reg, w)
    Ug = ctx.get_embeddings(fh.SIDE_USER)
    Uo, rc = O.step(up, uc, V, O.gramian(V), 0, reg, w, out=U.copy())
    assert rc == 0
    assert rel_rows(Ug, Uo).max() < TOL_ROW
    # idle user untouched
    np.testing.assert_array_equal(Ug[5], U[5])
    # V half-step from identical U
    ctx.set_embeddings(fh.SIDE_USER, Uo)
    ctx.gramian(fh.SIDE_USER)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, reg, w)
    Vg = ctx.get_embeddings(fh.SIDE_ITEM)
    Vo, rc = O.step(ip, ic, Uo, O.gramian(Uo), 0, reg, w, out=V.copy())
    assert rc == 0
    assert rel_rows(Vg, Vo).max() < TOL_ROW
    np.testing.assert_array_equal(Vg[9], V[9])
    del Gv


@pytest.mark.parametrize("dim", [8, 16, 32, 64, 96, 256])
@pytest.mark.parametrize("reg_exp", [1.0, 0.5])
def test_ials_reg_exp(quirk_data, dim, reg_exp):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    ctx.gramian(fh.SIDE_ITEM)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, 0.01, 0.05, reg_exp=reg_exp)
    Uo, rc = O.step(up, uc, V, O.gramian(V), 0, 0.01, 0.05, reg_exp=reg_exp, out=U.copy())
    assert rel_rows(ctx.get_embeddings(fh.SIDE_USER), Uo).max() < TOL_ROW


def _weights(nu, seed=5):
    return (0.05 + 0.95 * np.random.default_rng(seed).random(nu)).astype(np.float32)


@pytest.mark.parametrize("dim", DIMS)
def test_weighted_u(quirk_data, dim):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    om = _weights(nu)
    reg, w = 0.004, 0.004
    ctx.gramian(fh.SIDE_ITEM)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_WEIGHTED_U, reg, w, entity_weight=om)
    Uo, rc = O.step(up, uc, V, O.gramian(V), 1, reg, w, entity_weight=om, out=U.copy())
    assert rc == 0
    assert rel_rows(ctx.get_embeddings(fh.SIDE_USER), Uo).max() < TOL_ROW


def _v_inputs(nu, ni, up, ip, ic, om):
    h = np.diff(up).astype(np.float32)
    # nu_u = omega_u / |H_u| (safer2.h:499-501); an idle user (h = 0) is in no
    # item's history, so its nu is never read: pass 0 instead of inf / NaN
    nu_w = np.where(h > 0, om / np.maximum(h, 1), 0).astype(np.float32)
    item_reg = np.zeros(ni, np.float32)
    for v in range(ni):
        acc = np.float32(0)
        for u in ic[ip[v]:ip[v + 1]]:
            acc = np.float32(np.float64(acc) + 1.0 / np.float64(h[u]))
        item_reg[v] = acc
    return nu_w, item_reg


@pytest.mark.parametrize("dim", DIMS)
@pytest.mark.parametrize("quirk", [True, False])
def test_weighted_v(quirk_data, dim, quirk):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic, quirks=quirk)
    om = _weights(nu)
    nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
    reg, w, alpha = 0.004, 0.004, 0.3
    G = ctx.gramian(fh.SIDE_USER, weights=om)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, reg, w, alpha=alpha, entity_reg=item_reg,
                   other_weight=nu_w)
    Vo, rc = O.step(ip, ic, U, O.gramian(U, om), 2, reg, w, alpha=alpha, quirk=int(quirk),
                    entity_reg=item_reg, other_weight=nu_w, out=V.copy())
    assert rc == 0
    assert rel_rows(ctx.get_embeddings(fh.SIDE_ITEM), Vo).max() < TOL_ROW
    del G


def test_tail_quirk_changes_result(quirk_data):
    """The quirk must matter on items with h > 128, h % 128 != 0 and only there."""
    nu, ni, up, uc, ip, ic = quirk_data
    dim = 32
    om = _weights(nu)
    nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
    outs = []
    for q in (True, False):
        ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic, quirks=q)
        ctx.gramian(fh.SIDE_USER, weights=om)
        ctx.solve_side(fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, 0.004, 0.004, alpha=0.3,
                       entity_reg=item_reg, other_weight=nu_w)
        outs.append(ctx.get_embeddings(fh.SIDE_ITEM))
    h = np.diff(ip)
    affected = (h > 128) & (h % 128 != 0)
    assert affected.sum() >= 3
    diff = np.abs(outs[0] - outs[1]).max(axis=1)
    assert (diff[affected] > 0).all()
    np.testing.assert_array_equal(outs[0][~affected], outs[1][~affected])


@pytest.mark.parametrize("dim", DIMS)
def test_cvar_grad_steps(quirk_data, dim):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    om = (np.random.default_rng(9).random(nu) < 0.4).astype(np.float32)
    reg, w, eta = 0.002, 0.008, 0.4
    ctx.gramian(fh.SIDE_ITEM)
    ctx.snapshot(fh.SIDE_USER)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_CVAR_GRAD_U, reg, w, stepsize=eta, entity_weight=om)
    Uo, _ = O.step(up, uc, V, O.gramian(V), 3, reg, w, stepsize=eta, entity_weight=om, E=U)
    assert rel_rows(ctx.get_embeddings(fh.SIDE_USER), Uo).max() < TOL_ROW
    # V step on the pre-step U (snapshot), cvar_mf.h:282,294
    nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
    ctx.gramian(fh.SIDE_USER, weights=om, from_snapshot=True)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_CVAR_GRAD_V, reg, w, alpha=0.3, stepsize=eta,
                   from_snapshot=True, entity_reg=item_reg, other_weight=nu_w)
    Vo, _ = O.step(ip, ic, U, O.gramian(U, om), 4, reg, w, alpha=0.3, stepsize=eta,
                   entity_reg=item_reg, other_weight=nu_w, E=V)
    assert rel_rows(ctx.get_embeddings(fh.SIDE_ITEM), Vo).max() < TOL_ROW


@pytest.mark.parametrize("dim", [8, 16, 32, 64, 100, 256])
@pytest.mark.parametrize("half", [False, True])
def test_user_loss(quirk_data, dim, half):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    ctx.gramian(fh.SIDE_ITEM)
    lg = ctx.user_loss(fh.SIDE_USER, 0.1, half)
    lo = O.user_loss(up, uc, U, V, O.gramian(V), 0.1, half)
    np.testing.assert_allclose(lg, lo, rtol=2e-5, atol=1e-7)
    assert lg[5] == 0.0  # idle user never written


def test_eval_side_fold_in(ml1m):
    tr, vt, ve = ml1m
    nu, ni = tr.max_user + 1, tr.max_item + 1
    up, uc = tr.by_user()
    ip, ic = tr.by_item()
    ctx, U, V = _ctx(32, nu, ni, up, uc, ip, ic)
    ids, ep, ec = vt.compact_users()
    ctx.load_csr(fh.SIDE_EVAL, ep, ec)
    ctx.gramian(fh.SIDE_ITEM)
    ctx.solve_side(fh.SIDE_EVAL, fh.KIND_IALS, 0.003, 0.1)
    Ue = ctx.get_embeddings(fh.SIDE_EVAL)
    Uo, rc = O.step(ep, ec, V, O.gramian(V), 0, 0.003, 0.1)
    assert rel_rows(Ue, Uo).max() < TOL_ROW


@pytest.mark.parametrize("dim", [64, 128, 256])
def test_not_spd_reported(quirk_data, dim):
    # d = 64 runs the 4-wave Cholesky, d >= 96 the 8-wave dataflow one whose
    # forward substitution has its own wave (chol.h chol_solve_df, NW >= 8)
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    ctx.gramian(fh.SIDE_ITEM)
    with pytest.raises(fh.FrecsysError) as ei:
        ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, -50.0, 0.1)  # negative lambda
    assert ei.value.code == fh.ERR_NOT_SPD
    assert 0 <= ei.value.entity < nu


def _rank_deficient_case(dim):
    """40 items at d = 64..256: G = V^T V has rank <= 40, so with a vanishing
    lambda both M = w G + lam I (history space) and A (d space) are singular
    up to fp32 rounding -- pivots fail on either path."""
    rng = np.random.default_rng(11)
    nu, ni = 100, 40
    users = np.repeat(np.arange(nu), 12)
    items = np.concatenate([rng.choice(ni, 12, replace=False) for _ in range(nu)])
    from frecsys_hip.data import _csr_from_pairs
    up, uc = _csr_from_pairs(users, items, nu)
    ip, ic = _csr_from_pairs(items, users, ni)
    return nu, ni, up, uc, ip, ic


@pytest.mark.parametrize("dim", [64, 128, 256])
def test_not_spd_history_space_falls_back(monkeypatch, dim):
    """A failed history-space pivot reruns the whole call on the d-space
    path, so the verdict (error code, entity, or the rows) is exactly the
    FRECSYS_DUAL=0 one."""
    nu, ni, up, uc, ip, ic = _rank_deficient_case(dim)
    res = []
    for dual in ("0", "1"):
        monkeypatch.setenv("FRECSYS_DUAL", dual)
        ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
        ctx.gramian(fh.SIDE_ITEM)
        try:
            ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, 1e-35, 1.0)
            res.append((0, -1, ctx.get_embeddings(fh.SIDE_USER)))
        except fh.FrecsysError as e:
            res.append((e.code, e.entity, None))
        res[-1] += (ctx.timing("solve_user")[1], ctx.timing("solve_user.hspace")[1])
        ctx.close()
    (c0, e0, x0, n0, _), (c1, e1, x1, n1, hs1) = res
    assert hs1 == 1 and n1 == 2 and n0 == 1  # history space ran, failed, d-space reran
    assert (c1, e1) == (c0, e0)
    if c0 == 0:
        np.testing.assert_array_equal(x1, x0)


def test_bad_csr_rejected(quirk_data):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx = fh.Context(16, nu, ni)
    bad = uc.copy()
    bad[3] = ni + 5
    with pytest.raises(fh.FrecsysError) as ei:
        ctx.load_csr(fh.SIDE_USER, up, bad)
    assert ei.value.code == fh.ERR_INVALID


def test_unsupported_dim():
    with pytest.raises(fh.FrecsysError) as ei:
        fh.Context(1025, 10, 10)
    assert ei.value.code == fh.ERR_UNSUPPORTED
