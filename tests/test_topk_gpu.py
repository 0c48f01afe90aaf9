"""Fold-in scoring + top-K on the GPU (csrc/topk.hip, frecsys_eval_topk):
the ranking half of EvaluateDatasetInternal / EvaluateUser
(recommender.h:78-199) against a float64 numpy ranking of the same
embeddings -- history items excluded, scores non-increasing, and the GPU's
k items equal to the exact top k except where scores tie within fp32
rounding of the k-th one.  Exact ties are broken by item id.
"""
import numpy as np
import pytest

import oracle as O
from conftest import make_quirk_data
from test_parity_gpu import _ctx

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")


def _ref_topk(Ue, V, ep, ec, k):
    S = Ue.astype(np.float64) @ V.astype(np.float64).T
    for r in range(len(ep) - 1):
        S[r, ec[ep[r]:ep[r + 1]]] = -np.inf
    order = np.lexsort((np.broadcast_to(np.arange(S.shape[1]), S.shape), -S), axis=1)
    return S, order[:, :k]


def _check(top, S, ref, ep, ec, k):
    n = top.shape[0]
    scale = np.abs(S[np.isfinite(S)]).max()
    tol = 2e-6 * scale
    for r in range(n):
        t = top[r]
        assert len(set(t.tolist())) == k
        hist = set(ec[ep[r]:ep[r + 1]].tolist())
        assert not (set(t.tolist()) & hist) or len(hist) + k > S.shape[1]
        st = S[r, t]
        assert np.all(np.diff(st) <= tol), r
        kth = S[r, ref[r, -1]]
        # everything strictly better than the k-th (beyond rounding) is in the list
        must = set(np.where(S[r] > kth + tol)[0].tolist())
        assert must <= set(t.tolist()), r
        assert np.all(st >= kth - tol), r


@pytest.mark.parametrize("dim", [8, 20, 64, 256])
@pytest.mark.parametrize("k", [1, 20, 100])
def test_topk_ml1m_fold_in(ml1m, dim, k):
    tr, vt, ve = ml1m
    nu, ni = tr.max_user + 1, tr.max_item + 1
    up, uc = tr.by_user()
    ip, ic = tr.by_item()
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    ids, ep, ec = vt.compact_users()
    ctx.load_csr(fh.SIDE_EVAL, ep, ec)
    ctx.gramian(fh.SIDE_ITEM)
    ctx.solve_side(fh.SIDE_EVAL, fh.KIND_IALS, 0.003, 0.1)
    Ue = ctx.get_embeddings(fh.SIDE_EVAL)
    top = ctx.eval_topk(k)
    S, ref = _ref_topk(Ue, V, ep, ec, k)
    _check(top, S, ref, ep, ec, k)
    # the lists agree with the exact ranking almost everywhere
    assert np.mean(np.all(top == ref, axis=1)) > 0.97


@pytest.mark.parametrize("dim", [32, 512])
def test_topk_wide_and_large_k(dim):
    nu, ni, up, uc, ip, ic = make_quirk_data(n_users=300, n_items=1500)
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    ctx.load_csr(fh.SIDE_EVAL, up, uc)
    ctx.set_embeddings(fh.SIDE_EVAL, U)
    for k in (7, 1024):
        top = ctx.eval_topk(k)
        S, ref = _ref_topk(U, V, up, uc, k)
        _check(top, S, ref, up, uc, k)


def test_topk_ties_by_item_id():
    rng = np.random.default_rng(2)
    nu, ni, dim = 40, 300, 32
    up = np.arange(nu + 1, dtype=np.int64)           # one history item per user
    uc = rng.integers(0, ni, nu).astype(np.int32)
    ctx = fh.Context(dim, nu, ni)
    V = rng.standard_normal((ni, dim)).astype(np.float32)
    V[200:260] = V[5]                                 # 61 identical item rows
    ctx.set_embeddings(fh.SIDE_ITEM, V)
    ctx.load_csr(fh.SIDE_EVAL, up, uc)
    Ue = np.tile(V[5], (nu, 1)).astype(np.float32)    # the tied items score highest
    ctx.set_embeddings(fh.SIDE_EVAL, Ue)
    top = ctx.eval_topk(30)
    for r in range(nu):
        tied = [j for j in [5] + list(range(200, 260)) if j != uc[r]]
        assert top[r].tolist() == tied[:30], r


def test_topk_bad_k():
    nu, ni, up, uc, ip, ic = make_quirk_data(n_users=50, n_items=40)
    ctx, U, V = _ctx(16, nu, ni, up, uc, ip, ic)
    ctx.load_csr(fh.SIDE_EVAL, up, uc)
    for k in (0, 41, 2000):
        with pytest.raises(fh.FrecsysError) as ei:
            ctx.eval_topk(k)
        assert ei.value.code == fh.ERR_INVALID
