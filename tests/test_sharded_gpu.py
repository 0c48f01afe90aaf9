"""The product's sharded (N-rank) path on one GPU, through the real C-ABI.

RCCL cannot put two ranks on one device ("Duplicate GPU detected"), so the
8-GPU path is rehearsed here with W contexts of one process on cuda:0, each
joined as rank r of W in external-exchange mode (frecsys_comm_init with no
id): each context computes the partial Gramian over its own rows, solves
only its nnz-balanced row range (its own LPT queue, its own d-space /
history-space split) and computes the loss of its own users -- exactly what
a rank does between collectives -- while the test performs the exchange the
library does over RCCL (sum of partial Gramians = ncclAllReduce; rows of
every rank copied to all = the grouped ncclBroadcast all-gather; losses
likewise).  The result must match the single-context run: solves are
per-entity independent, so the only difference is the Gramian's summation
order (fp32 noise, well inside the 1e-4 bar).
"""
import numpy as np
import pytest

import frecsys_hip as fh
from conftest import rel_rows

pytestmark = pytest.mark.gpu


def _contexts(world, dim, nu, ni, up, uc, ip, ic):
    ctxs = []
    for r in range(world):
        c = fh.Context(dim, nu, ni, device=0)
        if world > 1:
            c.comm_init(world, r, None)
        c.load_csr(fh.SIDE_USER, up, uc)
        c.load_csr(fh.SIDE_ITEM, ip, ic)
        c.init_embeddings(1, 0.1)
        ctxs.append(c)
    return ctxs


def _allreduce_gram(ctxs, side, weights=None):
    parts = [c.gramian(side, weights) for c in ctxs]
    if len(ctxs) == 1:
        return parts[0]
    G = np.sum(np.stack(parts).astype(np.float64), axis=0).astype(np.float32)
    for c in ctxs:
        c.set_gramian(side, G)
    return G


def _allgather_rows(ctxs, side):
    if len(ctxs) == 1:
        return ctxs[0].get_embeddings(side)
    full = ctxs[0].get_embeddings(side)
    for c in ctxs[1:]:
        lo, hi = c.shard_range(side)
        full[lo:hi] = c.get_embeddings(side)[lo:hi]
    for c in ctxs:
        c.set_embeddings(side, full)
    return full


def _allgather_loss(ctxs, w):
    outs = [c.user_loss(fh.SIDE_USER, w, True) for c in ctxs]
    full = outs[0].copy()
    for c, o in zip(ctxs[1:], outs[1:]):
        lo, hi = c.shard_range(fh.SIDE_USER)
        full[lo:hi] = o[lo:hi]
    return full


def _ials_epochs(ctxs, epochs, reg, w):
    for _ in range(epochs):                                      # ials.h:187-206
        _allreduce_gram(ctxs, fh.SIDE_ITEM)
        for c in ctxs:
            c.solve_side(fh.SIDE_USER, fh.KIND_IALS, reg, w)
        _allgather_rows(ctxs, fh.SIDE_USER)
        _allreduce_gram(ctxs, fh.SIDE_USER)
        for c in ctxs:
            c.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, reg, w)
        _allgather_rows(ctxs, fh.SIDE_ITEM)
    return ctxs[0].get_embeddings(fh.SIDE_USER), ctxs[0].get_embeddings(fh.SIDE_ITEM)


def _close(ctxs):
    for c in ctxs:
        c.close()


@pytest.fixture(scope="module")
def ml1m_csr(ml1m):
    tr, _, _ = ml1m
    up, uc = tr.by_user()
    ip, ic = tr.by_item()
    return tr.max_user + 1, tr.max_item + 1, up, uc, ip, ic


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("dim", [32, 64, 256])
def test_sharded_ials_matches_single(ml1m_csr, world, dim):
    nu, ni, up, uc, ip, ic = ml1m_csr
    reg, w = 0.003, 0.1
    single = _contexts(1, dim, nu, ni, up, uc, ip, ic)
    U1, V1 = _ials_epochs(single, 2, reg, w)
    _close(single)
    ctxs = _contexts(world, dim, nu, ni, up, uc, ip, ic)
    # the shards tile the rows and are nnz-balanced like frecsys_partition
    for side, ptr in ((fh.SIDE_USER, up), (fh.SIDE_ITEM, ip)):
        b = fh.partition(ptr, world)
        assert [c.shard_range(side) for c in ctxs] == [(int(b[r]), int(b[r + 1]))
                                                         for r in range(world)]
    Uw, Vw = _ials_epochs(ctxs, 2, reg, w)
    _close(ctxs)
    eu, ev = rel_rows(Uw, U1), rel_rows(Vw, V1)
    assert eu.max() < 1e-4 and ev.max() < 1e-4, (eu.max(), ev.max())


def test_sharded_rank_touches_only_its_rows(ml1m_csr):
    """Without the exchange, a rank's solve leaves every other row as it was."""
    nu, ni, up, uc, ip, ic = ml1m_csr
    ctxs = _contexts(3, 64, nu, ni, up, uc, ip, ic)
    U0 = ctxs[1].get_embeddings(fh.SIDE_USER)
    _allreduce_gram(ctxs, fh.SIDE_ITEM)
    ctxs[1].solve_side(fh.SIDE_USER, fh.KIND_IALS, 0.003, 0.1)
    U = ctxs[1].get_embeddings(fh.SIDE_USER)
    lo, hi = ctxs[1].shard_range(fh.SIDE_USER)
    assert 0 < lo < hi < nu
    assert np.array_equal(U[:lo], U0[:lo]) and np.array_equal(U[hi:], U0[hi:])
    assert not np.array_equal(U[lo:hi], U0[lo:hi])
    _close(ctxs)


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_safer2_halfsteps_match_single(ml1m_csr, world):
    """SAFER2's weighted kinds and the gathered loss on shards
    (safer2.h:277-299): ProjectU with omega, the omega-weighted U Gramian,
    ProjectV with nu and the item regulariser (tail quirk on), V^T V, loss."""
    nu, ni, up, uc, ip, ic = ml1m_csr
    dim, reg, w, alpha = 64, 0.004, 0.004, 0.3
    rng = np.random.default_rng(5)
    omega = rng.uniform(0.05, 1.0, nu).astype(np.float32)
    hu = np.diff(up).astype(np.float32)
    nu_w = np.where(hu > 0, omega / np.maximum(hu, 1), 0).astype(np.float32)
    item_reg = np.zeros(ni, np.float32)
    inv_h = np.where(hu > 0, 1.0 / np.maximum(hu, 1), 0).astype(np.float32)
    for i in range(ni):
        for u in ic[ip[i]:ip[i + 1]]:
            item_reg[i] += inv_h[u]

    def run(world_):
        ctxs = _contexts(world_, dim, nu, ni, up, uc, ip, ic)
        _allreduce_gram(ctxs, fh.SIDE_ITEM)
        for c in ctxs:
            c.solve_side(fh.SIDE_USER, fh.KIND_WEIGHTED_U, reg, w, alpha=alpha, entity_weight=omega)
        _allgather_rows(ctxs, fh.SIDE_USER)
        _allreduce_gram(ctxs, fh.SIDE_USER, weights=omega)
        for c in ctxs:
            c.solve_side(fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, reg, w, alpha=alpha,
                         entity_reg=item_reg, other_weight=nu_w)
        _allgather_rows(ctxs, fh.SIDE_ITEM)
        _allreduce_gram(ctxs, fh.SIDE_ITEM)
        loss = _allgather_loss(ctxs, w)
        U, V = ctxs[0].get_embeddings(fh.SIDE_USER), ctxs[0].get_embeddings(fh.SIDE_ITEM)
        _close(ctxs)
        return U, V, loss

    U1, V1, l1 = run(1)
    Uw, Vw, lw = run(world)
    eu, ev = rel_rows(Uw, U1), rel_rows(Vw, V1)
    assert eu.max() < 1e-4 and ev.max() < 1e-4, (eu.max(), ev.max())
    np.testing.assert_allclose(lw, l1, rtol=1e-4, atol=1e-7)
