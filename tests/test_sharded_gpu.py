"""The product's sharded (N-rank) path on one GPU, through the real C-ABI.

RCCL cannot put two ranks on one device ("Duplicate GPU detected"), so the
8-GPU path is rehearsed here with W contexts of one process on cuda:0, each
joined as rank r of W in external-exchange mode (frecsys_comm_init with no
id): each context computes the partial Gramian over its own rows, solves
only its nnz-balanced row range (its own LPT queue, its own d-space /
history-space split) and computes the loss of its own users -- exactly what
a rank does between collectives -- while the test performs the exchange the
library does over RCCL (the Gramian's group slabs gathered from their owners
= the grouped ncclBroadcast of frecsys_gramian, then summed in group order by
frecsys_set_gram_groups; rows of every rank copied to all = the factor
all-gather; losses likewise).  The result must equal the single-context run
BIT FOR BIT: solves are per-entity independent and the Gramian
is partition-independent (fixed leaves and groups, fixed summation order).
"""
import numpy as np
import pytest

import frecsys_hip as fh

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
    # the exchange frecsys_gramian does over RCCL: every group slab from its owner
    slabs = None
    for c in ctxs:
        ng, lo, hi, _ = c.gram_groups(side)
        mine = c.get_gram_groups(side)
        if slabs is None:
            slabs = np.zeros_like(mine)
        assert not mine[:lo].any() and not mine[hi:].any()  # only its own groups
        slabs[lo:hi] = mine[lo:hi]
    owned = sorted(c.gram_groups(side)[1:3] for c in ctxs)
    assert owned[0][0] == 0 and owned[-1][1] == slabs.shape[0]
    assert all(a[1] == b[0] for a, b in zip(owned, owned[1:]))  # the ranks tile the groups
    for c in ctxs:
        c.set_gram_groups(side, slabs)
    return ctxs[0].get_gramian(side)


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


@pytest.mark.parametrize("world,dim", [(w, d) for w in (2, 3, 8) for d in (8, 32, 64, 256, 512)]
                         + [(2, 1000), (3, 1000)])
def test_sharded_ials_matches_single(ml1m_csr, world, dim):
    # dim 1000 (Dp = 1024): the history-space wide bucket (256 < h_eff <= 512)
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
    np.testing.assert_array_equal(Uw, U1)
    np.testing.assert_array_equal(Vw, V1)


@pytest.mark.parametrize("dim", [8, 64, 256, 512])
def test_gramian_partition_independent(ml1m_csr, dim):
    """G (plain and omega-weighted) is bitwise the same for world 1, 2, 3, 8,
    and on every rank."""
    nu, ni, up, uc, ip, ic = ml1m_csr
    omega = np.random.default_rng(3).uniform(0.05, 1.0, nu).astype(np.float32)
    cases = ((fh.SIDE_USER, None), (fh.SIDE_ITEM, None), (fh.SIDE_USER, omega))
    ref = None
    for world in (1, 2, 3, 8):
        ctxs = _contexts(world, dim, nu, ni, up, uc, ip, ic)
        Gs = []
        for side, wts in cases:
            _allreduce_gram(ctxs, side, wts)
            Gs.append([c.get_gramian(side) for c in ctxs])
        _close(ctxs)
        for G in Gs:
            for g in G[1:]:
                np.testing.assert_array_equal(g, G[0])
        if ref is None:
            ref = [G[0] for G in Gs]
        else:
            for G, R in zip(Gs, ref):
                np.testing.assert_array_equal(G[0], R)
