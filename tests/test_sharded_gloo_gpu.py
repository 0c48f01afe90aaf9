"""The product's sharded path in separate processes on one GPU, exchanging
over torch.distributed (gloo): world 2 and 3.

RCCL cannot put two ranks on one device, so each process joins rank r of W
in external-exchange mode (frecsys_comm_init with no id) and gloo carries
what RCCL carries on an 8-GPU node: the Gramian's group slabs (each rank's
own groups; summing the zero-filled slab arrays over ranks reproduces every
slab exactly, x + 0 = x), then frecsys_set_gram_groups sums them in group
order; the factor rows of every rank's nnz-balanced range; the user losses.
Two iALS epochs and a SAFER2 half-step pair per rank, all through the real
C-ABI and HIP kernels; rank 0 must reproduce the single-process run bit for
bit (solves are per-entity independent, the Gramian partition-independent).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    from conftest import ML1M
    from frecsys_hip.data import Dataset
    tr = Dataset.from_csv(os.path.join(ML1M, "train.csv"))
    up, uc = tr.by_user()
    ip, ic = tr.by_item()
    return tr.max_user + 1, tr.max_item + 1, up, uc, ip, ic


def _run(world, rank, dim, exchange):
    """Two iALS epochs, then ProjectU / weighted Gramian / ProjectV / loss."""
    nu, ni, up, uc, ip, ic = _data()
    ctx = fh.Context(dim, nu, ni, device=0)
    if world > 1:
        ctx.comm_init(world, rank, None)
    ctx.load_csr(fh.SIDE_USER, up, uc)
    ctx.load_csr(fh.SIDE_ITEM, ip, ic)
    ctx.init_embeddings(1, 0.1)
    gram, rows, losses = exchange(ctx)
    reg, w = 0.003, 0.1
    for _ in range(2):  # ials.h:187-206
        gram(fh.SIDE_ITEM, None)
        ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, reg, w)
        rows(fh.SIDE_USER)
        gram(fh.SIDE_USER, None)
        ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, reg, w)
        rows(fh.SIDE_ITEM)
    rng = np.random.default_rng(5)
    om = rng.uniform(0.05, 1.0, nu).astype(np.float32)
    hu = np.diff(up).astype(np.float32)
    nu_w = np.where(hu > 0, om / np.maximum(hu, 1), 0).astype(np.float32)
    item_reg = rng.uniform(0.5, 2.0, ni).astype(np.float32)
    gram(fh.SIDE_ITEM, None)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_WEIGHTED_U, 0.004, 0.004, entity_weight=om)
    rows(fh.SIDE_USER)
    gram(fh.SIDE_USER, om)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, 0.004, 0.004, alpha=0.3, entity_reg=item_reg,
                   other_weight=nu_w)
    rows(fh.SIDE_ITEM)
    gram(fh.SIDE_ITEM, None)
    loss = losses(0.004)
    out = (ctx.get_embeddings(fh.SIDE_USER), ctx.get_embeddings(fh.SIDE_ITEM),
           ctx.get_gramian(fh.SIDE_ITEM), loss)
    ctx.close()
    return out


def _local(ctx):
    def gram(side, wts):
        ctx.gramian(side, wts, fetch=False)

    return gram, (lambda side: None), (lambda beta: ctx.user_loss(fh.SIDE_USER, beta, True))


def _gloo(dist, torch):
    def make(ctx):
        world = dist.get_world_size()

        def gram(side, wts):
            ctx.gramian(side, wts, fetch=False)
            ng, lo, hi, _ = ctx.gram_groups(side)
            mine = ctx.get_gram_groups(side)
            assert not mine[:lo].any() and not mine[hi:].any()
            t = torch.from_numpy(mine)
            dist.all_reduce(t)  # every element has one non-zero contributor: exact
            ctx.set_gram_groups(side, t.numpy())

        def rows(side):
            lo, hi = ctx.shard_range(side)
            full = ctx.get_embeddings(side)
            bounds = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(bounds, torch.tensor([lo, hi]))
            mx = max(int(b[1] - b[0]) for b in bounds)
            buf = torch.zeros((mx, full.shape[1]), dtype=torch.float32)
            buf[: hi - lo] = torch.from_numpy(full[lo:hi])
            parts = [torch.zeros_like(buf) for _ in range(world)]
            dist.all_gather(parts, buf)
            for b, p in zip(bounds, parts):
                full[int(b[0]):int(b[1])] = p[: int(b[1] - b[0])].numpy()
            ctx.set_embeddings(side, full)

        def losses(beta):
            lo, hi = ctx.shard_range(fh.SIDE_USER)
            mine = ctx.user_loss(fh.SIDE_USER, beta, True)
            mask = np.zeros_like(mine)
            mask[lo:hi] = mine[lo:hi]
            t = torch.from_numpy(mask)
            dist.all_reduce(t)
            return t.numpy()

        return gram, rows, losses
    return make


def _worker(rank, world, port, dim, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(os.path.dirname(here), "safer2-recommender_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = _run(world, rank, dim, _gloo(dist, torch))
        if rank == 0:
            q.put(out)
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,dim", [(2, 64), (3, 256), (2, 512)])
def test_gloo_ranks_match_single(world, dim):
    ref = _run(1, 0, dim, _local)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, dim, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
