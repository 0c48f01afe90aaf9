"""world_size-2 rehearsal of the sharded half-step's host protocol on CPU
(gloo; no GPU here -- tests/test_sharded_gloo_gpu.py runs the same exchange
between processes driving the real HIP kernels on the GPU box).

The product's N>1 path (capi.hip) is: the rank's groups of the partition-
independent Gramian plan (frecsys_gram_plan, called here through the real
C-ABI: fixed leaves of rows, fixed groups of leaves, each rank a contiguous
run of groups) -> all-gather of the group slabs -> every rank sums the slabs
in group order; solve the rank's nnz-balanced row range (frecsys_partition,
real C-ABI) -> all-gather of the updated rows.  Each gloo rank computes its
leaves and solves its rows with the CPU oracle (the arithmetic stand-in for
the kernels), the collectives go through torch.distributed, and the result
must equal the single-process one BIT FOR BIT: the solves are per-entity
independent and the Gramian's additions do not depend on the rank count.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import frecsys_hip as fh
from conftest import make_quirk_data


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def group_slabs(X, d, world, rank):
    """This rank's group slabs of the plan (zeros elsewhere): each leaf's
    partial Gramian, summed in leaf order within the group (float32)."""
    rpl, nleaf, ng, lo, hi = fh.gram_plan(d, X.shape[0], world, rank)
    slabs = np.zeros((ng, d, d), np.float32)
    for g in range(lo, hi):
        for leaf in range(g * nleaf // ng, (g + 1) * nleaf // ng):
            slabs[g] += O_gramian(X[leaf * rpl:(leaf + 1) * rpl])
    return slabs


def O_gramian(X):
    import oracle as O
    return O.gramian(X, nthreads=1).astype(np.float32)


def finish_gramian(slabs):
    G = np.zeros(slabs.shape[1:], np.float32)
    for s in slabs:  # group order
        G += s
    return G


def _worker(rank, world, port, q):
    import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nu, ni, up, uc, ip, ic = make_quirk_data(seed=13, n_users=300, n_items=200)
    d = 12
    U, V = O.init_embeddings(7, 0.1, d, nu, ni)
    # item Gramian: this rank's groups, the slabs all-gathered (a sum over
    # zero-filled arrays: one non-zero contributor per element, exact)
    sl = torch.from_numpy(group_slabs(V, d, world, rank))
    dist.all_reduce(sl)
    G = finish_gramian(sl.numpy())
    # user half-step on this rank's nnz-balanced range
    bu = fh.partition(up, world)
    lo, hi = int(bu[rank]), int(bu[rank + 1])
    sub_ptr = up[lo:hi + 1] - up[lo]
    sub_col = uc[up[lo]:up[hi]]
    Us, rc = O.step(sub_ptr, sub_col, V, G, 0, 0.003, 0.1, out=U[lo:hi].copy(), nthreads=1)
    assert rc == 0
    # all-gather with uneven counts: pad to the max range, gather, trim
    mx = int(np.max(np.diff(bu)))
    buf = torch.zeros((mx, d), dtype=torch.float32)
    buf[: hi - lo] = torch.from_numpy(Us)
    parts = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    Ug = np.concatenate([parts[r][: int(bu[r + 1] - bu[r])].numpy() for r in range(world)])
    if rank == 0:
        q.put((Ug, G))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_user_halfstep_matches_single(world):
    import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    Ug, G = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    nu, ni, up, uc, ip, ic = make_quirk_data(seed=13, n_users=300, n_items=200)
    U, V = O.init_embeddings(7, 0.1, 12, nu, ni)
    G1 = finish_gramian(group_slabs(V, 12, 1, 0))  # the single-process plan
    np.testing.assert_array_equal(G, G1)
    np.testing.assert_allclose(G, O.gramian(V, nthreads=1), rtol=1e-5, atol=1e-6)
    Ur, _ = O.step(up, uc, V, G1, 0, 0.003, 0.1, out=U.copy(), nthreads=1)
    np.testing.assert_array_equal(Ug, Ur)


def test_gram_plan_tiles_groups():
    """Host-only plan: the ranks' groups tile [0, n_groups) for any world."""
    for d, n in ((12, 200), (256, 116_677), (512, 471_355), (1024, 2_000_000), (64, 5)):
        rpl, nleaf, ng, _, _ = fh.gram_plan(d, n)
        assert (nleaf - 1) * rpl < n <= nleaf * rpl and 1 <= ng <= 16
        for world in (1, 2, 3, 8, 16, 24):
            own = [fh.gram_plan(d, n, world, r)[3:] for r in range(world)]
            assert own[0][0] == 0 and own[-1][1] == ng
            assert all(a[1] == b[0] and a[0] <= a[1] for a, b in zip(own, own[1:]))
