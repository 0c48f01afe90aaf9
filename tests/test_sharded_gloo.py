"""world_size-2 rehearsal of the sharded half-step on CPU (gloo).

The product's N>1 path (capi.hip) is: partial Gramian over the rank's own
rows -> all-reduce; solve the rank's nnz-balanced row range
(frecsys_partition, called here through the real C-ABI) -> all-gather of the
updated rows.  Here each gloo rank runs its shard with the CPU oracle as the
stand-in solver and the collectives through torch.distributed; the test
checks that the sharded half-step reproduces the single-process one
(bit-exact solves: they are per-entity independent; Gramian within fp32
summation order).
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


def _worker(rank, world, port, q):
    import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nu, ni, up, uc, ip, ic = make_quirk_data(seed=13, n_users=300, n_items=200)
    d = 12
    U, V = O.init_embeddings(7, 0.1, d, nu, ni)
    # item Gramian: partial over this rank's item rows, all-reduced
    bi = fh.partition(ip, world)
    Gp = torch.from_numpy(O.gramian(V[bi[rank]:bi[rank + 1]], nthreads=1).astype(np.float64))
    dist.all_reduce(Gp)
    G = Gp.numpy().astype(np.float32)
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
    Gs = O.gramian(V, nthreads=1)
    np.testing.assert_allclose(G, Gs, rtol=1e-5, atol=1e-6)
    Ur, _ = O.step(up, uc, V, G, 0, 0.003, 0.1, out=U.copy(), nthreads=1)
    np.testing.assert_array_equal(Ug, Ur)
