"""Sharded iALS++ / SAFER2++ block steps in separate processes on one GPU with
the in-call exchange of frecsys_pp_step.

frecsys_pp_step at world > 1 exchanges inside the call: the rows of every
rank (an all-gather), the other ranks' prediction updates replayed from them
(pp_refresh_kernel), the NOT_SPD verdict (a min over ranks) and every rank's
per-row residuals summed in the single-rank order.  RCCL and a caller-
provided transport (frecsys_set_transport) run that one code path and differ
only in the transport call (capi.hip xchg_rows / xchg_min_u64).  RCCL cannot
put two ranks on one device, so here each process joins rank r of W in
external-exchange mode and registers gloo as its transport; the Gramian's
group slabs move as in test_sharded_gloo_gpu.py.  One epoch of user + item
block steps of iALS++ (ialspp.h:351-424) and of SAFER2++ (safer2pp.h:449-653)
at world 2 and 3: the embeddings, the prediction vector of the training
tuples after the epoch and after the next block step, and every block's
residual are bitwise those of the single-process run.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")

DIM, BS = 64, 24
REG, W, ALPHA = 0.003, 0.1, 0.3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    from conftest import make_quirk_data
    from test_parity_gpu import _v_inputs, _weights
    nu, ni, up, uc, ip, ic = make_quirk_data()
    urix = np.arange(len(uc), dtype=np.int32)
    irix = np.argsort(np.asarray(uc), kind="stable").astype(np.int32)
    om = _weights(nu)
    nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
    return (nu, ni, up, uc, ip, ic), urix, irix, om, nu_w, item_reg


def _epoch(world, rank, model, gram_x, transport):
    """One epoch of block steps (+ the next user block step) on rank r of W."""
    (nu, ni, up, uc, ip, ic), urix, irix, om, nu_w, item_reg = _inputs()
    ctx = fh.Context(DIM, nu, ni, device=0)
    if world > 1:
        ctx.comm_init(world, rank, None)
        ctx.set_transport(*transport(ctx))
    ctx.load_csr(fh.SIDE_USER, up, uc)
    ctx.load_csr(fh.SIDE_ITEM, ip, ic)
    ctx.init_embeddings(1, 0.1)
    ctx.pp_set_rating_index(fh.SIDE_USER, urix)
    ctx.pp_set_rating_index(fh.SIDE_ITEM, irix)
    ctx.pp_predict(fh.SIDE_USER)
    if model == "ialspp":
        ukw, vkw, gw = {}, {}, None
    else:
        ukw = dict(kind=fh.KIND_WEIGHTED_U, entity_weight=om)
        vkw = dict(kind=fh.KIND_WEIGHTED_V, alpha=ALPHA, entity_reg=item_reg, other_weight=nu_w)
        gw = om
    resid = []
    for start in range(0, DIM, BS):
        end = min(start + BS, DIM)
        gram_x(ctx, fh.SIDE_ITEM, None)
        resid.append(ctx.pp_step(fh.SIDE_USER, start, end, REG, W, **ukw))
        gram_x(ctx, fh.SIDE_USER, gw)
        resid.append(ctx.pp_step(fh.SIDE_ITEM, start, end, REG, W, **vkw))
    pred = ctx.pp_predictions(fh.SIDE_USER, len(uc))
    out = [ctx.get_embeddings(fh.SIDE_USER), ctx.get_embeddings(fh.SIDE_ITEM), pred,
           np.array(resid, np.float64)]
    gram_x(ctx, fh.SIDE_ITEM, None)  # the next step reads the predictions
    out.append(np.array([ctx.pp_step(fh.SIDE_USER, 0, BS, REG, W, **ukw)], np.float64))
    out.append(ctx.get_embeddings(fh.SIDE_USER))
    out.append(ctx.pp_predictions(fh.SIDE_USER, len(uc)))
    ctx.close()
    return out


def _gram_local(ctx, side, wts):
    ctx.gramian(side, wts, fetch=False)


def _gloo(dist, torch):
    world = dist.get_world_size()

    def gram_x(ctx, side, wts):
        ctx.gramian(side, wts, fetch=False)
        ng, lo, hi, _ = ctx.gram_groups(side)
        mine = ctx.get_gram_groups(side)
        t = torch.from_numpy(mine)
        dist.all_reduce(t)  # each slab has one non-zero contributor: exact
        ctx.set_gram_groups(side, t.numpy())

    def transport(ctx):
        calls = {"rows": 0, "min": 0}

        def rows(side, arr, lo, hi):
            calls["rows"] += 1
            bounds = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(bounds, torch.tensor([lo, hi]))
            mx = max(int(b[1] - b[0]) for b in bounds)
            buf = torch.zeros((max(mx, 1), arr.shape[1]), dtype=torch.float32)
            buf[: hi - lo] = torch.from_numpy(arr[lo:hi].copy())
            parts = [torch.zeros_like(buf) for _ in range(world)]
            dist.all_gather(parts, buf)
            for b, p in zip(bounds, parts):
                arr[int(b[0]):int(b[1])] = p[: int(b[1] - b[0])].numpy()

        def vmin(v):
            calls["min"] += 1
            got = [None] * world
            dist.all_gather_object(got, v)
            return min(got)

        return rows, vmin

    return gram_x, transport


def _worker(rank, world, port, model, q):
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
        gram_x, transport = _gloo(dist, torch)
        out = _epoch(world, rank, model, gram_x, transport)
        q.put((rank, out))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model", ["ialspp", "safer2pp"])
@pytest.mark.parametrize("world", [2, 3])
def test_pp_transport_ranks_match_single(world, model):
    ref = _epoch(1, 0, model, _gram_local, None)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, model, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    names = ("U", "V", "predictions", "residuals", "next residual", "next U", "next predictions")
    for r in range(world):  # every rank holds the single-rank state, bit for bit
        for name, a, b in zip(names, got[r], ref):
            np.testing.assert_array_equal(a, b, err_msg=f"rank {r}: {name}")
