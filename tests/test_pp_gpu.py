"""iALS++ block coordinate descent on the GPU (csrc/pp.hip; reference
ialspp.h: Step :351-424, ProjectBlock :85-145, PredictDataset :480-520)
against the oracle restatement, one full epoch of user/item block steps from
identical inputs (1e-4 relative per row, like every other solve), the
fold-in from zero embeddings, and the reference's own quality gate
(ialspp_test.cc: d=8, block 4, 10 epochs, NDCG@20 >= 0.2) through run_model.
"""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle as O
from conftest import ML1M, PKG, rel_rows
from test_parity_gpu import _ctx

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")

TOL_ROW = 1e-4


def _rix(uc):
    """Rating index of the user CSR (tuple order) and the item CSR entries."""
    return (np.arange(len(uc), dtype=np.int32),
            np.argsort(np.asarray(uc), kind="stable").astype(np.int32))


@pytest.mark.parametrize("dim,bs", [(8, 4), (32, 32), (64, 24), (100, 64), (256, 128)])
def test_pp_epoch_matches_oracle(quirk_data, dim, bs):
    nu, ni, up, uc, ip, ic = quirk_data
    reg, w = 0.003, 0.1
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    urix, irix = _rix(uc)
    ctx.pp_set_rating_index(fh.SIDE_USER, urix)
    ctx.pp_set_rating_index(fh.SIDE_ITEM, irix)
    ctx.pp_predict(fh.SIDE_USER)
    pred = np.zeros(len(uc), np.float32)
    O.pp_predict(up, uc, urix, V, U, pred)
    Uo, Vo = U.copy(), V.copy()
    for start in range(0, dim, bs):
        end = min(start + bs, dim)
        ctx.gramian(fh.SIDE_ITEM)
        ru = ctx.pp_step(fh.SIDE_USER, start, end, reg, w)
        rc, ro = O.pp_step(up, uc, urix, Vo, Uo, pred, start, end, reg, w)
        assert rc == 0 and abs(ru - ro) <= 1e-3 * ro + 1e-12
        ctx.gramian(fh.SIDE_USER)
        ctx.pp_step(fh.SIDE_ITEM, start, end, reg, w)
        rc, _ = O.pp_step(ip, ic, irix, Uo, Vo, pred, start, end, reg, w)
        assert rc == 0
    Ug, Vg = ctx.get_embeddings(fh.SIDE_USER), ctx.get_embeddings(fh.SIDE_ITEM)
    assert rel_rows(Ug, Uo).max() < TOL_ROW
    assert rel_rows(Vg, Vo).max() < TOL_ROW
    np.testing.assert_array_equal(Ug[5], U[5])  # idle user untouched
    np.testing.assert_array_equal(Vg[9], V[9])


@pytest.mark.parametrize("dim,bs", [(32, 8), (64, 64)])
def test_pp_fold_in_from_zero(ml1m, dim, bs):
    tr, vt, ve = ml1m
    nu, ni = tr.max_user + 1, tr.max_item + 1
    up, uc = tr.by_user()
    ip, ic = tr.by_item()
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    ids, ep, ec = vt.compact_users()
    ctx.load_csr(fh.SIDE_EVAL, ep, ec)
    ctx.set_embeddings(fh.SIDE_EVAL, np.zeros((len(ep) - 1, dim), np.float32))
    Ue = np.zeros((len(ep) - 1, dim), np.float32)
    pred = np.zeros(len(ec), np.float32)
    rix = np.arange(len(ec), dtype=np.int32)
    ctx.gramian(fh.SIDE_ITEM)
    for _ in range(2):
        ctx.pp_predict(fh.SIDE_EVAL)
        O.pp_predict(ep, ec, rix, V, Ue, pred)
        for start in range(0, dim, bs):
            end = min(start + bs, dim)
            ctx.pp_step(fh.SIDE_EVAL, start, end, 0.003, 0.1)
            rc, _ = O.pp_step(ep, ec, rix, V, Ue, pred, start, end, 0.003, 0.1)
            assert rc == 0
    assert rel_rows(ctx.get_embeddings(fh.SIDE_EVAL), Ue).max() < TOL_ROW


def test_pp_rejects_bad_block(quirk_data):
    nu, ni, up, uc, ip, ic = quirk_data
    ctx, U, V = _ctx(256, nu, ni, up, uc, ip, ic)
    urix, irix = _rix(uc)
    ctx.pp_set_rating_index(fh.SIDE_USER, urix)
    ctx.pp_predict(fh.SIDE_USER)
    for s, e in ((0, 0), (0, 129), (250, 257)):
        with pytest.raises(fh.FrecsysError) as ei:
            ctx.pp_step(fh.SIDE_USER, s, e, 0.003, 0.1)
        assert ei.value.code == fh.ERR_INVALID


def test_gate_ialspp_run_model():  # ialspp_test.cc:14-80
    cmd = [os.path.join(PKG, "bin", "run_model"), "--train_data", os.path.join(ML1M, "train.csv"),
           "--test_train_data", os.path.join(ML1M, "validation_tr.csv"),
           "--test_test_data", os.path.join(ML1M, "validation_te.csv"), "--seed", "1",
           "--model_name", "ialspp", "--dim", "8", "--block_size", "4", "--uobs_weight", "0.1",
           "--l2_reg", "0.003", "--epoch", "10", "--print_train_stats", "1",
           "--print_residual_stats", "1", "--print_var_stats", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    tail = r.stderr[r.stderr.rindex("Validation Results"):]
    m = re.search(r"Mean NDCG@20=([0-9.]+)", tail)
    assert m and float(m.group(1)) >= 0.2, tail[-2000:]
    assert len(re.findall(r"U residual: [0-9.e+-]+, V residual", r.stderr)) == 10


@pytest.mark.parametrize("dim,bs", [(8, 4), (64, 32), (128, 128)])
def test_safer2pp_blocks_match_oracle(quirk_data, dim, bs):
    """SAFER2++ StepU / StepV (safer2pp.h:449-653): weighted block steps."""
    from test_parity_gpu import _v_inputs, _weights
    nu, ni, up, uc, ip, ic = quirk_data
    reg, w, alpha = 0.004, 0.004, 0.3
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    om = _weights(nu)
    nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
    urix, irix = _rix(uc)
    ctx.pp_set_rating_index(fh.SIDE_USER, urix)
    ctx.pp_set_rating_index(fh.SIDE_ITEM, irix)
    ctx.pp_predict(fh.SIDE_USER)
    pred = np.zeros(len(uc), np.float32)
    O.pp_predict(up, uc, urix, V, U, pred)
    Uo, Vo = U.copy(), V.copy()
    for start in range(0, dim, bs):
        end = min(start + bs, dim)
        ctx.gramian(fh.SIDE_ITEM)
        ctx.pp_step(fh.SIDE_USER, start, end, reg, w, kind=fh.KIND_WEIGHTED_U, entity_weight=om)
        rc, _ = O.pp_step(up, uc, urix, Vo, Uo, pred, start, end, reg, w, kind=1,
                          entity_weight=om)
        assert rc == 0
        ctx.gramian(fh.SIDE_USER, weights=om)
        ctx.pp_step(fh.SIDE_ITEM, start, end, reg, w, kind=fh.KIND_WEIGHTED_V, alpha=alpha,
                    entity_reg=item_reg, other_weight=nu_w)
        rc, _ = O.pp_step(ip, ic, irix, Uo, Vo, pred, start, end, reg, w, kind=2, alpha=alpha,
                          entity_reg=item_reg, other_weight=nu_w, gram_w=om)
        assert rc == 0
    assert rel_rows(ctx.get_embeddings(fh.SIDE_USER), Uo).max() < TOL_ROW
    assert rel_rows(ctx.get_embeddings(fh.SIDE_ITEM), Vo).max() < TOL_ROW


def test_gate_safer2pp_run_model():  # safer2pp_test.cc:100-145
    cmd = [os.path.join(PKG, "bin", "run_model"), "--train_data", os.path.join(ML1M, "train.csv"),
           "--test_train_data", os.path.join(ML1M, "validation_tr.csv"),
           "--test_test_data", os.path.join(ML1M, "validation_te.csv"), "--seed", "1",
           "--model_name", "safer2pp", "--dim", "8", "--block_size", "4", "--uobs_weight",
           "0.004", "--l2_reg", "0.004", "--bandwidth", "0.15", "--alpha", "0.3",
           "--xi_iterations", "5", "--pd_iterations", "1", "--epoch", "10",
           "--print_var_stats", "1", "--print_train_stats", "1", "--print_residual_stats", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    tail = r.stderr[r.stderr.rindex("Validation Results"):]
    m = re.search(r"Mean NDCG@20=([0-9.]+)", tail)
    assert m and float(m.group(1)) >= 0.2, tail[-2000:]
    means = [float(x) for x in re.findall(r"Min: [0-9.]+, Mean: ([0-9.]+), Max", r.stderr)]
    assert len(means) == 10 and all(abs(x - 0.3) <= 0.02 for x in means), means


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("dim,bs,kind", [(64, 24, fh.KIND_IALS), (256, 128, fh.KIND_IALS),
                                          (64, 32, fh.KIND_WEIGHTED_U)])
def test_pp_sharded_bitwise(quirk_data, world, dim, bs, kind):
    """Sharded iALS++ / SAFER2++ block steps: W contexts on cuda:0 joined as
    ranks in external-exchange mode each solve their own rows; the test does
    what RCCL does (Gramian group slabs, the rows), and every rank replays
    the others' prediction updates (frecsys_pp_sync).  Embeddings after a
    full epoch of user + item block steps equal the single-rank run BIT FOR
    BIT, and the residual sums over the ranks."""
    from test_parity_gpu import _v_inputs, _weights
    from test_sharded_gpu import _allgather_rows, _allreduce_gram
    nu, ni, up, uc, ip, ic = quirk_data
    reg, w, alpha = 0.003, 0.1, 0.3
    urix, irix = _rix(uc)
    om = _weights(nu)
    nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)

    def make(W, r):
        c = fh.Context(dim, nu, ni, device=0)
        if W > 1:
            c.comm_init(W, r, None)
        c.load_csr(fh.SIDE_USER, up, uc)
        c.load_csr(fh.SIDE_ITEM, ip, ic)
        c.init_embeddings(1, 0.1)
        c.pp_set_rating_index(fh.SIDE_USER, urix)
        c.pp_set_rating_index(fh.SIDE_ITEM, irix)
        c.pp_predict(fh.SIDE_USER)
        return c

    def ukw():
        return dict(kind=kind, entity_weight=om) if kind == fh.KIND_WEIGHTED_U else {}

    def vkw():
        if kind == fh.KIND_WEIGHTED_U:
            return dict(kind=fh.KIND_WEIGHTED_V, alpha=alpha, entity_reg=item_reg,
                        other_weight=nu_w)
        return {}

    gw = om if kind == fh.KIND_WEIGHTED_U else None
    ref = make(1, 0)
    ctxs = [make(world, r) for r in range(world)]
    for start in range(0, dim, bs):
        end = min(start + bs, dim)
        ref.gramian(fh.SIDE_ITEM)
        r_ref = ref.pp_step(fh.SIDE_USER, start, end, reg, w, **ukw())
        _allreduce_gram(ctxs, fh.SIDE_ITEM)
        r_sh = sum(c.pp_step(fh.SIDE_USER, start, end, reg, w, **ukw()) for c in ctxs)
        _allgather_rows(ctxs, fh.SIDE_USER)
        for c in ctxs:
            c.pp_sync(fh.SIDE_USER)
        assert abs(r_sh - r_ref) <= 1e-9 * max(r_ref, 1e-30)
        ref.gramian(fh.SIDE_USER, weights=gw)
        ref.pp_step(fh.SIDE_ITEM, start, end, reg, w, **vkw())
        _allreduce_gram(ctxs, fh.SIDE_USER, gw)
        for c in ctxs:
            c.pp_step(fh.SIDE_ITEM, start, end, reg, w, **vkw())
        _allgather_rows(ctxs, fh.SIDE_ITEM)
        for c in ctxs:
            c.pp_sync(fh.SIDE_ITEM)
    Ur, Vr = ref.get_embeddings(fh.SIDE_USER), ref.get_embeddings(fh.SIDE_ITEM)
    for c in ctxs:
        np.testing.assert_array_equal(c.get_embeddings(fh.SIDE_USER), Ur)
        np.testing.assert_array_equal(c.get_embeddings(fh.SIDE_ITEM), Vr)
    # the predictions too: the next block step of every rank reads them
    ref.gramian(fh.SIDE_ITEM)
    r_ref = ref.pp_step(fh.SIDE_USER, 0, min(bs, dim), reg, w, **ukw())
    _allreduce_gram(ctxs, fh.SIDE_ITEM)
    for c in ctxs:
        c.pp_step(fh.SIDE_USER, 0, min(bs, dim), reg, w, **ukw())
    _allgather_rows(ctxs, fh.SIDE_USER)
    np.testing.assert_array_equal(ctxs[0].get_embeddings(fh.SIDE_USER),
                                  ref.get_embeddings(fh.SIDE_USER))
    for c in ctxs + [ref]:
        c.close()


def test_pp_sync_pending_rejected(quirk_data):
    """External-exchange mode: a sharded block step leaves a snapshot for
    frecsys_pp_sync; another pp_step or pp_predict before the sync is refused
    (FRECSYS_ERR_INVALID, 'pp_sync pending'), and the sequence goes on after
    the sync."""
    from test_sharded_gpu import _allgather_rows, _allreduce_gram
    nu, ni, up, uc, ip, ic = quirk_data
    urix, irix = _rix(uc)
    ctxs = []
    for r in range(2):
        c = fh.Context(32, nu, ni, device=0)
        c.comm_init(2, r, None)
        c.load_csr(fh.SIDE_USER, up, uc)
        c.load_csr(fh.SIDE_ITEM, ip, ic)
        c.init_embeddings(1, 0.1)
        c.pp_set_rating_index(fh.SIDE_USER, urix)
        c.pp_set_rating_index(fh.SIDE_ITEM, irix)
        c.pp_predict(fh.SIDE_USER)
        ctxs.append(c)
    _allreduce_gram(ctxs, fh.SIDE_ITEM)
    for c in ctxs:
        c.pp_step(fh.SIDE_USER, 0, 16, 0.003, 0.1)
    for c in ctxs:
        with pytest.raises(fh.FrecsysError, match="pp_sync pending"):
            c.pp_step(fh.SIDE_USER, 16, 32, 0.003, 0.1)
        with pytest.raises(fh.FrecsysError, match="pp_sync pending"):
            c.pp_step(fh.SIDE_ITEM, 0, 16, 0.003, 0.1)
        with pytest.raises(fh.FrecsysError, match="pp_sync pending"):
            c.pp_predict(fh.SIDE_USER)
    _allgather_rows(ctxs, fh.SIDE_USER)
    for c in ctxs:
        c.pp_sync(fh.SIDE_USER)
        with pytest.raises(fh.FrecsysError, match="no sharded block step"):
            c.pp_sync(fh.SIDE_USER)
    for c in ctxs:
        c.pp_step(fh.SIDE_USER, 16, 32, 0.003, 0.1)
    _allgather_rows(ctxs, fh.SIDE_USER)
    for c in ctxs:
        c.pp_sync(fh.SIDE_USER)
        c.close()
