"""The RCCL exchange code of the sharded path, executed on one GPU: a
world-1 communicator (frecsys_comm_init with a unique id) makes every
collective of a half-step run -- the grouped ncclBroadcast all-gather of the
Gramian's group slabs, the all-gather of factor rows and of the user losses,
and the ncclMin agreement on a failed pivot (include/frecsys_hip.h,
capi.hip).  Results must be bit-identical to the communicator-free context.
"""
import numpy as np
import pytest

from test_parity_gpu import _ctx, _v_inputs, _weights

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")


def _epoch(ctx, nu, ni, up, ip, ic):
    reg, w = 0.004, 0.004
    om = _weights(nu)
    ctx.gramian(fh.SIDE_ITEM)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, 0.003, 0.1)
    ctx.gramian(fh.SIDE_USER)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, 0.003, 0.1)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_WEIGHTED_U, reg, w, entity_weight=om)
    nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
    ctx.gramian(fh.SIDE_USER, weights=om)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, reg, w, alpha=0.3, entity_reg=item_reg,
                   other_weight=nu_w)
    ctx.gramian(fh.SIDE_ITEM)
    loss = ctx.user_loss(fh.SIDE_USER, w, True)
    return (ctx.get_embeddings(fh.SIDE_USER), ctx.get_embeddings(fh.SIDE_ITEM), loss,
            ctx.gramian(fh.SIDE_ITEM))


@pytest.mark.parametrize("dim", [32, 256, 512])
def test_world1_rccl_matches_no_comm(quirk_data, dim):
    nu, ni, up, uc, ip, ic = quirk_data
    ref_ctx, _, _ = _ctx(dim, nu, ni, up, uc, ip, ic)
    ref = _epoch(ref_ctx, nu, ni, up, ip, ic)
    ref_ctx.close()
    ctx, _, _ = _ctx(dim, nu, ni, up, uc, ip, ic)
    ctx.comm_init(1, 0, fh.unique_id())
    got = _epoch(ctx, nu, ni, up, ip, ic)
    # every collective site ran through RCCL: the four Gramians formed, and
    # not the closing plain Gramian of the item side, which repeats the one
    # before the loss on unchanged rows -- reused, no exchange (every rank
    # makes the same reuse decision, so the collectives stay matched)
    assert ctx.comm_world() == (1, 0, 1)
    assert ctx.timing("gram_exchange")[1] == 4
    assert ctx.timing("allgather")[1] >= 4
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
    # NOT_SPD through the ncclMin agreement
    with pytest.raises(fh.FrecsysError) as ei:
        ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, -50.0, 0.1)
    assert ei.value.code == fh.ERR_NOT_SPD
    ref_ctx, _, _ = _ctx(dim, nu, ni, up, uc, ip, ic)
    ref_ctx.set_embeddings(fh.SIDE_ITEM, got[1])
    ref_ctx.gramian(fh.SIDE_ITEM)
    with pytest.raises(fh.FrecsysError) as e2:
        ref_ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, -50.0, 0.1)
    assert e2.value.entity == ei.value.entity
    ctx.close()
    ref_ctx.close()
