"""The rotation GEMM from LDS-DMA stages (spectral.hip rotate_lds_kernel, Dp =
256 / 512 / 1024, launches of >= 256 blocks of 256 rows x 256 columns) against the register-fed
rotation kernels it replaces there (FRECSYS_ROT_LDS=0): the forward rotation
X Q of the other side, the back rotation x' Q^T of the history-space rows
(position-blocked input, scattered output rows) and, at the wide dims, the
u^T G u partials of the user loss all run through it in one iALS epoch + user
loss.  Same products in the same order per element, so U, V and the losses
must be BITWISE equal."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")
from frecsys_hip.data import SynthShape, synthetic  # noqa: E402

SHAPE = SynthShape(70_000, 18_000, 2_000_000, min_uc=5)


@pytest.fixture(scope="module")
def data():
    return synthetic(SHAPE)


def _epoch(data, dim):
    up, uc, ip, ic = data
    ctx = fh.Context(dim, len(up) - 1, len(ip) - 1)
    try:
        ctx.load_csr(fh.SIDE_USER, up, uc)
        ctx.load_csr(fh.SIDE_ITEM, ip, ic)
        ctx.init_embeddings(1, 0.1)
        ctx.gramian(fh.SIDE_ITEM, fetch=False)
        ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, 0.003, 0.1)
        ctx.gramian(fh.SIDE_USER, fetch=False)
        ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, 0.003, 0.1)
        ctx.gramian(fh.SIDE_ITEM, fetch=False)
        loss = ctx.user_loss(fh.SIDE_USER, 0.1, True)
        nh = ctx.work("solve_user.hspace")[2]
        assert ctx.counter("hspace_reruns") == 0
        return ctx.get_embeddings(fh.SIDE_USER), ctx.get_embeddings(fh.SIDE_ITEM), loss, nh
    finally:
        ctx.close()


@pytest.mark.parametrize("dim", [256, 500, 1000])
def test_rotate_lds_bitwise(monkeypatch, data, dim):
    monkeypatch.setenv("FRECSYS_ROT_LDS", "0")
    U0, V0, l0, nh = _epoch(data, dim)
    assert nh >= 65536  # the back rotation of the user side takes the LDS kernel
    monkeypatch.setenv("FRECSYS_ROT_LDS", "1")
    U1, V1, l1, _ = _epoch(data, dim)
    np.testing.assert_array_equal(U1, U0)
    np.testing.assert_array_equal(V1, V0)
    np.testing.assert_array_equal(l1, l0)
