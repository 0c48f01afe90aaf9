"""Wide-dim workspaces bounded by the device's memory (capi.hip ws_budget,
ensure_batch).

At d = 257..1024 the d-space solve assembles A in HBM workspaces a batch of
entities at a time, long histories cut into slabs, from a pre-split copy of
the other side.  Each workspace takes at most FRECSYS_WIDE_WS_MB and a
quarter of the free device memory; a failed allocation halves the batch (or
cuts the slabs, or drops the pre-split table for the register-staged SYRK)
instead of failing the call.  None of that changes a result: entities are
independent and the split / pre-split SYRKs are bit-identical at the wide
dims.  Checked on the MSD shape (BASELINE configs[3], d = 512, 471K x 41K,
28.8M interactions, items up to 193K rows):

* a tiny budget (FRECSYS_WIDE_WS_MB=64) gives bitwise the default's U and V
  after two iALS epochs;
* a device squeezed by another tenant (a hipMalloc leaving ~1.5 GB free)
  with the free-memory cap off (FRECSYS_WS_FREE_CAP=0: every 16 GB request
  is tried and fails) completes the second epoch through the
  shrink paths (frecsys_counter "ws_shrinks" > 0), bitwise the default.
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

fh = pytest.importorskip("frecsys_hip")
from frecsys_hip.data import SHAPES, synthetic  # noqa: E402

DIM = 512
REG, W = 0.002, 0.05  # README.md:105


@pytest.fixture(scope="module")
def msd():
    return synthetic(SHAPES["msd"])


def _context(up, uc, ip, ic):
    ctx = fh.Context(DIM, len(up) - 1, len(ip) - 1)
    ctx.load_csr(fh.SIDE_USER, up, uc)
    ctx.load_csr(fh.SIDE_ITEM, ip, ic)
    ctx.init_embeddings(1, 0.1)
    return ctx


def _epoch(ctx):
    ctx.gramian(fh.SIDE_ITEM, fetch=False)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, REG, W)
    ctx.gramian(fh.SIDE_USER, fetch=False)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, REG, W)


def _two_epochs(msd, between=None):
    ctx = _context(*msd)
    try:
        _epoch(ctx)
        if between:
            between(ctx)
        _epoch(ctx)
        assert ctx.counter("hspace_reruns") == 0
        return (ctx.get_embeddings(fh.SIDE_USER), ctx.get_embeddings(fh.SIDE_ITEM),
                ctx.counter("ws_shrinks"))
    finally:
        ctx.close()


@pytest.fixture(scope="module")
def default_run(msd):
    return _two_epochs(msd)


def test_tiny_budget_bitwise(msd, default_run, monkeypatch):
    U0, V0, s0 = default_run
    assert s0 == 0
    monkeypatch.setenv("FRECSYS_WIDE_WS_MB", "64")
    U, V, _ = _two_epochs(msd)
    np.testing.assert_array_equal(U, U0)
    np.testing.assert_array_equal(V, V0)


class _Filler:
    """Device memory held by "another tenant": a plain hipMalloc through the
    HIP runtime the library already loaded (no second runtime client such as
    torch in this process)."""

    def __init__(self, keep):
        import ctypes
        self.hip = ctypes.CDLL("libamdhip64.so")
        free, total = ctypes.c_size_t(), ctypes.c_size_t()
        assert self.hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
        self.ptr = ctypes.c_void_p()
        self.size = free.value - keep
        if self.size <= 2**28:
            pytest.skip(f"only {free.value / 2**30:.1f} GB free")
        assert self.hip.hipMalloc(ctypes.byref(self.ptr), ctypes.c_size_t(self.size)) == 0

    def release(self):
        if self.ptr:
            assert self.hip.hipFree(self.ptr) == 0
            self.ptr = None


def test_squeezed_device_bitwise(msd, default_run, monkeypatch):
    U0, V0, _ = default_run
    monkeypatch.setenv("FRECSYS_WS_FREE_CAP", "0")
    fillers = []

    def squeeze(ctx):
        # every other buffer of the context exists after epoch 1; the wide
        # workspaces are freed and then have ~1.5 GB to share
        ctx.release_workspaces()
        fillers.append(_Filler(int(1.5 * 2**30)))

    try:
        U, V, shrinks = _two_epochs(msd, squeeze)
    finally:
        for f in fillers:
            f.release()
    assert shrinks > 0  # the 16 GB requests failed and were cut
    np.testing.assert_array_equal(U, U0)
    np.testing.assert_array_equal(V, V0)
