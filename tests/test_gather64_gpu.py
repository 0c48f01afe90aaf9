"""The 64-bit gather-offset variants of the d-space kernels are bit-identical
to the 32-bit ones.

The split-bf16 SYRK gathers (solve_tiled_kernel, wide_syrk2_kernel) address
the other side's rows with 32-bit element offsets while n_other * Dp < 2^32
and dispatch 64-bit variants above that (kernels.h gather_off64: Dp = 256
beyond 16.7M rows, Dp = 1024 beyond 4.19M).  A table of that size takes
17 GB of host and device memory to build, so the dispatch is forced here with
FRECSYS_GATHER64=1 (read at every launch) and both widths must give the same
bits: every kind, the long-history split slabs included.
"""
import numpy as np
import pytest

import frecsys_hip as fh

pytestmark = pytest.mark.gpu


def _run(monkeypatch, quirk_data, dim, off64):
    nu, ni, up, uc, ip, ic = quirk_data
    monkeypatch.setenv("FRECSYS_GATHER64", "1" if off64 else "0")
    monkeypatch.setenv("FRECSYS_DUAL", "0")        # every entity on the d-space kernels
    monkeypatch.setenv("FRECSYS_SPLIT_ROWS", "64")  # long histories through the split slabs
    ctx = fh.Context(dim, nu, ni, device=0)
    ctx.load_csr(fh.SIDE_USER, up, uc)
    ctx.load_csr(fh.SIDE_ITEM, ip, ic)
    ctx.init_embeddings(1, 0.1)
    rng = np.random.default_rng(2)
    omega = rng.uniform(0.1, 1.0, nu).astype(np.float32)
    hu = np.diff(up).astype(np.float32)
    nu_w = np.where(hu > 0, omega / np.maximum(hu, 1), 0).astype(np.float32)
    item_reg = rng.uniform(0.5, 2.0, ni).astype(np.float32)
    out = []
    ctx.gramian(fh.SIDE_ITEM, fetch=False)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, 0.003, 0.1)
    out.append(ctx.get_embeddings(fh.SIDE_USER))
    ctx.solve_side(fh.SIDE_USER, fh.KIND_WEIGHTED_U, 0.003, 0.1, entity_weight=omega)
    out.append(ctx.get_embeddings(fh.SIDE_USER))
    ctx.gramian(fh.SIDE_USER, weights=omega, fetch=False)
    out.append(ctx.get_gramian(fh.SIDE_USER))
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, 0.003, 0.1, alpha=0.3,
                   entity_reg=item_reg, other_weight=nu_w)
    out.append(ctx.get_embeddings(fh.SIDE_ITEM))
    ctx.snapshot(fh.SIDE_USER)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_CVAR_GRAD_V, 0.003, 0.1, alpha=0.3, stepsize=0.01,
                   entity_reg=item_reg, other_weight=nu_w, from_snapshot=True)
    out.append(ctx.get_embeddings(fh.SIDE_ITEM))
    ctx.close()
    return out


@pytest.mark.parametrize("dim", [64, 256, 512, 1000])
def test_gather_offsets_64_bit_identical(monkeypatch, quirk_data, dim):
    a = _run(monkeypatch, quirk_data, dim, False)
    b = _run(monkeypatch, quirk_data, dim, True)
    for x, y in zip(a, b):
        assert np.all(np.isfinite(x))
        np.testing.assert_array_equal(x, y)
