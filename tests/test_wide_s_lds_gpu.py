"""S = I + Z D^-1 Z^T of the history-space wide bucket (Dp = 1024) from
LDS-DMA stages (dual.hip dual_wide_s_lds_kernel<0 / 1>, the default) against
the per-wave-fragment kernel it replaces (FRECSYS_WIDE_S_LDS=0): the tiles
holding rows see the same products in the same order, so the solved rows
must be BITWISE equal -- iALS on both sides, ProjectU (omega) and ProjectV
(nu, item_reg, with and without the tail quirk), on the mid-length data of
test_dual_wide_gpu.py (640 users / 1,200 items in the wide bucket)."""
import numpy as np
import pytest

from test_dual_wide_gpu import _run, mid_data  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")


@pytest.mark.parametrize("dim", [1000, 1024])
@pytest.mark.parametrize("case", ["ials_user", "ials_item", "u", "v_quirk", "v"])
def test_wide_s_lds_bitwise(monkeypatch, mid_data, dim, case):  # noqa: F811
    side, kind, quirk = {
        "ials_user": (fh.SIDE_USER, fh.KIND_IALS, True),
        "ials_item": (fh.SIDE_ITEM, fh.KIND_IALS, True),
        "u": (fh.SIDE_USER, fh.KIND_WEIGHTED_U, True),
        "v_quirk": (fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, True),
        "v": (fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, False),
    }[case]
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("FRECSYS_WIDE_S_LDS", flag)
        X, _, n_hs = _run(monkeypatch, mid_data, dim, side, kind, True, quirk)
        assert n_hs > 0
        outs.append(X)
    np.testing.assert_array_equal(outs[1], outs[0])
