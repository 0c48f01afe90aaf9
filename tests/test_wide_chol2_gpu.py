"""The two-panel wide Cholesky at Dp = 1024 (wide.hip wide_chol2_kernel, the
default) against the one-panel kernel it replaces (FRECSYS_WIDE_CHOL2=0):
every panel tile sees the same split-bf16 products in the same order, the
same f32 finishes and the same forward-substitution chains, so the solved
rows must be BITWISE equal.  Every entity goes through the d-space wide
path (FRECSYS_DUAL=0) on the mid-length data of test_dual_wide_gpu.py
(users with 1..600 rows, items with ~250..500): iALS on both sides, ProjectU
(omega) and ProjectV (nu, item_reg, with and without the tail quirk), at
d = 1000 and 1024 -- the reference's Project / ProjectU / ProjectV LLT
(ials.h:140-142, safer2.h:217-219) at config 5's width."""
import numpy as np
import pytest

from test_dual_wide_gpu import _run, mid_data  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")


@pytest.mark.parametrize("dim", [1000, 1024])
@pytest.mark.parametrize("case", ["ials_user", "ials_item", "u", "v_quirk", "v"])
def test_wide_chol2_bitwise(monkeypatch, mid_data, dim, case):  # noqa: F811
    side, kind, quirk = {
        "ials_user": (fh.SIDE_USER, fh.KIND_IALS, True),
        "ials_item": (fh.SIDE_ITEM, fh.KIND_IALS, True),
        "u": (fh.SIDE_USER, fh.KIND_WEIGHTED_U, True),
        "v_quirk": (fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, True),
        "v": (fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, False),
    }[case]
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("FRECSYS_WIDE_CHOL2", flag)
        X, _, _ = _run(monkeypatch, mid_data, dim, side, kind, False, quirk)
        assert np.isfinite(X).all()
        outs.append(X)
    np.testing.assert_array_equal(outs[1], outs[0])
