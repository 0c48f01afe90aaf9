"""iALS with l2_reg_exp = 0 at the wide dims on a WELL-CONDITIONED fixture.

With l2_reg_exp = 0 every entity shares lambda = reg (ials.h:310-315), so
the history-space path takes the Cholesky basis (one M = w G + reg I, L^-T
explicit) and FRECSYS_CHOL_BASIS=0 falls back to the tridiagonal
one.  The quirk fixture (300-400 entities) leaves G rank-deficient at d = 512
/ 1024, where cond(M) is set by reg alone and two fp32 solves differ by
cond x eps whatever their order (test_dual_gpu.py::
test_chol_basis_conditioning holds that case to the float64 solution).  Here
the other side is ML-1M's 3,706 items / 6,040 users (tests/golden/ml-1m, the
reference's fixture): G is full rank and the 1e-4 oracle row bar applies to
both bases, on both sides, at d = 512 and 1024, through both the history-
space rows (h <= 256) and the wide d-space rows.  The worst rows are also
compared with the float64 solution (numpy_ref.ials) to attribute what is
left: the margins go to parity_report.jsonl.
"""
import os

import numpy as np
import pytest

import numpy_ref as R
import oracle as O
from conftest import rel_rows
from test_dual_gpu import _spread_embeddings
from test_models_gpu import ml1m_csr, report  # noqa: F401  (fixture)
from test_parity_gpu import _ctx

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")

TOL_ROW = 1e-4
REG, W = 0.003, 0.1  # the ML-1M iALS flags of test_models_gpu.py CASES


@pytest.mark.parametrize("side", ["user", "item"])
@pytest.mark.parametrize("dim", [512, 1024])
def test_reg_exp0_well_conditioned_half_step(monkeypatch, ml1m_csr, dim, side):  # noqa: F811
    nu, ni, up, uc, ip, ic = ml1m_csr
    if side == "user":
        s, o, ptr, col, n_o, tag = fh.SIDE_USER, fh.SIDE_ITEM, up, uc, ni, "solve_user"
    else:
        s, o, ptr, col, n_o, tag = fh.SIDE_ITEM, fh.SIDE_USER, ip, ic, nu, "solve_item"
    X0 = _spread_embeddings(n_o, dim, 31 + dim)
    monkeypatch.setenv("FRECSYS_DUAL", "1")
    bases = ("chol", "tridiag")
    outs = {}
    for basis in bases:
        monkeypatch.setenv("FRECSYS_CHOL_BASIS", "1" if basis == "chol" else "0")
        ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
        ctx.set_embeddings(o, X0)
        ctx.gramian(o)
        ctx.timing_reset()
        ctx.solve_side(s, fh.KIND_IALS, REG, W, reg_exp=0.0)
        assert ctx.timing(tag + ".hspace")[1] == 1 and ctx.timing(tag + ".dspace")[1] >= 1
        assert ctx.work("basis_chol")[2] == (basis == "chol")
        assert ctx.counter("hspace_reruns") == 0
        outs[basis] = ctx.get_embeddings(s)
        # users 320 / items 256 at Dp = 512, 512 at Dp = 1024 (the wide bucket)
        max_h = ctx.history_space_max_h(s)
        X = U if side == "user" else V
        ctx.close()
    G0 = O.gramian(X0)
    Xo, rc = O.step(ptr, col, X0, G0, 0, REG, W, reg_exp=0.0, out=X.copy())
    assert rc == 0
    h = np.diff(ptr)
    short, long_ = (h > 0) & (h <= max_h), h > max_h
    errs = {b: rel_rows(x, Xo) for b, x in outs.items()}
    # float64 solutions of the worst rows of either basis and of the oracle's
    # own error there (lambda = reg for every row)
    rows = np.unique(np.concatenate([np.argsort(e)[-16:] for e in errs.values()]))
    rows = rows[h[rows] > 0]
    X64 = np.array([R.ials(col[ptr[r]:ptr[r + 1]], X0, G0, REG, W) for r in rows])
    rec = dict(test="reg_exp0_well_conditioned", side=side, dim=dim, n_other=int(n_o),
               f64_oracle=float(rel_rows(Xo[rows], X64).max()),
               env={k: v for k, v in os.environ.items() if k.startswith("FRECSYS_")})
    for b, e in errs.items():
        rec[f"{b}_hspace_max"] = float(e[short].max())
        rec[f"{b}_dspace_max"] = float(e[long_].max())
        rec[f"{b}_f64"] = float(rel_rows(outs[b][rows], X64).max())
    rec["margin"] = TOL_ROW / max(max(e.max() for e in errs.values()), 1e-30)
    report(**rec)
    print(rec)
    for b, e in errs.items():
        assert e.max() < TOL_ROW, (b, e[short].max(), e[long_].max())
    # the wide d-space rows do not depend on the basis
    np.testing.assert_array_equal(outs["chol"][long_], outs["tridiag"][long_])
