"""Train-loss diagnostics on the GPU (frecsys_train_stats; the parts of
ComputeLosses / PrintLosses, ials.h:226-305, safer2.h:337-413,
erm_mf.h:303-377, cvar_mf.h:332-406) against float64 numpy, and the
run_model log lines they feed (--print_train_stats 1, the CLI default)."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, ML1M, make_quirk_data
from test_parity_gpu import _ctx

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")


@pytest.mark.parametrize("dim", [8, 16, 64, 256, 512])
def test_train_stats_match_numpy(dim):
    nu, ni, up, uc, ip, ic = make_quirk_data(n_users=300, n_items=200)
    ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
    obs, unobs, un, vn = ctx.train_stats()
    U64, V64 = U.astype(np.float64), V.astype(np.float64)
    rows = np.repeat(np.arange(nu), np.diff(up))
    pred = np.einsum("ij,ij->i", U64[rows], V64[uc])
    ref_obs = np.sum((pred - 1.0) ** 2)
    ref_unobs = np.sum((U64.T @ U64) * (V64.T @ V64))
    assert abs(obs - ref_obs) <= 1e-5 * ref_obs
    assert abs(unobs - ref_unobs) <= 1e-5 * abs(ref_unobs) + 1e-9
    np.testing.assert_allclose(un, np.sum(U64 ** 2, axis=1), rtol=1e-5)
    np.testing.assert_allclose(vn, np.sum(V64 ** 2, axis=1), rtol=1e-5)


@pytest.mark.parametrize("model,extra", [
    ("ials", ["--uobs_weight", "0.1", "--l2_reg", "0.003"]),
    ("ERM_MF", ["--uobs_weight", "0.004", "--l2_reg", "0.005"]),
    ("cvar_mf", ["--uobs_weight", "0.008", "--l2_reg", "0.002", "--stepsize", "0.4"]),
    ("safer2", ["--uobs_weight", "0.004", "--l2_reg", "0.004", "--bandwidth", "0.15"]),
])
def test_run_model_prints_train_losses(model, extra):
    cmd = [os.path.join(PKG, "bin", "run_model"), "--train_data", os.path.join(ML1M, "train.csv"),
           "--test_train_data", os.path.join(ML1M, "validation_tr.csv"),
           "--test_test_data", os.path.join(ML1M, "validation_te.csv"), "--seed", "1",
           "--model_name", model, "--dim", "16", "--epoch", "2", "--print_train_stats", "1"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = re.findall(r"Loss=([-0-9.e+]+) Loss_observed=([-0-9.e+]+) Loss_unobserved=([-0-9.e+]+)",
                       r.stderr)
    assert len(lines) >= 2, r.stderr[-2000:]
    for t in lines:
        assert all(np.isfinite(float(x)) for x in t)
    assert "(train-loss diagnostics" not in r.stderr
