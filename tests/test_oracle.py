"""Pin the CPU oracle (oracle/frecsys_oracle.c) before trusting it:

1. against the reference's own known-answer tests on its own fixture
   (tests/ml-1m, copied to tests/golden/ml-1m): NDCG@20 >= 0.2 after the
   reference's epochs/hyper-parameters (ials_test.cc:17-45,
   erm_mf_test.cc:17-45, cvar_mf_test.cc:17-46, safer2_test.cc:17-99) and the
   SAFER2 mean dual weight within alpha +- 0.02 after every epoch
   (safer2_test.cc:135, 183, 230), the SNR variant (safer2_test.cc:37-58,
   sub-sampled Newton on the seeded sample stream) included;
2. against an independent float64 numpy restatement (tests/numpy_ref.py);
3. against libstdc++'s own std::mt19937 / std::normal_distribution<float>
   (a tiny C++ program compiled with g++ at test time).
Element-wise agreement with the reference binary itself is unpinned: the
reference needs Eigen/glog/bazel, none of which exist in this image.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import numpy_ref as R
import oracle as O
from conftest import make_quirk_data, rel_rows

K_LIST = (5, 10, 20, 50, 100)


def test_mt19937_known_answer():
    # C++ [rand.predef]: the 10000th output of a default-seeded mt19937 is 4123659995
    import ctypes
    st = (ctypes.c_uint32 * 625)()
    O.lib().oracle_mt_seed(st, 5489)
    v = None
    for _ in range(10000):
        v = O.lib().oracle_mt_next(st)
    assert v == 4123659995


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ missing")
def test_init_matches_libstdcxx(tmp_path):
    src = tmp_path / "gen.cc"
    src.write_text(r'''
#include <cmath>
#include <cstdio>
#include <random>
int main() {
  int dim = 7; long nu = 5, ni = 3;
  std::mt19937 gen{4242u};
  float s = 0.1 / sqrt(dim);
  for (int m = 0; m < 2; ++m) {
    std::normal_distribution<float> d(0, s);
    long n = (m == 0 ? nu : ni) * dim;
    for (long i = 0; i < n; ++i) printf("%.9g\n", d(gen));
  }
}''')
    exe = tmp_path / "gen"
    subprocess.run(["g++", "-O2", "-o", str(exe), str(src)], check=True)
    ref = np.array([float(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                                     check=True).stdout.split()], np.float32)
    U, V = O.init_embeddings(4242, 0.1, 7, 5, 3)
    np.testing.assert_array_equal(np.concatenate([U.ravel(), V.ravel()]), ref)


@pytest.fixture(scope="module")
def small():
    nu, ni, up, uc, ip, ic = make_quirk_data(seed=11, n_users=400, n_items=300)
    return nu, ni, up, uc, ip, ic


def _rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.mark.parametrize("dim", [4, 8, 33])
def test_projections_vs_numpy(small, dim):
    nu, ni, up, uc, ip, ic = small
    U, V = O.init_embeddings(3, 0.1, dim, nu, ni)
    Gv, Gu = O.gramian(V), O.gramian(U)
    np.testing.assert_allclose(Gv, V.astype(np.float64).T @ V, rtol=1e-5, atol=1e-7)
    om = (0.1 + np.random.default_rng(1).random(nu)).astype(np.float32)
    hu = np.diff(up).astype(np.float32)
    with np.errstate(divide="ignore"):
        nuw = (om / hu).astype(np.float32)
    Ui, _ = O.step(up, uc, V, Gv, 0, 0.003, 0.1)
    Uu, _ = O.step(up, uc, V, Gv, 1, 0.004, 0.004, entity_weight=om)
    er = np.linspace(0.5, 2.0, ni).astype(np.float32)
    Vv, _ = O.step(ip, ic, U, Gu, 2, 0.004, 0.004, alpha=0.3, entity_reg=er, other_weight=nuw)
    Uc, _ = O.step(up, uc, V, Gv, 3, 0.002, 0.008, stepsize=0.4, entity_weight=om, E=U)
    Vc, _ = O.step(ip, ic, U, Gu, 4, 0.002, 0.008, alpha=0.3, stepsize=0.4, entity_reg=er,
                   other_weight=nuw, E=V)
    for u in range(nu):
        hist = uc[up[u]:up[u + 1]]
        if len(hist) == 0:
            continue
        lam_i = 0.003 * (len(hist) + 0.1 * ni)
        assert _rel(Ui[u], R.ials(hist, V, Gv, lam_i, 0.1)) < 1e-4
        lam_u = 0.004 * (1 + 0.004 * ni)
        assert _rel(Uu[u], R.project_u(hist, V, Gv, lam_u, 0.004, om[u])) < 1e-4
        lam_c = 0.002 * (1 + 0.008 * ni)
        assert _rel(Uc[u], R.cvar_u(hist, U[u], V, Gv, lam_c, 0.008, 0.4, om[u])) < 1e-4
    for v in range(ni):
        hist = ic[ip[v]:ip[v + 1]]
        if len(hist) == 0:
            continue
        lam_v = np.float32(0.004) * (er[v] + np.float32(0.3) * np.float32(0.004) * nu)
        assert _rel(Vv[v], R.project_v(hist, U, Gu, lam_v, 0.004, nuw, True)) < 1e-4
        lam_cv = np.float32(0.002) * (er[v] + np.float32(0.3) * np.float32(0.008) * nu)
        assert _rel(Vc[v], R.cvar_v(hist, V[v], U, Gu, lam_cv, 0.008, nuw, 0.4, True)) < 1e-4


def test_quirk_matters_in_numpy_and_oracle(small):
    nu, ni, up, uc, ip, ic = small
    U, V = O.init_embeddings(3, 0.1, 8, nu, ni)
    Gu = O.gramian(U)
    hu = np.diff(up).astype(np.float32)
    with np.errstate(divide="ignore"):
        nuw = (0.3 / hu).astype(np.float32)
    er = np.ones(ni, np.float32)
    a, _ = O.step(ip, ic, U, Gu, 2, 0.004, 0.004, alpha=0.3, entity_reg=er, other_weight=nuw,
                  quirk=1)
    b, _ = O.step(ip, ic, U, Gu, 2, 0.004, 0.004, alpha=0.3, entity_reg=er, other_weight=nuw,
                  quirk=0)
    h = np.diff(ip)
    aff = (h > 128) & (h % 128 != 0)
    assert aff.any()
    assert np.all(np.abs(a - b).max(1)[aff] > 0)
    np.testing.assert_array_equal(a[~aff], b[~aff])


def test_user_loss_vs_numpy(small):
    nu, ni, up, uc, ip, ic = small
    U, V = O.init_embeddings(5, 0.3, 16, nu, ni)
    G = O.gramian(V)
    for half in (False, True):
        lo = O.user_loss(up, uc, U, V, G, 0.05, half)
        for u in range(nu):
            hist = uc[up[u]:up[u + 1]]
            if len(hist):
                assert abs(lo[u] - R.user_loss(hist, U[u], V, G, 0.05, half)) <= 1e-5 * abs(lo[u])
            else:
                assert lo[u] == 0


@pytest.mark.parametrize("epan,bw", [(False, 0.15), (True, 0.7)])
def test_safer2_scalar_math_vs_numpy(epan, bw):
    rng = np.random.default_rng(2)
    losses = (0.2 + 0.3 * rng.random(500)).astype(np.float32)
    for xi in (0.1, 0.3, 0.45):
        for l in losses[:20]:
            assert abs(O.safer2_weight(float(l), xi, bw, epan) -
                       R.safer2_weight(float(l), xi, bw, epan)) < 2e-6
    x_o = O.safer2_xi(losses, float(losses.mean()), 5, 0.3, bw, epan)
    x_r = R.safer2_xi(losses.astype(np.float64), float(losses.mean()), 5, 0.3, bw, epan)
    assert abs(x_o - x_r) < 1e-4 * max(1.0, abs(x_r))


def test_cvar_exact_quantile():
    l = np.array([0.5, 0.1, 0.9, 0.3, 0.7, 0.2, 0.8, 0.4, 0.6, 0.0], np.float32)
    # k = floor(10 * 0.3) = 3 -> 4th largest
    assert O.cvar_xi(l, 0.3) == pytest.approx(0.6)


def _run_gate(ml1m, model, epochs, dim=8, **kw):
    tr, vt, ve = ml1m
    nu, ni = tr.max_user + 1, tr.max_item + 1
    up, uc = tr.by_user()
    ip, ic = tr.by_item()
    ids, ep, ec = vt.compact_users()
    ids2, gp, gc = ve.compact_users()
    assert np.array_equal(ids, ids2)
    m = O.Model(model, dim, nu, ni, seed=1, **kw)
    m.set_data(up, uc, ip, ic)
    m.initialize()
    weights = []
    for _ in range(epochs):
        assert m.train() == 0
        weights.append(O.mean(m.state()[1]))  # GetMeanWeight: Eigen float mean
    Ue, rc = m.fold_in(ep, ec)
    assert rc == 0
    _, V = m.embeddings()
    rec, ndcg = O.evaluate(Ue, V, ep, ec, gp, gc, K_LIST)
    return ndcg.mean(0), weights


def test_gate_ials(ml1m):  # ials_test.cc:17-45
    ndcg, _ = _run_gate(ml1m, O.MODEL_IALS, 10, reg=0.003, w=0.1)
    assert ndcg[2] >= 0.2


def test_gate_erm(ml1m):  # erm_mf_test.cc:17-45
    ndcg, _ = _run_gate(ml1m, O.MODEL_ERM, 10, reg=0.005, w=0.004)
    assert ndcg[2] >= 0.2


def test_gate_cvar(ml1m):  # cvar_mf_test.cc:17-46
    ndcg, _ = _run_gate(ml1m, O.MODEL_CVAR, 50, reg=0.002, w=0.008, stepsize=0.4)
    assert ndcg[2] >= 0.2


@pytest.mark.parametrize("epan,bw", [(False, 0.15), (True, 0.7)])
def test_gate_safer2(ml1m, epan, bw):  # safer2_test.cc:17-32, 66-99, 135, 230
    ndcg, weights = _run_gate(ml1m, O.MODEL_SAFER2, 10, reg=0.004, w=0.004, bandwidth=bw,
                              epan=epan, xi_iterations=5, pd_iterations=1)
    assert ndcg[2] >= 0.2
    for mw in weights:
        assert abs(mw - 0.3) <= 0.02


def test_gate_safer2_snr(ml1m):  # safer2_test.cc:37-58, 149-185 (EXPECT_NEAR at :183)
    ndcg, weights = _run_gate(ml1m, O.MODEL_SAFER2, 10, reg=0.004, w=0.004, bandwidth=0.15,
                              xi_iterations=5, pd_iterations=1, use_snr=True, sampling_ratio=0.5)
    assert ndcg[2] >= 0.2
    for mw in weights:
        assert abs(mw - 0.3) <= 0.02


_LIBSTDCXX_PROG = r'''
#include <cstdio>
#include <random>
#include <vector>
int main() {
  // uniform_int_distribution<int>(0, n - 1) over mt19937, as ComputeXi's
  // SNR sampling (safer2.h:727-734) and the product's safer2.h use it
  std::mt19937 g(777u);
  for (int n : {1, 2, 3, 7, 1000, 4034, 116677, 2000000, 2147483647}) {
    std::uniform_int_distribution<int> uni(0, n - 1);
    for (int k = 0; k < 50; ++k) printf("%d\n", uni(g));
  }
}
'''


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ missing")
def test_uniform_int_matches_libstdcxx(tmp_path):
    src = tmp_path / "uni.cc"
    src.write_text(_LIBSTDCXX_PROG)
    exe = tmp_path / "uni"
    subprocess.run(["g++", "-O2", "-o", str(exe), str(src)], check=True)
    ref = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    import ctypes
    g = (ctypes.c_uint32 * 626)()
    O.lib().oracle_mt_seed(g, 777)
    got = []
    for n in (1, 2, 3, 7, 1000, 4034, 116677, 2000000, 2147483647):
        got += [int(O.lib().oracle_uniform_int(g, n)) for _ in range(50)]
    assert got == ref


@pytest.mark.parametrize("n", [1, 5, 15, 16, 17, 31, 32, 33, 47, 48, 64, 100, 4034, 116677])
def test_eigen_mean_restatement(n):
    """The packet-sum restatement is a float sum: equal to the exact mean to
    fp32 summation accuracy, and identical between oracle and a direct
    Python transcription of the same order."""
    x = np.random.default_rng(n).random(n).astype(np.float32)
    m = O.mean(x)
    assert abs(m - float(x.astype(np.float64).mean())) <= 1e-6 * max(1, n ** 0.5)
    P = 16
    f = np.float32
    al, al2 = n // P * P, n // (2 * P) * (2 * P)
    if al == 0:
        r = x[0]
        for v in x[1:]:
            r = f(r + v)
    else:
        p0 = x[:P].copy()
        if al > P:
            p1 = x[P:2 * P].copy()
            for i in range(2 * P, al2, 2 * P):
                p0 = (p0 + x[i:i + P]).astype(f)
                p1 = (p1 + x[i + P:i + 2 * P]).astype(f)
            p0 = (p0 + p1).astype(f)
            if al > al2:
                p0 = (p0 + x[al2:al2 + P]).astype(f)
        s8 = (p0[:8] + p0[8:]).astype(f)
        s4 = (s8[:4] + s8[4:]).astype(f)
        r = f(f(s4[0] + s4[2]) + f(s4[1] + s4[3]))
        for v in x[al:]:
            r = f(r + v)
    assert np.float32(m) == np.float32(r / f(n))


@pytest.mark.parametrize("dim", [8, 50, 256])
def test_cpu_baseline_matches_oracle(quirk_data, dim):
    """The timed CPU baseline (oracle/cpu_baseline.c: blocked SYRK, blocked
    LLT with an explicit panel inverse) computes the same half-steps as the
    oracle (kinds 0 / 1 / 2, tail quirk on) within rounding."""
    nu, ni, up, uc, ip, ic = quirk_data
    U, V = O.init_embeddings(1, 0.1, dim, nu, ni)
    G = O.gramian(V)
    hu = np.diff(up)
    Uo, rc = O.step(up, uc, V, G, 0, 0.003, 0.1, out=U.copy())
    Ub, rc2 = O.baseline_step(up, uc, V, G, 0, 0.003, 0.1, out=U.copy(), nthreads=4)
    assert rc == rc2 == 0
    assert rel_rows(Ub[hu > 0], Uo[hu > 0]).max() < 1e-4
    om = (0.05 + 0.95 * np.random.default_rng(5).random(nu)).astype(np.float32)
    Uo, _ = O.step(up, uc, V, G, 1, 0.004, 0.004, entity_weight=om, out=U.copy())
    Ub, _ = O.baseline_step(up, uc, V, G, 1, 0.004, 0.004, entity_weight=om, out=U.copy(),
                            nthreads=4)
    assert rel_rows(Ub[hu > 0], Uo[hu > 0]).max() < 1e-4
    hs = np.where(hu > 0, hu, 1).astype(np.float32)
    nuw = (om / hs).astype(np.float32)
    er = np.add.reduceat((1.0 / hs.astype(np.float64))[ic], ip[:-1]).astype(np.float32)
    Gw = O.gramian(U, om)
    hi = np.diff(ip)
    Vo, _ = O.step(ip, ic, U, Gw, 2, 0.004, 0.004, alpha=0.3, entity_reg=er, other_weight=nuw,
                   out=V.copy())
    Vb, _ = O.baseline_step(ip, ic, U, Gw, 2, 0.004, 0.004, alpha=0.3, entity_reg=er,
                            other_weight=nuw, out=V.copy(), nthreads=4)
    assert rel_rows(Vb[hi > 0], Vo[hi > 0]).max() < 1e-4
