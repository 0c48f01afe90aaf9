"""Parity at the BASELINE workload sizes (BASELINE.json configs[1..4]).

The small fixtures of test_parity_gpu.py never reach what these shapes hold:
item histories of ~55K rows (ML-20M head; split-slab SYRK), every
history-space bucket on both streams, the 344 MB LDL tables, d = 512 / 1024
through wide.hip with workspace batching.  Each test runs the product's
half-steps (or a whole Train() epoch) at the full size on the GPU and checks
against the CPU oracle on a fixed sample of rows that includes the longest
histories -- the oracle's d^3 cost bounds the sample, not the GPU run.
Bar: every sampled row within 1e-4 relative (north_star).

Reference hyper-parameters: README.md:84 (iALS ML-20M), :79 (SAFER2 ML-20M,
use_snr 0 for parity), :105 (iALS MSD), :100 (SAFER2 MSD flags, used for the
2M x 500K slice at d = 1024).
"""
import numpy as np
import pytest

import oracle as O
from conftest import rel_rows
from test_models_gpu import report

pytestmark = pytest.mark.gpu

fh = pytest.importorskip("frecsys_hip")
from frecsys_hip.data import SHAPES, SynthShape, synthetic  # noqa: E402

TOL_ROW = 1e-4
# a 2M x 500K-proportioned slice (mean 50 per user, 200 per item as config 5)
SLICE_2M500K = SynthShape(200_000, 50_000, 10_000_000, min_uc=5)


def _sample(ptr, n_long, n_rand, seed):
    """The n_long longest histories + n_rand random non-empty rows, sorted."""
    h = np.diff(ptr)
    longest = np.argsort(-h, kind="stable")[:n_long]
    rng = np.random.default_rng(seed)
    nz = np.nonzero(h > 0)[0]
    rand = rng.choice(nz, min(n_rand, len(nz)), replace=False)
    return np.unique(np.concatenate([longest, rand]))


def _sub_csr(ptr, col, rows):
    h = np.diff(ptr)[rows]
    rp = np.concatenate([[0], np.cumsum(h)]).astype(np.int64)
    cl = np.concatenate([col[ptr[r]:ptr[r + 1]] for r in rows]).astype(np.int32)
    return rp, cl


def _check(name, got, ref, rows, ptr, **kw):
    e = rel_rows(got[rows], ref)
    h = np.diff(ptr)[rows]
    report(test="workload", case=name, rows=int(len(rows)), max_h=int(h.max()),
           max=float(e.max()), p999=float(np.percentile(e, 99.9)),
           worst_h=int(h[int(np.argmax(e))]), over_1e4=int((e > TOL_ROW).sum()), **kw)
    assert e.max() < TOL_ROW, (name, float(e.max()), int(h[int(np.argmax(e))]))


def _no_slow_path(ctx):
    """No history-space side reran in d-space and no tagged poll timed out
    (frecsys_counter): the benchmark data never takes the silent slow path."""
    assert ctx.counter("hspace_reruns") == 0
    assert ctx.counter("tagged_timeouts") == 0


@pytest.fixture(scope="module")
def ml20m():
    return synthetic(SHAPES["ml20m"])


def _context(dim, up, uc, ip, ic, seed=1):
    nu, ni = len(up) - 1, len(ip) - 1
    ctx = fh.Context(dim, nu, ni)
    ctx.load_csr(fh.SIDE_USER, up, uc)
    ctx.load_csr(fh.SIDE_ITEM, ip, ic)
    ctx.init_embeddings(seed, 0.1)
    return ctx


def test_ials_ml20m_d256_half_steps(ml20m):
    """configs[1]: one seeded iALS half-step each way at full size."""
    up, uc, ip, ic = ml20m
    reg, w, d = 0.003, 0.1, 256
    ctx = _context(d, up, uc, ip, ic)
    U0 = ctx.get_embeddings(fh.SIDE_USER)
    V0 = ctx.get_embeddings(fh.SIDE_ITEM)
    ctx.gramian(fh.SIDE_ITEM, fetch=False)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, reg, w)
    Ug = ctx.get_embeddings(fh.SIDE_USER)
    rows = _sample(up, 50, 1000, 11)
    rp, cl = _sub_csr(up, uc, rows)
    Uo, rc = O.step(rp, cl, V0, O.gramian(V0), 0, reg, w, out=U0[rows].copy())
    assert rc == 0
    _check("ials_ml20m_d256_user", Ug, Uo, rows, up)
    # V half-step from the GPU's U (identical inputs on both sides)
    ctx.gramian(fh.SIDE_USER, fetch=False)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, reg, w)
    Vg = ctx.get_embeddings(fh.SIDE_ITEM)
    rows = _sample(ip, 50, 1000, 12)  # includes the > 2048-row split-slab items
    assert np.diff(ip)[rows].max() > 2 * 1024
    rp, cl = _sub_csr(ip, ic, rows)
    Vo, rc = O.step(rp, cl, Ug, O.gramian(Ug), 0, reg, w, out=V0[rows].copy())
    assert rc == 0
    _check("ials_ml20m_d256_item", Vg, Vo, rows, ip)
    _no_slow_path(ctx)
    ctx.close()


@pytest.mark.parametrize("use_snr", [False, True])
def test_safer2_ml20m_d256_train_epoch(ml20m, use_snr):
    """configs[2]: Initialize() + one SAFER2 Train() epoch of the product's C++
    model (libfrecsys_model.so) vs the oracle's whole-model restatement, every
    row compared (README.md:79 flags; use_snr 0, and use_snr 1 with
    sampling_ratio 0.1 as the bench times it: ComputeXi on N_u / 10 samples
    drawn from the same seeded stream, safer2.h:716-742)."""
    up, uc, ip, ic = ml20m
    nu, ni = len(up) - 1, len(ip) - 1
    d = 256
    flags = dict(l2_reg=0.002, uobs_weight=0.002, alpha=0.3, bandwidth=0.18, xi_iterations=5,
                 pd_iterations=1)
    users = np.repeat(np.arange(nu, dtype=np.int32), np.diff(up))
    m = fh.Model("safer2", users, uc, dim=d, stdev=0.1, seed=1, print_train_stats=False,
                 use_snr=use_snr, sampling_ratio=0.1, **flags)
    assert (m.n_users, m.n_items) == (nu, ni)
    m.initialize()
    m.train(1)
    ctx = m.context()
    U, V = ctx.get_embeddings(fh.SIDE_USER), ctx.get_embeddings(fh.SIDE_ITEM)
    mw = m.mean_weight()
    w_gpu, l_gpu, _, xi_gpu = m.dual_state()
    _no_slow_path(ctx)
    m.close()
    om = O.Model(O.MODEL_SAFER2, d, nu, ni, reg=flags["l2_reg"], w=flags["uobs_weight"],
                 alpha=flags["alpha"], bandwidth=flags["bandwidth"], xi_iterations=5,
                 pd_iterations=1, seed=1, use_snr=use_snr, sampling_ratio=0.1)
    om.set_data(up, uc, ip, ic)
    om.initialize()
    assert om.train() == 0
    Uo, Vo = om.embeddings()
    lo, wo, xo = om.state()
    all_u, all_i = np.arange(nu), np.arange(ni)
    tag = "_snr" if use_snr else ""
    _check(f"safer2_ml20m_d256_epoch{tag}_user", U, Uo, all_u, up)
    _check(f"safer2_ml20m_d256_epoch{tag}_item", V, Vo, all_i, ip)
    assert abs(mw - float(np.mean(wo.astype(np.float64)))) < 1e-4, (mw, float(np.mean(wo)))
    # the dual state after the epoch: losses, xi (the same seeded SNR draws)
    np.testing.assert_allclose(l_gpu, lo, rtol=1e-4, atol=1e-7)
    assert abs(xi_gpu - float(xo)) <= 1e-4 * max(1.0, abs(float(xo))), (xi_gpu, float(xo))
    np.testing.assert_allclose(w_gpu, wo, rtol=0, atol=1e-4)


@pytest.fixture(scope="module")
def msd():
    return synthetic(SHAPES["msd"])


def test_ials_msd_d512_half_steps(msd):
    """configs[3] (one GPU): d = 512, wide d-space path for h > 256 (items up to
    ~190K rows), history-space for the rest."""
    up, uc, ip, ic = msd
    reg, w, d = 0.002, 0.05, 512
    ctx = _context(d, up, uc, ip, ic)
    U0 = ctx.get_embeddings(fh.SIDE_USER)
    V0 = ctx.get_embeddings(fh.SIDE_ITEM)
    ctx.gramian(fh.SIDE_ITEM, fetch=False)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, reg, w)
    Ug = ctx.get_embeddings(fh.SIDE_USER)
    rows = _sample(up, 20, 500, 21)
    rp, cl = _sub_csr(up, uc, rows)
    Uo, rc = O.step(rp, cl, V0, O.gramian(V0), 0, reg, w, out=U0[rows].copy())
    assert rc == 0
    _check("ials_msd_d512_user", Ug, Uo, rows, up)
    ctx.gramian(fh.SIDE_USER, fetch=False)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, reg, w)
    Vg = ctx.get_embeddings(fh.SIDE_ITEM)
    rows = _sample(ip, 8, 300, 22)
    rp, cl = _sub_csr(ip, ic, rows)
    Vo, rc = O.step(rp, cl, Ug, O.gramian(Ug), 0, reg, w, out=V0[rows].copy())
    assert rc == 0
    _check("ials_msd_d512_item", Vg, Vo, rows, ip)
    _no_slow_path(ctx)
    ctx.close()


def test_safer2_2m500k_slice_d1024_half_steps(monkeypatch):
    """configs[4] on one GPU: a 200K x 50K slice with config 5's history means,
    d = 1024, the weighted SAFER2 kinds (ProjectU with omega, ProjectV with
    nu and the tail quirk), the wide workspace in many batches."""
    monkeypatch.setenv("FRECSYS_WIDE_WS_MB", "256")  # ~116 entities per workspace batch
    up, uc, ip, ic = synthetic(SLICE_2M500K, seed=4242)
    nu, ni = len(up) - 1, len(ip) - 1
    reg, w, alpha, d = 0.0012, 0.0004, 0.3, 1024
    ctx = _context(d, up, uc, ip, ic)
    U0 = ctx.get_embeddings(fh.SIDE_USER)
    V0 = ctx.get_embeddings(fh.SIDE_ITEM)
    om = (0.05 + 0.95 * np.random.default_rng(5).random(nu)).astype(np.float32)
    ctx.gramian(fh.SIDE_ITEM, fetch=False)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_WEIGHTED_U, reg, w, entity_weight=om)
    Ug = ctx.get_embeddings(fh.SIDE_USER)
    rows = _sample(up, 10, 80, 31)
    rp, cl = _sub_csr(up, uc, rows)
    Uo, rc = O.step(rp, cl, V0, O.gramian(V0), 1, reg, w, entity_weight=om[rows],
                    out=U0[rows].copy())
    assert rc == 0
    _check("safer2_slice_d1024_user", Ug, Uo, rows, up)
    # ProjectV inputs (safer2.h:499-509, 827-837)
    h = np.diff(up).astype(np.float32)
    nu_w = (om / h).astype(np.float32)
    inv = (1.0 / h.astype(np.float64))[ic]
    rows = _sample(ip, 10, 80, 32)
    # item_reg_ for every item (float64 sums; only the sampled rows, with the
    # reference's float accumulation in by_item order, safer2.h:831-837, are
    # compared -- both sides get the same values)
    full_reg = np.add.reduceat(inv, ip[:-1]).astype(np.float32)
    for v in rows:
        acc = np.float32(0)
        for x in inv[ip[v]:ip[v + 1]]:
            acc = np.float32(np.float64(acc) + x)
        full_reg[v] = acc
    ctx.gramian(fh.SIDE_USER, weights=om, fetch=False)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, reg, w, alpha=alpha, entity_reg=full_reg,
                   other_weight=nu_w)
    Vg = ctx.get_embeddings(fh.SIDE_ITEM)
    rp, cl = _sub_csr(ip, ic, rows)
    Vo, rc = O.step(rp, cl, Ug, O.gramian(Ug, om), 2, reg, w, alpha=alpha,
                    entity_reg=full_reg[rows], other_weight=nu_w, out=V0[rows].copy())
    assert rc == 0
    _check("safer2_slice_d1024_item", Vg, Vo, rows, ip)
    _no_slow_path(ctx)
    ctx.close()
