"""BASELINE configs[4] at its real size on one GPU: SAFER2, d = 1024, the
2M x 500K synthetic set with 1e8 interactions (README.md:100 flags,
use_snr 0), the default wide workspace budget (FRECSYS_WIDE_WS_MB unset:
16 GB per workspace, capped by the device's free memory, capi.hip).

The product's C++ model (libfrecsys_model.so) runs Initialize() and one
Train() epoch (safer2.h:266-334, 819-838): ComputeUserWeights, StepU over 2M
users (history-space buckets, the history-space wide bucket of the users with
256 < h <= 512 and the wide d-space batches of the longer ones), StepV over
500K items (the omega-weighted Gramian of 2M user rows, the basis of it, the
wide bucket, the wide d-space items incl. the split slabs of the head items
up to 581K rows, the tail quirk), V^T V, ComputeUserLoss, xi.

Each sampled row is then stepped from the GPU's own inputs (V0 and its
Gramian after Initialize(), the omega the epoch used, U after the epoch and
the omega-weighted Gramian the V step used, item_reg_) by the CPU oracle and
compared at the 1e-4 row bar: the 20 longest users and items, 100 random
rows per side.  The 20 longest items (up to 581K rows; one oracle SYRK of
the head item alone would take minutes single-threaded) are stepped by the
float64 restatement tests/numpy_ref.py (BLAS), which test_oracle.py pins to
the oracle.  The two Gramians are checked against float64 products on
random probe vectors, item_reg_ against the reference's float accumulation
(safer2.h:831-837) on the sampled items.

The fixture takes ~1-2 min on the box (data ~40 s, seeded init of 2.56G
normals, one epoch ~2 s, downloads); progress goes to
gpurun_out/progress_config5.log.
"""
import os
import time

import numpy as np
import pytest

import numpy_ref as R
import oracle as O
from conftest import ROOT, rel_rows
from test_models_gpu import report

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

fh = pytest.importorskip("frecsys_hip")
from frecsys_hip.data import SHAPES, synthetic  # noqa: E402

TOL_ROW = 1e-4
FLAGS = dict(l2_reg=0.0012, uobs_weight=0.0004, alpha=0.3, bandwidth=0.1, xi_iterations=5,
             pd_iterations=1)
D = 1024
PROGRESS = os.path.join(ROOT, "gpurun_out", "progress_config5.log")


def _progress(msg, t0=[time.time()]):
    try:
        os.makedirs(os.path.dirname(PROGRESS), exist_ok=True)
        with open(PROGRESS, "a") as f:
            f.write(f"[{time.time() - t0[0]:7.1f}s] {msg}\n")
    except OSError:
        pass


@pytest.fixture(scope="module")
def c5():
    _progress("generating 2M x 500K data")
    up, uc, ip, ic = synthetic(SHAPES["2m500k"])
    nu, ni = len(up) - 1, len(ip) - 1
    _progress(f"data {nu} x {ni}, nnz {int(up[-1])}; creating model")
    users = np.repeat(np.arange(nu, dtype=np.int32), np.diff(up))
    m = fh.Model("safer2", users, uc, dim=D, stdev=0.1, seed=1, print_train_stats=False,
                 use_snr=False, **FLAGS)
    del users
    assert (m.n_users, m.n_items) == (nu, ni)
    ctx = m.context()
    _progress("initialize()")
    m.initialize()
    V0 = ctx.get_embeddings(fh.SIDE_ITEM)
    U0 = ctx.get_embeddings(fh.SIDE_USER)
    GV0 = ctx.get_gramian(fh.SIDE_ITEM)
    _progress("train(1)")
    t = time.time()
    m.train(1)
    epoch_s = time.time() - t
    _progress(f"epoch {epoch_s:.2f} s; fetching state")
    U1 = ctx.get_embeddings(fh.SIDE_USER)
    V1 = ctx.get_embeddings(fh.SIDE_ITEM)
    GU1 = ctx.get_gramian(fh.SIDE_USER)  # U1^T diag(omega) U1 of the V step
    omega, loss, item_reg, xi = m.dual_state()
    # the silent slow path never taken (frecsys_counter)
    reruns, timeouts = ctx.counter("hspace_reruns"), ctx.counter("tagged_timeouts")
    m.close()
    assert (reruns, timeouts) == (0, 0)
    _progress("fixture done")
    return dict(up=up, uc=uc, ip=ip, ic=ic, U0=U0, V0=V0, GV0=GV0, U1=U1, V1=V1, GU1=GU1,
                omega=omega, loss=loss, item_reg=item_reg, xi=xi, epoch_s=epoch_s)


def _sample(ptr, n_long, n_rand, seed):
    h = np.diff(ptr)
    longest = np.argsort(-h, kind="stable")[:n_long]
    rng = np.random.default_rng(seed)
    nz = np.nonzero(h > 0)[0]
    rand = rng.choice(np.setdiff1d(nz, longest), n_rand, replace=False)
    return np.sort(longest), np.sort(rand)


def _sub_csr(ptr, col, rows):
    h = np.diff(ptr)[rows]
    rp = np.concatenate([[0], np.cumsum(h)]).astype(np.int64)
    cl = np.concatenate([col[ptr[r]:ptr[r + 1]] for r in rows]).astype(np.int32)
    return rp, cl


def _check(name, got, ref, rows, ptr):
    e = rel_rows(got, ref)
    h = np.diff(ptr)[rows]
    report(test="config5", case=name, rows=int(len(rows)), max_h=int(h.max()), max=float(e.max()),
           worst_h=int(h[int(np.argmax(e))]), over_1e4=int((e > TOL_ROW).sum()))
    _progress(f"{name}: {len(rows)} rows, max h {int(h.max())}, max row err {float(e.max()):.2e}")
    assert e.max() < TOL_ROW, (name, float(e.max()), int(h[int(np.argmax(e))]))


def test_config5_user_halfstep(c5):
    """ProjectU (safer2.h:104-163) of the 20 longest + 100 random users, from V0,
    its Gramian and the epoch's omega."""
    up, uc = c5["up"], c5["uc"]
    longest, rand = _sample(up, 20, 100, 51)
    rows = np.concatenate([longest, rand])
    rp, cl = _sub_csr(up, uc, rows)
    Uo, rc = O.step(rp, cl, c5["V0"], c5["GV0"], 1, FLAGS["l2_reg"], FLAGS["uobs_weight"],
                    entity_weight=c5["omega"][rows], out=c5["U0"][rows].copy())
    assert rc == 0
    assert np.diff(up)[longest].min() > 256  # the wide d-space path
    _check("config5_user", c5["U1"][rows], Uo, rows, up)
    # omega = 1 - Kcdf(-(loss0 - xi0)) (safer2.h:770-776): in (0, 1)
    assert 0.0 < float(np.mean(c5["omega"])) < 1.0


def _item_reg_ref(ip, ic, up, rows):
    """item_reg_[v] = sum over H_v of 1/|H_u|, double adds stored as float in
    by_item order (safer2.h:831-837)."""
    h = np.diff(up).astype(np.float32)
    out = np.zeros(len(rows), np.float32)
    for k, v in enumerate(rows):
        inv = 1.0 / h[ic[ip[v]:ip[v + 1]]].astype(np.float64)
        acc = np.float32(0)
        for x in inv:
            acc = np.float32(np.float64(acc) + x)
        out[k] = acc
    return out


def test_config5_item_halfstep_random(c5):
    """ProjectV (safer2.h:166-221, tail quirk) of 100 random items by the oracle,
    from U after the epoch, the omega-weighted Gramian of the V step, nu and
    item_reg_."""
    up, ip, ic = c5["up"], c5["ip"], c5["ic"]
    _, rows = _sample(ip, 20, 100, 52)
    reg_rows = _item_reg_ref(ip, ic, up, rows)
    np.testing.assert_array_equal(c5["item_reg"][rows], reg_rows)
    nu_w = (c5["omega"] / np.diff(up).astype(np.float32)).astype(np.float32)
    rp, cl = _sub_csr(ip, ic, rows)
    Vo, rc = O.step(rp, cl, c5["U1"], c5["GU1"], 2, FLAGS["l2_reg"], FLAGS["uobs_weight"],
                    alpha=FLAGS["alpha"], entity_reg=reg_rows, other_weight=nu_w,
                    out=c5["V0"][rows].copy())
    assert rc == 0
    _check("config5_item_random", c5["V1"][rows], Vo, rows, ip)


def _heff_v(h):
    return np.where((h > 128) & (h % 128 != 0), h + 128 - h % 128, h)


def test_config5_wide_bucket_rows(c5):
    """Rows the history-space wide bucket solves at this size (256 < h_eff <=
    512, on by default at Dp = 1024): 40 users (ProjectU, omega) and 40 items
    (ProjectV, nu, item_reg_, the tail quirk's h_eff) by the oracle.  The
    random samples above hold only a couple of them."""
    up, uc, ip, ic = c5["up"], c5["uc"], c5["ip"], c5["ic"]
    rng = np.random.default_rng(55)
    hu = np.diff(up)
    urows = np.sort(rng.choice(np.nonzero((hu > 256) & (hu <= 512))[0], 40, replace=False))
    rp, cl = _sub_csr(up, uc, urows)
    Uo, rc = O.step(rp, cl, c5["V0"], c5["GV0"], 1, FLAGS["l2_reg"], FLAGS["uobs_weight"],
                    entity_weight=c5["omega"][urows], out=c5["U0"][urows].copy())
    assert rc == 0
    _check("config5_user_wide_bucket", c5["U1"][urows], Uo, urows, up)
    he = _heff_v(np.diff(ip))
    irows = np.sort(rng.choice(np.nonzero((he > 256) & (he <= 512))[0], 40, replace=False))
    reg_rows = _item_reg_ref(ip, ic, up, irows)
    nu_w = (c5["omega"] / hu.astype(np.float32)).astype(np.float32)
    rp, cl = _sub_csr(ip, ic, irows)
    Vo, rc = O.step(rp, cl, c5["U1"], c5["GU1"], 2, FLAGS["l2_reg"], FLAGS["uobs_weight"],
                    alpha=FLAGS["alpha"], entity_reg=reg_rows, other_weight=nu_w,
                    out=c5["V0"][irows].copy())
    assert rc == 0
    _check("config5_item_wide_bucket", c5["V1"][irows], Vo, irows, ip)


def test_config5_item_halfstep_longest(c5):
    """The 20 longest items (up to ~581K rows: split slabs, two-level
    accumulation, tail quirk) by the float64 restatement (numpy_ref.py)."""
    up, ip, ic = c5["up"], c5["ip"], c5["ic"]
    rows, _ = _sample(ip, 20, 0, 53)
    h_items = np.diff(ip)[rows]
    assert h_items.max() > 100_000
    reg_rows = _item_reg_ref(ip, ic, up, rows)
    np.testing.assert_array_equal(c5["item_reg"][rows], reg_rows)
    nu_w = (c5["omega"] / np.diff(up).astype(np.float32)).astype(np.float32)
    lam_base = np.float32(FLAGS["alpha"] * FLAGS["uobs_weight"] * (len(up) - 1))
    U1, G = c5["U1"], c5["GU1"].astype(np.float64)
    ref = np.zeros((len(rows), D), np.float64)
    for k, v in enumerate(rows):
        # lambda_v = l2_reg * (item_reg_[v] + alpha * w * N_u)   (safer2.h:426-432)
        lam = np.float32(np.float32(FLAGS["l2_reg"]) * (reg_rows[k] + lam_base))
        ref[k] = R.project_v(ic[ip[v]:ip[v + 1]], U1, G, float(lam), FLAGS["uobs_weight"],
                             nu_w, True)
    _check("config5_item_longest", c5["V1"][rows], ref, rows, ip)


def test_config5_gramians(c5):
    """G_V0 = V0^T V0 and G_U1 = U1^T diag(omega) U1 on float64 probes."""
    rng = np.random.default_rng(54)
    for name, X, w, G in (("V0^T V0", c5["V0"], None, c5["GV0"]),
                          ("U1^T diag(omega) U1", c5["U1"], c5["omega"], c5["GU1"])):
        Z = rng.standard_normal((D, 3))
        ref = np.zeros((D, 3))
        for i in range(0, X.shape[0], 250_000):  # X^T diag(w) X Z in float64, by row chunks
            Xc = X[i:i + 250_000].astype(np.float64)
            Y = Xc @ Z
            if w is not None:
                Y *= w[i:i + 250_000, None]
            ref += Xc.T @ Y
        got = G.astype(np.float64) @ Z
        for k in range(3):
            err = np.linalg.norm(got[:, k] - ref[:, k]) / np.linalg.norm(ref[:, k])
            assert err < 1e-5, (name, err)
        # symmetric, bitwise (the reduce mirrors the lower triangle)
        np.testing.assert_array_equal(G, G.T)
