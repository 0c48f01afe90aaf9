"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the timed CPU baseline.  See
frecsys_oracle.h for the parity status of the restatement.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "liboracle.so")
P, I32, I64, F = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float

MODEL_IALS, MODEL_ERM, MODEL_CVAR, MODEL_SAFER2 = range(4)


class SolveParams(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("reg", F), ("reg_exp", F), ("w", F), ("alpha", F),
                ("stepsize", F), ("quirk", ctypes.c_int), ("entity_weight", P),
                ("entity_reg", P), ("other_weight", P)]


class ModelParams(ctypes.Structure):
    _fields_ = [("model", ctypes.c_int), ("dim", ctypes.c_int), ("n_users", I64),
                ("n_items", I64), ("reg", F), ("reg_exp", F), ("w", F), ("stdev", F),
                ("alpha", F), ("bandwidth", F), ("stepsize", F), ("xi_iterations", ctypes.c_int),
                ("pd_iterations", ctypes.c_int), ("use_epanechnikov", ctypes.c_int),
                ("quirk", ctypes.c_int), ("nthreads", ctypes.c_int), ("use_snr", ctypes.c_int),
                ("sampling_ratio", F)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "oracle_init_embeddings": (None, [ctypes.c_uint32, F, ctypes.c_int, P, I64, P, I64]),
            "oracle_gramian": (None, [P, I64, ctypes.c_int, P, P, ctypes.c_int]),
            "oracle_step": (I64, [I64, P, P, P, I64, ctypes.c_int, P, P, P, P, ctypes.c_int]),
            "oracle_user_loss": (None, [I64, P, P, P, P, ctypes.c_int, P, F, ctypes.c_int, P,
                                        ctypes.c_int]),
            "oracle_safer2_weight": (F, [F, F, F, ctypes.c_int]),
            "oracle_safer2_xi": (F, [P, I64, F, ctypes.c_int, F, F, ctypes.c_int]),
            "oracle_cvar_xi": (F, [P, I64, F]),
            "oracle_model_create": (P, [P, ctypes.c_uint32]),
            "oracle_model_destroy": (None, [P]),
            "oracle_model_set_data": (None, [P, P, P, P, P]),
            "oracle_model_set_embeddings": (None, [P, P, P]),
            "oracle_model_get_embeddings": (None, [P, P, P]),
            "oracle_model_initialize": (None, [P]),
            "oracle_model_train": (I64, [P]),
            "oracle_model_get_state": (None, [P, P, P, P]),
            "oracle_model_fold_in": (I64, [P, I64, P, P, P]),
            "oracle_evaluate": (None, [I64, P, P, I64, ctypes.c_int, P, P, P, P, P, ctypes.c_int,
                                       P, P, ctypes.c_int]),
            "oracle_pp_predict": (None, [I64, P, P, P, P, ctypes.c_int, P, P, ctypes.c_int]),
            "oracle_pp_step": (I64, [I64, P, P, P, P, I64, ctypes.c_int, P, P, ctypes.c_int,
                                     ctypes.c_int, P, P, P, ctypes.c_int]),
            "oracle_mt_seed": (None, [P, ctypes.c_uint32]),
            "oracle_mt_next": (ctypes.c_uint32, [P]),
            "oracle_uniform_int": (ctypes.c_uint32, [P, ctypes.c_uint32]),
            "oracle_mean": (F, [P, I64]),
            "oracle_safer2_xi_snr": (F, [P, I64, F, ctypes.c_int, F, F, ctypes.c_int, F, P]),
            "cpu_baseline_step": (I64, [I64, P, P, P, I64, ctypes.c_int, P, ctypes.c_int, F, F, F,
                                        F, ctypes.c_int, P, P, P, P, ctypes.c_int]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(P)


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def init_embeddings(seed, stdev, dim, n_users, n_items):
    U = np.empty((n_users, dim), np.float32)
    V = np.empty((n_items, dim), np.float32)
    lib().oracle_init_embeddings(seed, stdev, dim, _p(U), n_users, _p(V), n_items)
    return U, V


def gramian(X, w=None, nthreads=0):
    X = f32(X)
    d = X.shape[1]
    G = np.empty((d, d), np.float32)
    wv = None if w is None else f32(w)
    lib().oracle_gramian(_p(X), X.shape[0], d, _p(wv), _p(G), nthreads)
    return G


def step(row_ptr, col, X, G, kind, reg, w, reg_exp=1.0, alpha=0.0, stepsize=0.0, quirk=1,
         entity_weight=None, entity_reg=None, other_weight=None, E=None, out=None, nthreads=0):
    """One side step; rows with empty history keep `out`'s values."""
    rp = np.ascontiguousarray(row_ptr, np.int64)
    cl = np.ascontiguousarray(col, np.int32)
    X, G = f32(X), f32(G)
    n = len(rp) - 1
    d = X.shape[1]
    if out is None:
        out = np.zeros((n, d), np.float32) if E is None else f32(E).copy()
    ew = None if entity_weight is None else f32(entity_weight)
    er = None if entity_reg is None else f32(entity_reg)
    ow = None if other_weight is None else f32(other_weight)
    Ev = None if E is None else f32(E)
    sp = SolveParams(kind, reg, reg_exp, w, alpha, stepsize, quirk, _p(ew), _p(er), _p(ow))
    rc = lib().oracle_step(n, _p(rp), _p(cl), _p(X), X.shape[0], d, _p(G), ctypes.byref(sp),
                           _p(Ev), _p(out), nthreads)
    return out, int(rc)


def baseline_step(row_ptr, col, X, G, kind, reg, w, reg_exp=1.0, alpha=0.0, quirk=1,
                  entity_weight=None, entity_reg=None, other_weight=None, out=None, nthreads=1):
    """The timed CPU baseline (cpu_baseline.c): the same half-step as step()
    for kinds 0 / 1 / 2, cache-blocked and vectorised like Eigen's path."""
    rp = np.ascontiguousarray(row_ptr, np.int64)
    cl = np.ascontiguousarray(col, np.int32)
    X, G = f32(X), f32(G)
    n = len(rp) - 1
    d = X.shape[1]
    if out is None:
        out = np.zeros((n, d), np.float32)
    ew = None if entity_weight is None else f32(entity_weight)
    er = None if entity_reg is None else f32(entity_reg)
    ow = None if other_weight is None else f32(other_weight)
    rc = lib().cpu_baseline_step(n, _p(rp), _p(cl), _p(X), X.shape[0], d, _p(G), kind, reg,
                                 reg_exp, w, alpha, quirk, _p(ew), _p(er), _p(ow), _p(out),
                                 nthreads)
    return out, int(rc)


def pp_predict(row_ptr, col, rix, X, E, pred, nthreads=0):
    """iALS++ PredictDataset into pred (float32, in place)."""
    rp = np.ascontiguousarray(row_ptr, np.int64)
    cl = np.ascontiguousarray(col, np.int32)
    rx = np.ascontiguousarray(rix, np.int32)
    X, E = f32(X), f32(E)
    assert pred.dtype == np.float32 and pred.flags.c_contiguous
    lib().oracle_pp_predict(len(rp) - 1, _p(rp), _p(cl), _p(rx), _p(X), X.shape[1], _p(E),
                            _p(pred), nthreads)


def pp_step(row_ptr, col, rix, X, E, pred, start, end, reg, w, reg_exp=1.0, kind=0, alpha=0.0,
            entity_weight=None, entity_reg=None, other_weight=None, gram_w=None, nthreads=0):
    """iALS++ (kind 0) / SAFER2++ U (1) / V (2) block Step on columns
    [start, end): E (float32) and pred updated in place.  Returns (first
    failing row + 1 or 0, residual)."""
    rp = np.ascontiguousarray(row_ptr, np.int64)
    cl = np.ascontiguousarray(col, np.int32)
    rx = np.ascontiguousarray(rix, np.int32)
    X = f32(X)
    assert E.dtype == np.float32 and E.flags.c_contiguous
    ew = None if entity_weight is None else f32(entity_weight)
    er = None if entity_reg is None else f32(entity_reg)
    ow = None if other_weight is None else f32(other_weight)
    gw = None if gram_w is None else f32(gram_w)
    sp = SolveParams(kind, reg, reg_exp, w, alpha, 0.0, 0, _p(ew), _p(er), _p(ow))
    res = ctypes.c_double(0.0)
    rc = lib().oracle_pp_step(len(rp) - 1, _p(rp), _p(cl), _p(rx), _p(X), X.shape[0], X.shape[1],
                              _p(E), _p(pred), start, end, ctypes.byref(sp), _p(gw),
                              ctypes.byref(res), nthreads)
    return int(rc), res.value


def user_loss(row_ptr, col, U, V, G, beta, half, nthreads=0):
    rp = np.ascontiguousarray(row_ptr, np.int64)
    cl = np.ascontiguousarray(col, np.int32)
    U, V, G = f32(U), f32(V), f32(G)
    out = np.zeros(len(rp) - 1, np.float32)
    lib().oracle_user_loss(len(rp) - 1, _p(rp), _p(cl), _p(U), _p(V), U.shape[1], _p(G), beta,
                           1 if half else 0, _p(out), nthreads)
    return out


def safer2_weight(loss, xi, bandwidth, epan=False):
    return float(lib().oracle_safer2_weight(loss, xi, bandwidth, 1 if epan else 0))


def safer2_xi(loss, prev_xi, iterations, alpha, bandwidth, epan=False):
    l = f32(loss)
    return float(lib().oracle_safer2_xi(_p(l), len(l), prev_xi, iterations, alpha, bandwidth,
                                        1 if epan else 0))


def cvar_xi(loss, alpha):
    l = f32(loss)
    return float(lib().oracle_cvar_xi(_p(l), len(l), alpha))


class Model:
    """Whole-model restatement (Train() sequences of the four models)."""

    def __init__(self, model, dim, n_users, n_items, reg, w, stdev=0.1, alpha=0.3, reg_exp=1.0,
                 bandwidth=1.0, stepsize=0.1, xi_iterations=5, pd_iterations=1, epan=False,
                 quirk=1, nthreads=0, seed=1, use_snr=False, sampling_ratio=0.1):
        self.p = ModelParams(model, dim, n_users, n_items, reg, reg_exp, w, stdev, alpha,
                             bandwidth, stepsize, xi_iterations, pd_iterations, 1 if epan else 0,
                             quirk, nthreads, 1 if use_snr else 0, sampling_ratio)
        self.h = lib().oracle_model_create(ctypes.byref(self.p), seed)
        self.dim, self.n_users, self.n_items = dim, n_users, n_items
        self._keep = []

    def set_data(self, up, uc, ip, ic):
        arrs = [np.ascontiguousarray(up, np.int64), np.ascontiguousarray(uc, np.int32),
                np.ascontiguousarray(ip, np.int64), np.ascontiguousarray(ic, np.int32)]
        self._keep = arrs
        lib().oracle_model_set_data(self.h, *[_p(a) for a in arrs])

    def set_embeddings(self, U, V):
        lib().oracle_model_set_embeddings(self.h, _p(f32(U)), _p(f32(V)))

    def embeddings(self):
        U = np.empty((self.n_users, self.dim), np.float32)
        V = np.empty((self.n_items, self.dim), np.float32)
        lib().oracle_model_get_embeddings(self.h, _p(U), _p(V))
        return U, V

    def initialize(self):
        lib().oracle_model_initialize(self.h)

    def train(self):
        return int(lib().oracle_model_train(self.h))

    def state(self):
        l = np.empty(self.n_users, np.float32)
        w = np.empty(self.n_users, np.float32)
        xi = ctypes.c_float()
        lib().oracle_model_get_state(self.h, _p(l), _p(w), ctypes.byref(xi))
        return l, w, float(xi.value)

    def fold_in(self, ptr, col):
        rp = np.ascontiguousarray(ptr, np.int64)
        cl = np.ascontiguousarray(col, np.int32)
        out = np.empty((len(rp) - 1, self.dim), np.float32)
        rc = lib().oracle_model_fold_in(self.h, len(rp) - 1, _p(rp), _p(cl), _p(out))
        return out, int(rc)

    def __del__(self):
        try:
            lib().oracle_model_destroy(self.h)
        except Exception:
            pass


def evaluate(Ueval, V, ex_ptr, ex_col, gt_ptr, gt_col, k_list=(5, 10, 20, 50, 100), nthreads=0):
    Ueval, V = f32(Ueval), f32(V)
    ks = np.asarray(k_list, np.int32)
    n = Ueval.shape[0]
    rec = np.zeros((n, len(ks)), np.float32)
    ndcg = np.zeros((n, len(ks)), np.float32)
    arrs = [np.ascontiguousarray(ex_ptr, np.int64), np.ascontiguousarray(ex_col, np.int32),
            np.ascontiguousarray(gt_ptr, np.int64), np.ascontiguousarray(gt_col, np.int32)]
    lib().oracle_evaluate(n, _p(Ueval), _p(V), V.shape[0], V.shape[1], _p(arrs[0]), _p(arrs[1]),
                          _p(arrs[2]), _p(arrs[3]), _p(ks), len(ks), _p(rec), _p(ndcg), nthreads)
    return rec, ndcg


def mean(x):
    """Eigen VectorXf::mean() restated (frecsys_oracle.c oracle_mean)."""
    x = f32(x)
    return float(lib().oracle_mean(_p(x), len(x)))


def safer2_xi_snr(loss, prev_xi, iterations, alpha, bandwidth, epan, sampling_ratio, seed):
    """SNR ComputeXi with a fresh generator seeded `seed`; returns xi."""
    loss = f32(loss)
    g = (ctypes.c_uint32 * 626)()
    lib().oracle_mt_seed(g, seed)
    return float(lib().oracle_safer2_xi_snr(_p(loss), len(loss), prev_xi, iterations, alpha,
                                            bandwidth, 1 if epan else 0, sampling_ratio, g))


def uniform_ints(seed, rng_range, count):
    """libstdc++ uniform_int_distribution<int>(0, rng_range-1) draws from mt19937(seed)."""
    g = (ctypes.c_uint32 * 626)()
    lib().oracle_mt_seed(g, seed)
    return [int(lib().oracle_uniform_int(g, rng_range)) for _ in range(count)]
