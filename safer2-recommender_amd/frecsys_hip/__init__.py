"""frecsys_hip -- ctypes binding of libfrecsys_hip.so (include/frecsys_hip.h).

Thin host-side plumbing over the C-ABI for the Python harnesses (tests,
bench.py, __graft_entry__).  The product's own host layer is C++
(include/frecsys/*.h, tools/run_model.cc); this module adds nothing to the
compute path: every call goes straight to the HIP library, and importing it
without the built library raises (there is no CPU fallback).

Sides / kinds mirror the C-ABI (`SIDE_USER`, `KIND_IALS`, ...).  Arrays are
numpy: CSR row_ptr int64, col int32, embeddings float32 [rows, dim].
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import numpy as np

SIDE_USER, SIDE_ITEM, SIDE_EVAL = 0, 1, 2
KIND_IALS, KIND_WEIGHTED_U, KIND_WEIGHTED_V, KIND_CVAR_GRAD_U, KIND_CVAR_GRAD_V = range(5)

OK = 0
ERR_INVALID, ERR_HIP, ERR_RCCL, ERR_NOT_SPD, ERR_NAN, ERR_UNSUPPORTED, ERR_NO_DEVICE = range(1, 8)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfrecsys_hip.so")
MODEL_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfrecsys_model.so")

# Every symbol include/frecsys_hip.h declares (checked by the CPU tests).
EXPORTS = (
    "frecsys_device_count", "frecsys_ctx_create", "frecsys_ctx_destroy",
    "frecsys_last_error", "frecsys_last_error_entity", "frecsys_padded_dim",
    "frecsys_partition", "frecsys_comm_unique_id", "frecsys_comm_init",
    "frecsys_shard_range", "frecsys_load_csr", "frecsys_set_embeddings",
    "frecsys_get_embeddings", "frecsys_init_embeddings", "frecsys_snapshot",
    "frecsys_gramian", "frecsys_set_gramian", "frecsys_solve_side", "frecsys_user_loss",
    "frecsys_synchronize", "frecsys_timing", "frecsys_timing_reset", "frecsys_debug_basis",
    "frecsys_eval_topk", "frecsys_train_stats", "frecsys_pp_set_rating_index",
    "frecsys_pp_predict", "frecsys_pp_step", "frecsys_debug_diag_factor",
    "frecsys_history_space_max_h", "frecsys_history_space_max_h_side", "frecsys_comm_world", "frecsys_gram_groups",
    "frecsys_get_gram_groups", "frecsys_set_gram_groups", "frecsys_get_gramian",
    "frecsys_gram_plan", "frecsys_work", "frecsys_snapshot_residual", "frecsys_counter",
    "frecsys_pp_sync", "frecsys_release_workspaces", "frecsys_pp_get_predictions",
    "frecsys_set_transport",
)

# Every symbol include/frecsys_model.h declares.
MODEL_EXPORTS = (
    "frecsys_model_config_default", "frecsys_model_create", "frecsys_model_initialize",
    "frecsys_model_train", "frecsys_model_context", "frecsys_model_mean_weight",
    "frecsys_model_destroy", "frecsys_model_last_error", "frecsys_model_dual_state",
)


class FrecsysError(RuntimeError):
    def __init__(self, code: int, msg: str, entity: int = -1):
        super().__init__(f"frecsys error {code}: {msg}")
        self.code = code
        self.entity = entity


class _Config(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("device", ctypes.c_int32),
                ("parity_quirks", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("n_users", ctypes.c_int64), ("n_items", ctypes.c_int64)]


# frecsys_transport (include/frecsys_hip.h)
_ROWS_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32,
                            ctypes.POINTER(ctypes.c_float), ctypes.c_int64, ctypes.c_int64,
                            ctypes.c_int64, ctypes.c_int64)
_MIN_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64))


class _Transport(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("allgather_rows", _ROWS_FN),
                ("allreduce_min_u64", _MIN_FN)]


class _SolveParams(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("reg", ctypes.c_float),
                ("reg_exp", ctypes.c_float), ("unobserved_weight", ctypes.c_float),
                ("alpha", ctypes.c_float), ("stepsize", ctypes.c_float),
                ("from_snapshot", ctypes.c_int32), ("lambda_is_reg", ctypes.c_int32),
                ("entity_weight", ctypes.c_void_p), ("entity_reg", ctypes.c_void_p),
                ("other_weight", ctypes.c_void_p)]


class _ModelConfig(ctypes.Structure):
    _fields_ = [("model_name", ctypes.c_char_p), ("dim", ctypes.c_int32),
                ("l2_reg", ctypes.c_float), ("l2_reg_exp", ctypes.c_float),
                ("uobs_weight", ctypes.c_float), ("stdev", ctypes.c_float),
                ("alpha", ctypes.c_float), ("bandwidth", ctypes.c_float),
                ("stepsize", ctypes.c_float), ("sampling_ratio", ctypes.c_float),
                ("block_size", ctypes.c_int32), ("xi_iterations", ctypes.c_int32),
                ("pd_iterations", ctypes.c_int32), ("use_epanechnikov", ctypes.c_int32),
                ("use_snr", ctypes.c_int32), ("print_train_stats", ctypes.c_int32),
                ("print_residual_stats", ctypes.c_int32), ("print_var_stats", ctypes.c_int32),
                ("seed", ctypes.c_int64), ("device", ctypes.c_int32),
                ("parity_quirks", ctypes.c_int32), ("world", ctypes.c_int32),
                ("rank", ctypes.c_int32), ("comm_id", ctypes.c_void_p)]


_lib = None
_model_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libfrecsys_hip.so; raises if it was not built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FrecsysError(ERR_INVALID, f"{path} missing: run __graft_entry__.build() / make")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    P, I32, I64, F = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float
    sig = {
        "frecsys_device_count": (ctypes.c_int, [P]),
        "frecsys_ctx_create": (ctypes.c_int, [P, P]),
        "frecsys_ctx_destroy": (None, [P]),
        "frecsys_last_error": (ctypes.c_char_p, [P]),
        "frecsys_last_error_entity": (I64, [P]),
        "frecsys_padded_dim": (I32, [I32]),
        "frecsys_partition": (ctypes.c_int, [I64, P, I32, P]),
        "frecsys_comm_unique_id": (ctypes.c_int, [P]),
        "frecsys_comm_init": (ctypes.c_int, [P, I32, I32, P]),
        "frecsys_shard_range": (ctypes.c_int, [P, I32, P, P]),
        "frecsys_load_csr": (ctypes.c_int, [P, I32, I64, P, P]),
        "frecsys_set_embeddings": (ctypes.c_int, [P, I32, P, I64]),
        "frecsys_get_embeddings": (ctypes.c_int, [P, I32, P, I64]),
        "frecsys_init_embeddings": (ctypes.c_int, [P, ctypes.c_uint32, F]),
        "frecsys_snapshot": (ctypes.c_int, [P, I32]),
        "frecsys_gramian": (ctypes.c_int, [P, I32, P, I32, P]),
        "frecsys_set_gramian": (ctypes.c_int, [P, I32, P, I64]),
        "frecsys_solve_side": (ctypes.c_int, [P, I32, P]),
        "frecsys_user_loss": (ctypes.c_int, [P, I32, F, I32, P]),
        "frecsys_synchronize": (ctypes.c_int, [P]),
        "frecsys_timing": (ctypes.c_int, [P, ctypes.c_char_p, P, P]),
        "frecsys_timing_reset": (ctypes.c_int, [P]),
        "frecsys_history_space_max_h": (I32, [P]),
        "frecsys_history_space_max_h_side": (I32, [P, I32]),
        "frecsys_comm_world": (ctypes.c_int, [P, P, P, P]),
        "frecsys_gram_groups": (ctypes.c_int, [P, I32, P, P, P, P]),
        "frecsys_get_gram_groups": (ctypes.c_int, [P, I32, P]),
        "frecsys_set_gram_groups": (ctypes.c_int, [P, I32, P]),
        "frecsys_get_gramian": (ctypes.c_int, [P, I32, P, I64]),
        "frecsys_gram_plan": (ctypes.c_int, [I32, I64, I32, I32, P, P, P, P, P]),
        "frecsys_work": (ctypes.c_int, [P, ctypes.c_char_p, P, P, P, P]),
        "frecsys_debug_basis": (ctypes.c_int, [P, I32, P, P, P]),
        "frecsys_debug_diag_factor": (ctypes.c_int, [P, I32, I32, P, P, P]),
        "frecsys_eval_topk": (ctypes.c_int, [P, I32, P]),
        "frecsys_train_stats": (ctypes.c_int, [P, P, P, P, P]),
        "frecsys_pp_set_rating_index": (ctypes.c_int, [P, I32, P]),
        "frecsys_pp_predict": (ctypes.c_int, [P, I32]),
        "frecsys_pp_step": (ctypes.c_int, [P, I32, I32, I32, P, P]),
        "frecsys_snapshot_residual": (ctypes.c_int, [P, I32, P]),
        "frecsys_counter": (ctypes.c_int, [P, ctypes.c_char_p, P]),
        "frecsys_pp_sync": (ctypes.c_int, [P, I32]),
        "frecsys_release_workspaces": (ctypes.c_int, [P]),
        "frecsys_pp_get_predictions": (ctypes.c_int, [P, I32, P]),
        "frecsys_set_transport": (ctypes.c_int, [P, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def load_model_library(path: str = MODEL_LIB_PATH) -> ctypes.CDLL:
    """Load libfrecsys_model.so (the C++ model classes behind a C-ABI)."""
    global _model_lib
    if _model_lib is not None:
        return _model_lib
    load_library()
    if not os.path.exists(path):
        raise FrecsysError(ERR_INVALID, f"{path} missing: run __graft_entry__.build() / make")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    sig = {
        "frecsys_model_config_default": (None, [P]),
        "frecsys_model_create": (ctypes.c_int, [P, P, P, I64, P]),
        "frecsys_model_initialize": (ctypes.c_int, [P]),
        "frecsys_model_train": (ctypes.c_int, [P, I32]),
        "frecsys_model_context": (P, [P]),
        "frecsys_model_mean_weight": (ctypes.c_float, [P]),
        "frecsys_model_destroy": (None, [P]),
        "frecsys_model_last_error": (ctypes.c_char_p, []),
        "frecsys_model_dual_state": (ctypes.c_int, [P, P, P, P, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _model_lib = lib
    return lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def device_count() -> int:
    lib = load_library()
    n = ctypes.c_int32(0)
    lib.frecsys_device_count(ctypes.byref(n))
    return int(n.value)


def padded_dim(dim: int) -> int:
    return int(load_library().frecsys_padded_dim(dim))


def partition(row_ptr: np.ndarray, nparts: int) -> np.ndarray:
    """nnz-balanced contiguous split (host-only; no GPU needed)."""
    lib = load_library()
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    out = np.zeros(nparts + 1, dtype=np.int64)
    rc = lib.frecsys_partition(len(rp) - 1, _ptr(rp), nparts, _ptr(out))
    if rc:
        raise FrecsysError(rc, lib.frecsys_last_error(None).decode())
    return out


def gram_plan(dim: int, n_rows: int, world: int = 1, rank: int = 0):
    """Host-only Gramian plan: (rows_per_leaf, n_leaves, n_groups, own_lo,
    own_hi) -- frecsys_gram_plan."""
    lib = load_library()
    rpl, nl = ctypes.c_int64(), ctypes.c_int64()
    ng, lo, hi = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    rc = lib.frecsys_gram_plan(dim, n_rows, world, rank, ctypes.byref(rpl), ctypes.byref(nl),
                               ctypes.byref(ng), ctypes.byref(lo), ctypes.byref(hi))
    if rc:
        raise FrecsysError(rc, lib.frecsys_last_error(None).decode())
    return int(rpl.value), int(nl.value), int(ng.value), int(lo.value), int(hi.value)


def unique_id() -> bytes:
    lib = load_library()
    buf = (ctypes.c_uint8 * 128)()
    rc = lib.frecsys_comm_unique_id(buf)
    if rc:
        raise FrecsysError(rc, lib.frecsys_last_error(None).decode())
    return bytes(buf)


class Context:
    """One device context (one GPU).  See include/frecsys_hip.h."""

    def __init__(self, dim: int, n_users: int, n_items: int, device: int = -1,
                 parity_quirks: bool = True, _borrowed=None):
        self.lib = load_library()
        self.owned = _borrowed is None
        if _borrowed is not None:  # a model's context (frecsys_model_context)
            self.h = ctypes.c_void_p(_borrowed)
            self.dim = dim
            self.n = {SIDE_USER: n_users, SIDE_ITEM: n_items, SIDE_EVAL: 0}
            return
        cfg = _Config(dim, device, 1 if parity_quirks else 0, 0, n_users, n_items)
        h = ctypes.c_void_p()
        rc = self.lib.frecsys_ctx_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc:
            raise FrecsysError(rc, self.lib.frecsys_last_error(None).decode())
        self.h = h
        self.dim = dim
        self.n = {SIDE_USER: n_users, SIDE_ITEM: n_items, SIDE_EVAL: 0}

    # -- helpers --
    def _check(self, rc: int):
        if rc:
            ent = int(self.lib.frecsys_last_error_entity(self.h))
            raise FrecsysError(rc, self.lib.frecsys_last_error(self.h).decode(), ent)

    def close(self):
        if getattr(self, "h", None):
            if self.owned:
                self.lib.frecsys_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- comm --
    def comm_init(self, world: int, rank: int, uid: Optional[bytes]):
        """uid None: external exchange (no RCCL; the caller moves partial
        Gramians and shard rows between ranks)."""
        buf = None if uid is None else (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        self._check(self.lib.frecsys_comm_init(self.h, world, rank, buf))

    def comm_world(self) -> Tuple[int, int, int]:
        """(world, rank, ranks of the RCCL communicator -- 0 without one)."""
        w, r, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        self._check(self.lib.frecsys_comm_world(self.h, ctypes.byref(w), ctypes.byref(r),
                                                ctypes.byref(n)))
        return int(w.value), int(r.value), int(n.value)

    def gram_groups(self, side: int) -> Tuple[int, int, int, int]:
        """(n_groups, own_lo, own_hi, floats_per_group) of side's Gramian plan."""
        ng, lo, hi, fl = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        self._check(self.lib.frecsys_gram_groups(self.h, side, ctypes.byref(ng), ctypes.byref(lo),
                                                 ctypes.byref(hi), ctypes.byref(fl)))
        return int(ng.value), int(lo.value), int(hi.value), int(fl.value)

    def get_gram_groups(self, side: int) -> np.ndarray:
        ng, _, _, fl = self.gram_groups(side)
        out = np.zeros((ng, fl), dtype=np.float32)
        self._check(self.lib.frecsys_get_gram_groups(self.h, side, _ptr(out)))
        return out

    def set_gram_groups(self, side: int, slabs: np.ndarray):
        ng, _, _, fl = self.gram_groups(side)
        a = np.ascontiguousarray(slabs, dtype=np.float32)
        assert a.shape == (ng, fl), (a.shape, ng, fl)
        self._check(self.lib.frecsys_set_gram_groups(self.h, side, _ptr(a)))

    def shard_range(self, side: int) -> Tuple[int, int]:
        lo, hi = ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.frecsys_shard_range(self.h, side, ctypes.byref(lo), ctypes.byref(hi)))
        return int(lo.value), int(hi.value)

    # -- data --
    def load_csr(self, side: int, row_ptr: np.ndarray, col: np.ndarray):
        rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
        cl = np.ascontiguousarray(col, dtype=np.int32)
        self._check(self.lib.frecsys_load_csr(self.h, side, len(rp) - 1, _ptr(rp), _ptr(cl)))
        if side == SIDE_EVAL:
            self.n[SIDE_EVAL] = len(rp) - 1

    def set_embeddings(self, side: int, emb: np.ndarray):
        e = np.ascontiguousarray(emb, dtype=np.float32)
        assert e.shape == (self.n[side], self.dim), (e.shape, self.n[side], self.dim)
        self._check(self.lib.frecsys_set_embeddings(self.h, side, _ptr(e), self.dim))

    def get_embeddings(self, side: int) -> np.ndarray:
        out = np.empty((self.n[side], self.dim), dtype=np.float32)
        self._check(self.lib.frecsys_get_embeddings(self.h, side, _ptr(out), self.dim))
        return out

    def init_embeddings(self, seed: int, stdev: float):
        self._check(self.lib.frecsys_init_embeddings(self.h, seed, stdev))

    def snapshot(self, side: int):
        self._check(self.lib.frecsys_snapshot(self.h, side))

    def snapshot_residual(self, side: int) -> float:
        """sum over rows of ||X_r - snapshot_r||^2 (double, on the device)."""
        sq = ctypes.c_double()
        self._check(self.lib.frecsys_snapshot_residual(self.h, side, ctypes.byref(sq)))
        return float(sq.value)

    def counter(self, what: str) -> int:
        """Cumulative event counter: "hspace_reruns", "tagged_timeouts" or
        "ws_shrinks"."""
        v = ctypes.c_int64()
        self._check(self.lib.frecsys_counter(self.h, what.encode(), ctypes.byref(v)))
        return int(v.value)

    def release_workspaces(self) -> None:
        """Free the wide-dim workspaces (resized at the next solve)."""
        self._check(self.lib.frecsys_release_workspaces(self.h))

    # -- compute --
    def gramian(self, side: int, weights: Optional[np.ndarray] = None,
                from_snapshot: bool = False, fetch: bool = True) -> Optional[np.ndarray]:
        w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float32)
        out = np.empty((self.dim, self.dim), dtype=np.float32) if fetch else None
        self._check(self.lib.frecsys_gramian(self.h, side, _ptr(w), 1 if from_snapshot else 0,
                                             _ptr(out)))
        return out

    def get_gramian(self, side: int) -> np.ndarray:
        """G[side] as the context holds it (no recomputation)."""
        out = np.empty((self.dim, self.dim), dtype=np.float32)
        self._check(self.lib.frecsys_get_gramian(self.h, side, _ptr(out), self.dim))
        return out

    def set_gramian(self, side: int, G: np.ndarray):
        g = np.ascontiguousarray(G, dtype=np.float32)
        assert g.shape == (self.dim, self.dim), g.shape
        self._check(self.lib.frecsys_set_gramian(self.h, side, _ptr(g), self.dim))

    def solve_side(self, side: int, kind: int, reg: float, unobserved_weight: float,
                   reg_exp: float = 1.0, alpha: float = 0.0, stepsize: float = 0.0,
                   from_snapshot: bool = False, entity_weight=None, entity_reg=None,
                   other_weight=None):
        ew = None if entity_weight is None else np.ascontiguousarray(entity_weight, np.float32)
        er = None if entity_reg is None else np.ascontiguousarray(entity_reg, np.float32)
        ow = None if other_weight is None else np.ascontiguousarray(other_weight, np.float32)
        p = _SolveParams(kind, reg, reg_exp, unobserved_weight, alpha, stepsize,
                         1 if from_snapshot else 0, 0,
                         None if ew is None else ew.ctypes.data,
                         None if er is None else er.ctypes.data,
                         None if ow is None else ow.ctypes.data)
        self._check(self.lib.frecsys_solve_side(self.h, side, ctypes.byref(p)))

    def user_loss(self, side: int, beta: float, half: bool, fetch: bool = True):
        out = np.zeros(self.n[side], dtype=np.float32) if fetch else None
        self._check(self.lib.frecsys_user_loss(self.h, side, beta, 1 if half else 0, _ptr(out)))
        return out

    def synchronize(self):
        self._check(self.lib.frecsys_synchronize(self.h))

    def timing(self, what: str) -> Tuple[float, int]:
        ms, n = ctypes.c_double(), ctypes.c_int64()
        self._check(self.lib.frecsys_timing(self.h, what.encode(), ctypes.byref(ms),
                                            ctypes.byref(n)))
        return float(ms.value), int(n.value)

    def work(self, what: str):
        """(flops, bytes, entities, launches) of timer key `what`: the
        algorithmic work the library launched (frecsys_work)."""
        f, b = ctypes.c_double(), ctypes.c_double()
        e, n = ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.frecsys_work(self.h, what.encode(), ctypes.byref(f), ctypes.byref(b),
                                          ctypes.byref(e), ctypes.byref(n)))
        return float(f.value), float(b.value), int(e.value), int(n.value)

    def history_space_max_h(self, side=None) -> int:
        if side is None:
            return int(self.lib.frecsys_history_space_max_h(self.h))
        return int(self.lib.frecsys_history_space_max_h_side(self.h, side))

    def timing_reset(self):
        self._check(self.lib.frecsys_timing_reset(self.h))

    def eval_topk(self, k: int):
        """[EVAL rows, k] int32: best k items per fold-in row, history excluded,
        score descending, ties by item id."""
        out = np.zeros((self.n[SIDE_EVAL], k), dtype=np.int32)
        self._check(self.lib.frecsys_eval_topk(self.h, k, _ptr(out)))
        return out

    def pp_set_rating_index(self, side: int, rix: np.ndarray):
        r = np.ascontiguousarray(rix, dtype=np.int32)
        self._check(self.lib.frecsys_pp_set_rating_index(self.h, side, _ptr(r)))

    def pp_sync(self, side: int):
        """External-exchange completion of a sharded pp_step (frecsys_pp_sync)."""
        self._check(self.lib.frecsys_pp_sync(self.h, side))

    def pp_predict(self, side: int):
        self._check(self.lib.frecsys_pp_predict(self.h, side))

    def pp_predictions(self, side: int, nnz: int) -> np.ndarray:
        """The prediction vector (frecsys_pp_get_predictions), nnz floats."""
        out = np.empty(max(nnz, 1), np.float32)
        self._check(self.lib.frecsys_pp_get_predictions(self.h, side, _ptr(out)))
        return out[:nnz]

    def set_transport(self, allgather_rows, allreduce_min_u64):
        """Exchange callbacks of external-exchange mode (frecsys_set_transport):
        allgather_rows(side, rows, lo, hi) fills every rank's rows of the
        (n_rows, ld) float32 array in place (rows [lo, hi) are this rank's);
        allreduce_min_u64(value) -> the minimum over ranks.  None clears."""
        if allgather_rows is None:
            self._transport = None
            self._check(self.lib.frecsys_set_transport(self.h, None))
            return

        def rows_cb(user, side, ptr, n, ld, lo, hi):
            try:
                arr = np.ctypeslib.as_array(ptr, shape=(max(n, 1) * ld,))[:n * ld].reshape(n, ld)
                allgather_rows(int(side), arr, int(lo), int(hi))
                return 0
            except Exception:  # noqa: BLE001 -- reported to the library as a failed exchange
                import traceback
                traceback.print_exc()
                return 1

        def min_cb(user, vp):
            try:
                vp[0] = int(allreduce_min_u64(int(vp[0])))
                return 0
            except Exception:  # noqa: BLE001
                import traceback
                traceback.print_exc()
                return 1

        t = _Transport(None, _ROWS_FN(rows_cb), _MIN_FN(min_cb))
        self._transport = t  # the callbacks live as long as the context uses them
        self._check(self.lib.frecsys_set_transport(self.h, ctypes.byref(t)))

    def pp_step(self, side: int, start: int, end: int, reg: float, w: float,
                reg_exp: float = 1.0, kind: int = 0, alpha: float = 0.0, entity_weight=None,
                entity_reg=None, other_weight=None) -> float:
        ew = None if entity_weight is None else np.ascontiguousarray(entity_weight, np.float32)
        er = None if entity_reg is None else np.ascontiguousarray(entity_reg, np.float32)
        ow = None if other_weight is None else np.ascontiguousarray(other_weight, np.float32)
        p = _SolveParams(kind, reg, reg_exp, w, alpha, 0.0, 0, 0,
                         None if ew is None else ew.ctypes.data,
                         None if er is None else er.ctypes.data,
                         None if ow is None else ow.ctypes.data)
        res = ctypes.c_double(0.0)
        self._check(self.lib.frecsys_pp_step(self.h, side, start, end, ctypes.byref(p),
                                             ctypes.byref(res)))
        return res.value

    def train_stats(self):
        """(observed, unobserved, ||U_r||^2, ||V_r||^2): ComputeLosses' parts."""
        obs = ctypes.c_double(0.0)
        unobs = ctypes.c_double(0.0)
        un = np.zeros(self.n[SIDE_USER], dtype=np.float32)
        vn = np.zeros(self.n[SIDE_ITEM], dtype=np.float32)
        self._check(self.lib.frecsys_train_stats(self.h, ctypes.byref(obs), ctypes.byref(unobs),
                                                 _ptr(un), _ptr(vn)))
        return obs.value, unobs.value, un, vn

    def debug_diag_factor(self, tiles: np.ndarray, blocked: bool):
        """L^-1 of each 32x32 SPD tile (diagnostic): (linv [n,32,32], ok [n])."""
        a = np.ascontiguousarray(tiles, dtype=np.float32).reshape(-1, 32, 32)
        out = np.zeros_like(a)
        ok = np.zeros(len(a), dtype=np.int32)
        self._check(self.lib.frecsys_debug_diag_factor(self.h, 1 if blocked else 0, len(a),
                                                       _ptr(a), _ptr(out), _ptr(ok)))
        return out, ok

    def debug_basis(self, side: int):
        """(Q, diag, sub) with G[side] = Q T Q^T (diagnostic, Dp >= 64)."""
        Dp = padded_dim(self.dim)
        q = np.zeros((Dp, Dp), dtype=np.float32)
        dg = np.zeros(Dp, dtype=np.float32)
        sb = np.zeros(Dp, dtype=np.float32)
        self._check(self.lib.frecsys_debug_basis(self.h, side, _ptr(q), _ptr(dg), _ptr(sb)))
        return q, dg, sb


class Model:
    """One model of include/frecsys_model.h: the run_model factory over the
    C++ classes.  `users`, `items`: the training tuples in file order;
    keyword arguments are the run_model flags (frecsys_model_config)."""

    def __init__(self, model_name: str, users: np.ndarray, items: np.ndarray, **flags):
        self.lib = load_model_library()
        cfg = _ModelConfig()
        self.lib.frecsys_model_config_default(ctypes.byref(cfg))
        self._name = model_name.encode()
        cfg.model_name = self._name
        self._cid = None
        for k, v in flags.items():
            if k == "comm_id":
                if v is not None:
                    self._cid = (ctypes.c_uint8 * 128).from_buffer_copy(v)
                    cfg.comm_id = ctypes.cast(self._cid, ctypes.c_void_p)
                continue
            if not hasattr(cfg, k):
                raise TypeError(f"unknown model flag {k}")
            setattr(cfg, k, int(v) if isinstance(v, bool) else v)
        u = np.ascontiguousarray(users, dtype=np.int32)
        it = np.ascontiguousarray(items, dtype=np.int32)
        assert u.shape == it.shape
        h = ctypes.c_void_p()
        rc = self.lib.frecsys_model_create(ctypes.byref(cfg), _ptr(u), _ptr(it), len(u),
                                           ctypes.byref(h))
        if rc:
            raise FrecsysError(rc, self.lib.frecsys_model_last_error().decode())
        self.h = h
        self.dim = cfg.dim
        self.n_users = int(u.max()) + 1
        self.n_items = int(it.max()) + 1

    def initialize(self):
        rc = self.lib.frecsys_model_initialize(self.h)
        if rc:
            raise FrecsysError(rc, self.lib.frecsys_model_last_error().decode())

    def train(self, epochs: int = 1):
        rc = self.lib.frecsys_model_train(self.h, epochs)
        if rc:
            raise FrecsysError(rc, self.lib.frecsys_model_last_error().decode())

    def context(self) -> Context:
        """The model's device context (borrowed: closing it is a no-op)."""
        ctx = Context(self.dim, self.n_users, self.n_items,
                      _borrowed=self.lib.frecsys_model_context(self.h))
        ctx._owner = self  # the native context lives as long as the model
        return ctx

    def dual_state(self):
        """(omega [n_users], user losses [n_users], item_reg [n_items], xi) of
        ERM-MF / CVaR-MF / SAFER2 (frecsys_model_dual_state)."""
        w = np.zeros(self.n_users, dtype=np.float32)
        l = np.zeros(self.n_users, dtype=np.float32)
        r = np.zeros(self.n_items, dtype=np.float32)
        xi = ctypes.c_float(0.0)
        rc = self.lib.frecsys_model_dual_state(self.h, _ptr(w), _ptr(l), _ptr(r), ctypes.byref(xi))
        if rc:
            raise FrecsysError(rc, self.lib.frecsys_model_last_error().decode())
        return w, l, r, float(xi.value)

    def mean_weight(self) -> float:
        return float(self.lib.frecsys_model_mean_weight(self.h))

    def close(self):
        if getattr(self, "h", None):
            self.lib.frecsys_model_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
