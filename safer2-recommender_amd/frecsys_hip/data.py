"""Interaction data as CSR for both orientations (host side, numpy).

`Dataset` mirrors frecsys::Dataset (dataset.h:71-99): a `uid,sid` CSV whose
header line is always skipped (dataset.h:80 -- the reference skips it inside
an assert, which its build keeps live), each entity's history in FILE ORDER
(dataset.h:87-88), max_user / max_item / num_tuples.  Instead of
unordered_map<int, vector<pair<int,int>>> it keeps CSR arrays:
  by_user: row_ptr[n_users+1] (int64), col[nnz] (int32 item ids)
  by_item: row_ptr[n_items+1] (int64), col[nnz] (int32 user ids)
The rating index of the reference's pairs is the file position; by_item rows
list users in file order (a stable sort of the user-major file by item).

`synthetic` builds the deterministic ML-20M / MSD-shaped inputs of
BASELINE.md section 4 directly in CSR (no CSV).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np


def _stable_order(rows: np.ndarray) -> np.ndarray:
    """np.argsort(rows, kind="stable") for non-negative ints: when row and
    position fit one int64 the (row, position) keys are distinct, so an
    unstable sort of them gives the same order, several times faster."""
    n = len(rows)
    pbits = max(int(n - 1).bit_length(), 1)
    if n == 0 or int(rows.max()).bit_length() + pbits > 63:
        return np.argsort(rows, kind="stable")
    key = (rows.astype(np.int64) << pbits) | np.arange(n, dtype=np.int64)
    key.sort()
    key &= (1 << pbits) - 1
    return key


def _csr_from_pairs(rows: np.ndarray, cols: np.ndarray, n_rows: int):
    order = _stable_order(rows)  # keeps file order inside a row
    counts = np.bincount(rows, minlength=n_rows)
    row_ptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.cumsum(counts, out=row_ptr[1:])
    return row_ptr, np.ascontiguousarray(cols[order], dtype=np.int32)


@dataclass
class Dataset:
    users: np.ndarray  # file-order user id per tuple
    items: np.ndarray  # file-order item id per tuple
    max_user: int
    max_item: int

    @classmethod
    def from_csv(cls, path: str) -> "Dataset":
        data = np.loadtxt(path, delimiter=",", skiprows=1, dtype=np.int64, ndmin=2)
        if data.size == 0:
            return cls(np.zeros(0, np.int64), np.zeros(0, np.int64), -1, -1)
        u, i = data[:, 0], data[:, 1]
        return cls(u, i, int(u.max()), int(i.max()))

    @property
    def num_tuples(self) -> int:
        return int(len(self.users))

    def by_user(self, n_users: int | None = None):
        n = self.max_user + 1 if n_users is None else n_users
        return _csr_from_pairs(self.users, self.items, n)

    def by_item(self, n_items: int | None = None):
        n = self.max_item + 1 if n_items is None else n_items
        return _csr_from_pairs(self.items, self.users, n)

    def compact_users(self):
        """Rows = distinct users (sorted by id) -> (user_ids, row_ptr, col).
        EvaluateDataset's user_to_ind compaction (ials.h:151-166)."""
        ids, inv = np.unique(self.users, return_inverse=True)
        rp, col = _csr_from_pairs(inv.astype(np.int64), self.items, len(ids))
        return ids, rp, col


@dataclass
class SynthShape:
    n_users: int
    n_items: int
    nnz: int
    min_uc: int = 5
    zipf_s: float = 1.0
    zipf_q: float = 10.0
    sigma: float = 1.0


SHAPES = {
    # BASELINE.md section 4 / SURVEY 8(d)
    "ml20m": SynthShape(116_677, 20_108, 8_540_000, min_uc=5),
    "msd": SynthShape(471_355, 41_140, 27_700_000, min_uc=20),
    "2m500k": SynthShape(2_000_000, 500_000, 100_000_000, min_uc=5),
    "tiny": SynthShape(3_000, 1_500, 90_000, min_uc=5),
}


def _searchsorted_uniform(cdf: np.ndarray, r: np.ndarray, log2_buckets: int = 24) -> np.ndarray:
    """np.searchsorted(cdf, r) (side 'left') for r in [0, 1), bucketed: with
    M = 2^k buckets the edges j/M are exact doubles and r*M floors exactly, so
    the answer for r in bucket j lies in [S[j], S[j+1]], S = searchsorted of
    the edges.  Buckets with S[j] == S[j+1] are answered by the table; the
    rest fall back to searchsorted.  Identical output, without the random
    accesses of one binary search per sample (2M x 500K: 74 s -> a few)."""
    M = 1 << log2_buckets
    S = np.searchsorted(cdf, np.arange(M + 1, dtype=np.float64) / M).astype(np.int64)
    j = (r * M).astype(np.int64)
    lo = S[j]
    amb = np.nonzero(S[j + 1] != lo)[0]
    if len(amb):
        lo[amb] = np.searchsorted(cdf, r[amb])
    return lo


def _first_per_user(users: np.ndarray, items: np.ndarray, nu: int) -> np.ndarray:
    """Positions of the first occurrence of each (user, item) pair, ascending
    -- np.unique(users * n_items + items, return_index=True)[1] sorted, for
    users in non-decreasing order: pairs never repeat across users, so the
    array is cut at user boundaries and the cuts are deduplicated on threads."""
    from concurrent.futures import ThreadPoolExecutor
    n = len(users)
    nch = max(1, min(16, n // 4_000_000))
    cuts = [0] + [int(np.searchsorted(users, users[min(n - 1, n * k // nch)], "left"))
                  for k in range(1, nch)] + [n]
    cuts = sorted(set(cuts))

    def one(k):
        a, b = cuts[k], cuts[k + 1]
        # (item, position) keys within the cut: item-major, position-minor
        u0 = users[a:b] - users[a]
        pbits = max(int(b - a - 1).bit_length(), 1)
        ibits = max(int(items[a:b].max()).bit_length(), 1)
        if int(u0[-1]).bit_length() + ibits + pbits <= 63:
            key = (((u0 << ibits) | items[a:b]) << pbits) | np.arange(b - a, dtype=np.int64)
            key.sort()
            pk = key >> pbits
            keep = np.ones(len(key), dtype=bool)
            keep[1:] = pk[1:] != pk[:-1]
            pos = key[keep] & ((1 << pbits) - 1)
        else:
            _, pos = np.unique(u0 * (1 << ibits) + items[a:b], return_index=True)
        pos.sort()
        return pos + a

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        parts = list(ex.map(one, range(len(cuts) - 1)))
    return np.concatenate(parts) if parts else np.zeros(0, np.int64)


def synthetic(shape: SynthShape, seed: int = 98765):
    """Deterministic synthetic interactions: Zipf-Mandelbrot
    item popularity 1/(rank+q)^s (s=1, q=10: the most popular item reaches
    ~55% of users, close to ML-20M's head; plain Zipf puts one item in >99%
    of histories) over a seeded permutation, lognormal user history lengths
    clipped at min_uc and rescaled to the target nnz, items per user drawn
    by popularity without repeats, every item given >= 1 interaction, rows in
    user-block order.  Returns (by_user_ptr, by_user_col, by_item_ptr,
    by_item_col)."""
    rng = np.random.default_rng(seed)
    nu, ni = shape.n_users, shape.n_items
    pop = 1.0 / (np.arange(1, ni + 1, dtype=np.float64) + shape.zipf_q) ** shape.zipf_s
    pop = pop[rng.permutation(ni)]
    cdf = np.cumsum(pop)
    cdf /= cdf[-1]
    lens = rng.lognormal(0.0, shape.sigma, nu)
    lens = lens / lens.sum() * shape.nnz
    lens = np.clip(np.round(lens), shape.min_uc, ni // 2).astype(np.int64)
    # oversample then drop repeats inside each user, trim to the target
    draw = (lens * 1.6 + 8).astype(np.int64)
    tot = int(draw.sum())
    users = np.repeat(np.arange(nu, dtype=np.int64), draw)
    items = _searchsorted_uniform(cdf, rng.random(tot))
    np.minimum(items, ni - 1, out=items)
    first = _first_per_user(users, items, nu)
    users, items = users[first], items[first]
    # rank inside the user (positions kept in draw order), keep < lens[u]
    starts = np.zeros(nu + 1, dtype=np.int64)
    np.cumsum(np.bincount(users, minlength=nu), out=starts[1:])
    rank = np.arange(len(users), dtype=np.int64) - starts[users]
    keep = rank < lens[users]
    users, items = users[keep], items[keep]
    # every item at least once: give each missing item to a random user
    seen = np.zeros(ni, dtype=bool)
    seen[items] = True
    missing = np.nonzero(~seen)[0]
    if len(missing):
        extra_u = rng.integers(0, nu, len(missing))
        users = np.concatenate([users, extra_u])
        items = np.concatenate([items, missing])
        order = np.argsort(users, kind="stable")
        users, items = users[order], items[order]
    up, uc = _csr_from_pairs(users, items, nu)
    ip, ic = _csr_from_pairs(items, users, ni)
    return up, uc, ip, ic
