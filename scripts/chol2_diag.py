"""A/B of the wide Cholesky kernels (FRECSYS_WIDE_CHOL2=1 vs 0): where do the
solutions differ (rows, columns, history lengths)."""
import os
import sys

import numpy as np

_R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(_R, "tests"), os.path.join(_R, "oracle"), os.path.join(_R, "safer2-recommender_amd")]
import test_wide_chol2_gpu as T  # noqa: E402
import frecsys_hip as fh  # noqa: E402


class Env:
    def setenv(self, k, v):
        os.environ[k] = v


def data():
    rng = np.random.default_rng(21)
    n_users, n_items = 12000, 40
    hs = [9000, 6150, 4097, 8192, 4100, 2500] + list(rng.integers(40, 600, n_items - 6))
    users, items = [], []
    for it, h in enumerate(hs):
        us = rng.choice(n_users, int(h), replace=False)
        users.append(us)
        items.append(np.full(len(us), it))
    users = np.concatenate(users).astype(np.int64)
    items = np.concatenate(items).astype(np.int64)
    perm = rng.permutation(len(users))
    users, items = users[perm], items[perm]
    from frecsys_hip.data import _csr_from_pairs
    up, uc = _csr_from_pairs(users, items, n_users)
    ip, ic = _csr_from_pairs(items, users, n_items)
    return n_users, n_items, up, uc, ip, ic, hs


d = data()
hs = d[-1]
d = d[:-1]
a = T._run(Env(), d, 512, fh.SIDE_ITEM, fh.KIND_IALS, True)
b = T._run(Env(), d, 512, fh.SIDE_ITEM, fh.KIND_IALS, False)
c = T._run(Env(), d, 512, fh.SIDE_ITEM, fh.KIND_IALS, False)
print("old vs old equal:", np.array_equal(b, c))
r, col = np.nonzero(a != b)
for i in sorted(set(r.tolist())):
    cs = col[r == i]
    print(f"item {i} h={hs[i]}: {len(cs)} cols differ, cols {cs[:12].tolist()} ... "
          f"max rel {np.max(np.abs(a[i]-b[i]))/np.max(np.abs(b[i])):.2e}")
