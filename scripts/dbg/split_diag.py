"""Diagnostic: which rows differ between split / unsplit / repeated runs of
the wide weighted-V solve (tests/test_wide_split_gpu.py fixture)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("tests", "oracle", "safer2-recommender_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import frecsys_hip as fh
from test_parity_gpu import _ctx, _v_inputs, _weights


def long_items():
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
    perm = rng.permutation(len(users))  # file order: interleaved
    users, items = users[perm], items[perm]
    from frecsys_hip.data import _csr_from_pairs
    up, uc = _csr_from_pairs(users, items, n_users)
    ip, ic = _csr_from_pairs(items, users, n_items)
    return n_users, n_items, up, uc, ip, ic


def run(data, kind, split, quirk):
    os.environ["FRECSYS_SPLIT_ROWS"] = "1024" if split else "0"
    nu, ni, up, uc, ip, ic = data
    ctx, U, V = _ctx(512, nu, ni, up, uc, ip, ic, quirks=quirk)
    om = _weights(nu)
    nu_w, item_reg = _v_inputs(nu, ni, up, ip, ic, om)
    ctx.gramian(fh.SIDE_USER, weights=om)
    ctx.solve_side(fh.SIDE_ITEM, kind, 0.004, 0.004, alpha=0.3, entity_reg=item_reg,
                   other_weight=nu_w)
    return ctx.get_embeddings(fh.SIDE_ITEM)


d = long_items()
for quirk in (True, False):
    a = run(d, fh.KIND_WEIGHTED_V, True, quirk)
    b = run(d, fh.KIND_WEIGHTED_V, True, quirk)
    c = run(d, fh.KIND_WEIGHTED_V, False, quirk)
    e = run(d, fh.KIND_WEIGHTED_V, False, quirk)
    for name, x, y in (("split/split", a, b), ("unsplit/unsplit", c, e), ("split/unsplit", a, c)):
        rows = np.nonzero((x != y).any(axis=1))[0]
        print(f"quirk={quirk} {name}: {len(rows)} rows differ: {rows[:20]} "
              f"(elements {(x != y).sum()})", flush=True)
