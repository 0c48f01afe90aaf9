"""Host data path: CSV -> CSR in file order (dataset.h:71-99) and the
deterministic synthetic generator."""
import numpy as np

from frecsys_hip.data import SHAPES, Dataset, synthetic


def test_csv_header_skipped_and_file_order(tmp_path):
    p = tmp_path / "d.csv"
    p.write_text("uid,sid\n2,7\n0,3\n2,1\n1,7\n0,0\n2,5\n")
    d = Dataset.from_csv(str(p))
    assert d.num_tuples == 6 and d.max_user == 2 and d.max_item == 7
    up, uc = d.by_user()
    assert list(up) == [0, 2, 3, 6]
    assert list(uc[0:2]) == [3, 0]          # user 0 in file order
    assert list(uc[3:6]) == [7, 1, 5]       # user 2 in file order
    ip, ic = d.by_item()
    assert list(ic[ip[7]:ip[8]]) == [2, 1]  # item 7: users in file order
    assert ip[2] == ip[3]                    # idle item has an empty row


def test_ml1m_fixture_shape(ml1m):
    tr, vt, ve = ml1m
    assert tr.num_tuples == 388246 and tr.max_user == 4033 and tr.max_item == 3467
    up, uc = tr.by_user()
    h = np.diff(up)
    assert h.min() == 5 and h.max() == 1435
    ids, ep, ec = vt.compact_users()
    assert len(ids) == 1000 and ids[0] == 4034 and ep[-1] == 74132


def test_synthetic_deterministic_and_shaped():
    a = synthetic(SHAPES["tiny"], seed=3)
    b = synthetic(SHAPES["tiny"], seed=3)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    up, uc, ip, ic = a
    assert np.all(np.diff(up) >= SHAPES["tiny"].min_uc)
    assert np.all(np.diff(ip) >= 1)           # every item observed
    assert abs(up[-1] - SHAPES["tiny"].nnz) < 0.05 * SHAPES["tiny"].nnz
    # no repeated item inside a user
    for u in range(0, len(up) - 1, 97):
        row = uc[up[u]:up[u + 1]]
        assert len(np.unique(row)) == len(row)
    # both orientations hold the same pairs
    pairs_u = set(zip(np.repeat(np.arange(len(up) - 1), np.diff(up)).tolist(), uc.tolist()))
    pairs_i = set(zip(ic.tolist(), np.repeat(np.arange(len(ip) - 1), np.diff(ip)).tolist()))
    assert pairs_u == pairs_i
