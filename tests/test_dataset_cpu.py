"""The C++ Dataset loader (include/frecsys/dataset.h; reference dataset.h:71-99)
parses in parallel chunks: the tuples must come out in
file order, identical for every thread count and to a plain Python parse,
with the header skipped, CRLF and blank lines tolerated."""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT


@pytest.fixture(scope="module")
def dataset_bin(tmp_path_factory):
    out = tmp_path_factory.mktemp("bin") / "dataset_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(PKG, "include"),
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "dataset_check.cc"), "-o", str(out)],
                   check=True, capture_output=True)
    return str(out)


def _python_parse(path):
    lines = open(path, "rb").read().split(b"\n")[1:]
    us, its = [], []
    for ln in lines:
        ln = ln.rstrip(b"\r")
        if not ln:
            continue
        a, _, b = ln.partition(b",")
        us.append(int(a))
        its.append(int(b) if b else 0)
    return us, its


def test_parallel_parse_is_file_order(tmp_path, dataset_bin):
    rng = np.random.default_rng(0)
    n = 150_000  # > 1 MB, so the loader splits it
    u = rng.integers(0, 5000, n)
    i = rng.integers(0, 3000, n)
    path = tmp_path / "d.csv"
    with open(path, "w", newline="") as f:
        f.write("uid,sid\n")
        for k in range(n):
            f.write(f"{u[k]},{i[k]}" + ("\r\n" if k % 7 == 0 else "\n"))
            if k % 1000 == 0:
                f.write("\n")
    outs = []
    for t in ("1", "3", "8", "16"):
        r = subprocess.run([dataset_bin, str(path)], capture_output=True, text=True, check=True,
                           env=dict(os.environ, FRECSYS_LOAD_THREADS=t))
        outs.append(r.stdout.split())
    assert all(o == outs[0] for o in outs), outs
    us, its = _python_parse(path)
    assert int(outs[0][0]) == len(us) == n
    assert int(outs[0][1]) == max(us) and int(outs[0][2]) == max(its)


def test_ml1m_fixture_counts(dataset_bin):
    path = os.path.join(ROOT, "tests", "golden", "ml-1m", "train.csv")
    r = subprocess.run([dataset_bin, path], capture_output=True, text=True, check=True)
    us, its = _python_parse(path)
    n, mu, mi, _ = r.stdout.split()
    assert (int(n), int(mu), int(mi)) == (len(us), max(us), max(its))
