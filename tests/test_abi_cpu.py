"""C-ABI checks that need no GPU: the library loads, exports every symbol
include/frecsys_hip.h declares, its host-only helpers work, and compute entry
points fail loudly (no CPU fallback) when no device is visible."""
import os
import re
import subprocess

import numpy as np
import pytest

import frecsys_hip as fh
from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "frecsys_hip.h")


def _declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(frecsys_[a-z_0-9]+)\s*\(", txt)))


def test_header_lists_expected_entry_points():
    names = _declared()
    assert set(names) == set(fh.EXPORTS), set(names) ^ set(fh.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = fh.load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", fh.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (frecsys_\w+)", out))
    for name in _declared():
        assert name in exported, name
        assert getattr(lib, name) is not None


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", fh.LIB_PATH],
                         capture_output=True, text=True)
    blob = open(fh.LIB_PATH, "rb").read()
    assert b"gfx950" in blob, "no gfx950 code object embedded"
    del out


def test_padded_dim():
    assert [fh.padded_dim(d) for d in (1, 8, 9, 16, 17, 32, 33, 200, 256)] == \
        [8, 8, 16, 16, 32, 32, 64, 224, 256]
    # wide dims (csrc/wide.hip): 512 and 1024 only
    assert [fh.padded_dim(d) for d in (257, 300, 512, 513, 1000, 1024)] == \
        [512, 512, 512, 1024, 1024, 1024]
    assert fh.padded_dim(1025) == 0


def test_partition_nnz_balanced():
    rng = np.random.default_rng(0)
    h = rng.integers(0, 50, 1001)
    h[10] = 5000  # one heavy row
    rp = np.concatenate([[0], np.cumsum(h)]).astype(np.int64)
    for P in (1, 2, 3, 4, 8):
        b = fh.partition(rp, P)
        assert b[0] == 0 and b[-1] == 1001 and np.all(np.diff(b) >= 0)
        nnz = rp[b[1:]] - rp[b[:-1]]
        assert nnz.sum() == rp[-1]
        # a contiguous split can only miss the even share by < one row
        assert np.all(nnz <= rp[-1] / P + h.max())


def test_partition_deterministic_and_empty_rows():
    rp = np.zeros(11, np.int64)  # ten empty rows
    b = fh.partition(rp, 4)
    assert b[0] == 0 and b[-1] == 10
    assert np.array_equal(b, fh.partition(rp, 4))


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is visible here")
def test_context_without_device_fails_loudly():
    with pytest.raises(fh.FrecsysError) as ei:
        fh.Context(16, 10, 10)
    assert ei.value.code in (fh.ERR_NO_DEVICE, fh.ERR_HIP)
