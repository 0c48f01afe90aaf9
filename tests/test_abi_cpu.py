"""C-ABI checks that need no GPU: the library loads, exports every symbol
include/frecsys_hip.h declares, its host-only helpers work, and compute entry
points fail loudly (no CPU fallback) when no device is visible."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import frecsys_hip as fh
from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "frecsys_hip.h")
MODEL_HEADER = os.path.join(ROOT, "include", "frecsys_model.h")


def _declared(header=HEADER):
    txt = open(header).read()
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


def test_model_library_exports_every_declared_symbol():
    names = _declared(MODEL_HEADER)
    assert set(names) == set(fh.MODEL_EXPORTS), set(names) ^ set(fh.MODEL_EXPORTS)
    lib = fh.load_model_library()
    out = subprocess.run(["nm", "-D", "--defined-only", fh.MODEL_LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (frecsys_\w+)", out))
    for name in names:
        assert name in exported, name
        assert getattr(lib, name) is not None


def test_model_config_defaults_are_run_model_flags():
    lib = fh.load_model_library()
    cfg = fh._ModelConfig()
    lib.frecsys_model_config_default(ctypes.byref(cfg))
    # run_model.cc:129-230
    assert (cfg.dim, cfg.block_size, cfg.xi_iterations, cfg.pd_iterations) == (8, 64, 5, 1)
    assert np.float32(cfg.l2_reg) == np.float32(0.002) and cfg.l2_reg_exp == 1.0
    assert np.float32(cfg.uobs_weight) == np.float32(0.1)
    assert np.float32(cfg.alpha) == np.float32(0.3) and cfg.bandwidth == 1.0
    assert cfg.print_train_stats == 1 and cfg.use_snr == 0 and cfg.seed == -1


def test_model_create_rejects_bad_arguments():
    u = np.array([0, 1, 1], np.int32)
    i = np.array([0, 0, 1], np.int32)
    with pytest.raises(fh.FrecsysError) as ei:
        fh.Model("als_unknown", u, i, dim=8)
    assert ei.value.code == fh.ERR_INVALID
    with pytest.raises(fh.FrecsysError) as ei:
        fh.Model("ials", u, i, dim=2048)
    assert ei.value.code == fh.ERR_UNSUPPORTED
    with pytest.raises(fh.FrecsysError) as ei:
        fh.Model("ials", np.array([0, -1], np.int32), np.array([0, 0], np.int32), dim=8)
    assert ei.value.code == fh.ERR_INVALID


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is visible here")
def test_model_without_device_fails_loudly():
    with pytest.raises(fh.FrecsysError) as ei:
        fh.Model("ials", np.array([0, 1], np.int32), np.array([1, 0], np.int32), dim=8)
    assert ei.value.code == fh.ERR_NO_DEVICE
